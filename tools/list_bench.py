#!/usr/bin/env python3
"""Re-bind cost of list values at real sizes (the list path had no number).

Lasp re-runs a combinator on every input change and binds its whole new output into
the old one (lasp_process.erl:61-95 -> lasp_core.erl:291-312 -> lasp_orset.erl:128-134):
`Value0 =:= Value`, orddict:merge run as written, is_inflation by keyfind.  Rows:
  * config 5's intersection output (1 pair of 100k-element OR-Sets, 50 % overlap, T = 3):
    50k entries {X, Cx ++ Cy}; the re-run after R changed (10 % of its elements get a
    token, 5 % a removal);
  * a product output 256 x 256 = 65,536 entries {{X, Y}, [[Tx, Ty]...]} (9 tokens each);
  * a batch of 1024 small intersection outputs (200 entries each): the batched path;
  * the Store: one update of R -> the intersection re-runs and re-binds (end to end).
Each row: microseconds per laspj_list_merge / list_equal / list_inflation(strict) call
(entry point, size pass + write pass, synchronous) and the bytes of the two operands.
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import _lib, engine  # noqa: E402

PAIR, COMP, REM = _lib.LIST_PAIR, _lib.LIST_COMPOUND, _lib.LIST_REMOVED


def identity_order(ctx, nkeys):
    kr = ctx.buffer(4 * nkeys)
    kr.upload(np.arange(nkeys, dtype=np.uint32))
    gr = ctx.buffer(4 * 64 * nkeys)
    gr.upload(np.arange(64 * nkeys, dtype=np.uint32))
    o = _lib.ListOrder()
    o.krank, o.nkeys, o.grank, o.ntokens = kr.h.value, nkeys, gr.h.value, 64 * nkeys
    return o, (kr, gr)


def cells(rng, n, T=3):
    p = rng.integers(1, 1 << T, n).astype(np.uint64)
    r = p & rng.integers(0, 1 << T, n).astype(np.uint64) & rng.integers(0, 2, n).astype(np.uint64) * 7
    return p, r


def run(e, p, r):
    return [(64 * int(e) + k) | (REM if (int(r) >> k) & 1 else 0) for k in range(8) if (int(p) >> k) & 1]


def intersection_list(keys, pl, rl, pr, rr):
    """{X, Cx ++ Cy} entries (lasp_core.erl:546-589) for common keys."""
    toks, toff = [], [0]
    for i, e in enumerate(keys):
        toks.extend(run(e, pl[i], rl[i]))
        toks.extend(run(e, pr[i], rr[i]))
        toff.append(len(toks))
    return (np.asarray(keys, np.uint64), np.asarray(toff, np.uint32),
            np.asarray(toks, np.uint64))


def product_list(nx, ny, px, rx, py, ry):
    """{{X, Y}, orset_causal_product(Cx, Cy)} X-major (lasp_core.erl:499-533,
    lasp_lattice.erl:303-308: both runs reversed, [Tx, Ty], Dx orelse Dy)."""
    keys, toff, toks = [], [0], []
    for x in range(nx):
        tx = run(x, px[x], rx[x])
        for y in range(ny):
            ty = run(nx + y, py[y], ry[y])
            keys.append(PAIR | (x << 31) | (nx + y))
            for a in reversed(tx):
                for b in reversed(ty):
                    toks.append(COMP | ((a & 0x7FFFFFFF) << 31) | (b & 0x7FFFFFFF) |
                                ((a | b) & REM))
            toff.append(len(toks))
    return (np.asarray(keys, np.uint64), np.asarray(toff, np.uint32),
            np.asarray(toks, np.uint64))


def timed(fn, it):
    fn()
    t0 = time.perf_counter()
    for _ in range(it):
        fn()
    return (time.perf_counter() - t0) / it * 1e6


def bench_pair(ctx, order, old, new, it=20, R=1):
    ce = max(max(len(o[0]) for o in old), max(len(o[0]) for o in new), 1)
    ct = max(max(len(o[2]) for o in old), max(len(o[2]) for o in new), 1)
    a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, ce, ct)
    b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, ce, ct)
    for rep in range(R):
        a.upload(*old[rep], replica=rep)
        b.upload(*new[rep], replica=rep)
    m = a.merge(b, order)
    out = {
        "entries_old": int(sum(len(o[0]) for o in old)),
        "tokens_old": int(sum(len(o[2]) for o in old)),
        "entries_new": int(sum(len(o[0]) for o in new)),
        "entries_merged": int(m.counts()[:, 0].sum()),
        "tokens_merged": int(m.counts()[:, 1].sum()),
        "us_merge": timed(lambda: a.merge(b, order), it),
        "us_equal": timed(lambda: a.equal(b, order), it),
        "us_inflation_strict": timed(lambda: m.is_inflation_of(a, order, strict=True), it),
        # lasp_core:bind/3 on the pair: =:=, merge, is_inflation as three calls, and
        # fused (laspj_list_bind: two synchronisations instead of six)
        "us_bind_separate": timed(lambda: (a.equal(b, order), a.merge(b, order)
                                           .is_inflation_of(a, order)), it),
        "us_bind_fused": timed(lambda: a.bind(b, order), it),
    }
    out["operand_bytes"] = 8 * (2 * (out["entries_old"] + out["entries_new"]) +
                                out["tokens_old"] + int(sum(len(o[2]) for o in new)))
    return out, m


def main():
    ctx = engine.Context(0)
    if os.environ.get("LASPJ_LIST_WALK"):          # 1: the step-by-step walk (A/B)
        ctx.set_tuning(_lib.TUNE_LIST_WALK, int(os.environ["LASPJ_LIST_WALK"]))
    res = {}
    rng = np.random.default_rng(5)
    # config 5 intersection output: L = [0, 100k), R = [50k, 150k) -> common [50k, 100k)
    N, D = 100_000, 150_000
    order, keep = identity_order(ctx, D)
    common = np.arange(D - N, N)
    pl, rl = cells(rng, len(common))
    pr, rr = cells(rng, len(common))
    old = intersection_list(common, pl, rl, pr, rr)
    pr2, rr2 = pr.copy(), rr.copy()
    ch = rng.random(len(common)) < 0.10
    pr2[ch] |= np.uint64(8)                                  # a new token (slot 3)
    rm = rng.random(len(common)) < 0.05
    rr2[rm] = pr2[rm]                                        # removals
    new = intersection_list(common, pl, rl, pr2, rr2)
    res["config5_intersection_rebind_50k"], _ = bench_pair(ctx, order, [old], [new])
    print(json.dumps(res), flush=True)
    # the same lists with their entries reversed: keys descend, so the merge takes the
    # clauses' sequential walk (what every list merge did before the merge path)
    rev = lambda l: (l[0][::-1].copy(), np.concatenate([[0], np.cumsum(np.diff(l[1])[::-1])]).astype(np.uint32),  # noqa: E731
                     np.concatenate([l[2][l[1][i]:l[1][i + 1]] for i in range(len(l[0]))][::-1]))
    res["config5_intersection_rebind_50k_unsorted_walk"], _ = bench_pair(
        ctx, order, [rev(old)], [rev(new)], it=5)
    print(json.dumps(res), flush=True)
    # the same entries in a random order shared by both sides (a hash-like map fun: all
    # ties again), and each side in its own random order (short runs everywhere)
    def perm(l, p):
        runs = [l[2][l[1][i]:l[1][i + 1]] for i in range(len(l[0]))]
        return (l[0][p].copy(), np.concatenate([[0], np.cumsum([len(runs[i]) for i in p])]).astype(np.uint32),
                np.concatenate([runs[i] for i in p]))
    p1, p2 = rng.permutation(len(common)), rng.permutation(len(common))
    res["config5_intersection_rebind_50k_shuffled_same"], _ = bench_pair(
        ctx, order, [perm(old, p1)], [perm(new, p1)], it=5)
    res["config5_intersection_rebind_50k_shuffled_each"], _ = bench_pair(
        ctx, order, [perm(old, p1)], [perm(new, p2)], it=3)
    print(json.dumps(res), flush=True)
    # product output 256 x 256
    nx = ny = 256
    order2, keep2 = identity_order(ctx, nx + ny)
    px, rx = cells(rng, nx)
    py, ry = cells(rng, ny)
    oldp = product_list(nx, ny, px, rx, py, ry)
    py2, ry2 = py.copy(), ry.copy()
    py2[::7] |= np.uint64(8)
    newp = product_list(nx, ny, px, rx, py2, ry2)
    res["product_rebind_256x256"], _ = bench_pair(ctx, order2, [oldp], [newp], it=10)
    # batched: 1024 replicas x 200-entry intersection outputs
    Rb, nb = 1024, 200
    olds, news = [], []
    for rep in range(Rb):
        k = np.arange(nb) + rep % 7
        a_, b_ = cells(rng, nb), cells(rng, nb)
        olds.append(intersection_list(k, *a_, *b_))
        b2 = (b_[0] | np.uint64(8), b_[1])
        news.append(intersection_list(k, *a_, *b2))
    res["batched_1024x200_rebind"], _ = bench_pair(ctx, order, olds, news, it=10, R=Rb)
    res["batched_1024x200_rebind"]["us_merge_per_replica"] = \
        res["batched_1024x200_rebind"]["us_merge"] / Rb
    # the Store end to end: update R -> intersection re-run -> re-bind 50k entries
    from lasp_amd import core
    from lasp_amd.terms import Atom
    st = core.Store(capacity=1 << 18)
    l, r, x = (st.declare("lasp_orset")[1] for _ in range(3))
    tk = lambda c, e: bytes([c]) + int(e).to_bytes(19, "big")    # noqa: E731
    st.bind(l, [(e, [(tk(1, e), False)]) for e in range(N)])
    st.bind(r, [(e, [(tk(2, e), False)]) for e in range(D - N, D)])
    st.intersection(l, r, x)
    assert len(st.value(x)) == N - (D - N)
    st.update(r, ("add_by_token", tk(3, 999), D - N + 1), Atom("a"))     # first-use pools
    k = 10
    prof = None
    if os.environ.get("PROFILE_STORE"):
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for i in range(k):
        st.update(r, ("add_by_token", tk(3, i), D - N + 17 * i), Atom("a"))
    res["store_update_rerun_rebind_50k_ms"] = (time.perf_counter() - t0) / k * 1e3
    if prof is not None:
        import pstats
        prof.disable()
        pstats.Stats(prof, stream=sys.stderr).sort_stats("cumulative").print_stats(30)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
