"""The parallel (merge-path) list merge on lists whose keys ascend — the common case of a
re-bound combinator output (intersection, filter or monotone map of canonical inputs) —
against the oracle's clauses (oracle/otp.py orddict_merge / ordsets_union, restating
lasp_orset.erl:128-134 and lasp_gset.erl:99-101 over OTP 17's stdlib).

Lists here are raw list items over a hand-made dictionary in which the int X and the
float X are different element slots of EQUAL rank (1 == 1.0): which of two equal keys a
merge keeps is then visible, so the tests pin orddict:merge's "key of the first list"
and ordsets:union's argument switch (the side of the last single step) across thread
and tile boundaries.  Sizes span several 2048-step tiles, runs of one key longer than a
tile's LDS window, empty sides and unsorted token runs (Cx ++ Cy)."""

import numpy as np
import pytest

from oracle import gset as ogset, orset as oorset
from oracle.terms import exact_eq

pytestmark = pytest.mark.gpu

V = 3000                      # distinct key values; slot 2v = int v, slot 2v+1 = float v
NTOK = 6


def tok_term(k):
    return b"t%02d" % k + b"\x00" * 17


@pytest.fixture(scope="module")
def env():
    from lasp_amd import _lib
    from lasp_amd.orset import context
    ctx = context()
    K = 2 * V
    kr = ctx.buffer(4 * K)
    kr.upload((np.arange(K) // 2).astype(np.uint32))
    # token g = 64 e + k: its term is tok_term(k) whatever e, so equal terms share a rank
    gr = ctx.buffer(4 * 64 * K)
    gr.upload(np.tile(np.arange(64, dtype=np.uint32), K))
    o = _lib.ListOrder()
    o.krank, o.nkeys, o.grank, o.ntokens = kr.h.value, K, gr.h.value, 64 * K
    return ctx, o, (kr, gr)


def key_term(slot):
    v = slot // 2
    return float(v) if slot & 1 else v


def gen(rng, n, runs=False, unsorted_tokens=False, strict=False):
    """A list with non-decreasing keys (strict: ascending ranks, n <= V): (term list,
    keys, toff, toks)."""
    vals = np.sort(rng.choice(V, n, replace=False) if strict else rng.integers(0, V, n))
    if runs and n:
        a = rng.integers(0, max(1, n - 1))
        vals[a:a + n // 2] = vals[a]             # one long run of a single key
        vals = np.sort(vals)
    slots = 2 * vals + rng.integers(0, 2, n)
    keys = slots.astype(np.uint64)
    toff, toks, terms = [0], [], []
    from lasp_amd._lib import LIST_REMOVED
    for s in slots:
        ks = list(rng.choice(NTOK, rng.integers(1, 4), replace=False))
        if not unsorted_tokens:
            ks.sort()
        fl = [bool(rng.integers(0, 2)) for _ in ks]
        toks.extend((64 * int(s) + int(k)) | (LIST_REMOVED if f else 0) for k, f in zip(ks, fl))
        toff.append(len(toks))
        terms.append((key_term(int(s)), [(tok_term(int(k)), f) for k, f in zip(ks, fl)]))
    return terms, keys, np.asarray(toff, np.uint32), np.asarray(toks, np.uint64)


def decode(lb, gset):
    keys, toff, toks = lb.download()
    if gset:
        return [key_term(int(k)) for k in keys]
    from lasp_amd._lib import LIST_REMOVED
    out = []
    for i, k in enumerate(keys):
        run = toks[int(toff[i]):int(toff[i + 1])]
        out.append((key_term(int(k)), [(tok_term(int(t) & 63), bool(int(t) & LIST_REMOVED))
                                       for t in run]))
    return out


SIZES = [(0, 0), (0, 700), (5, 0), (1, 1), (300, 40), (2500, 2600), (6000, 5000),
         (4000, 100), (7, 9000)]


@pytest.mark.parametrize("na,nb", SIZES)
@pytest.mark.parametrize("runs", [False, True])
def test_sorted_orset_list_merge(env, na, nb, runs):
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(na * 7 + nb + runs)
    ta, *ia = gen(rng, na, runs, unsorted_tokens=True)
    tb, *ib = gen(rng, nb, runs, unsorted_tokens=True)
    A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ia)
    B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ib)
    assert exact_eq(decode(A.merge(B, order), False), oorset.merge(ta, tb))
    assert exact_eq(decode(B.merge(A, order), False), oorset.merge(tb, ta))
    from oracle import core as ocore
    assert exact_eq(decode(A.union(B, order), False), ocore.union_body("lasp_orset", ta, tb))


@pytest.mark.parametrize("na,nb", SIZES)
@pytest.mark.parametrize("runs", [False, True])
def test_sorted_gset_list_merge(env, na, nb, runs):
    """ordsets:union: with 1 == 1.0 in different slots the emitted item shows the
    argument switch (the side of the last single step before each pair)."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(1000 + na * 7 + nb + runs)
    ta, ka, _o, _t = gen(rng, na, runs)
    tb, kb, _o, _t = gen(rng, nb, runs)
    ga, gb = [t[0] for t in ta], [t[0] for t in tb]
    A = engine.ListBatch(ctx, _lib.KIND_GSET_LIST).upload(ka)
    B = engine.ListBatch(ctx, _lib.KIND_GSET_LIST).upload(kb)
    assert exact_eq(decode(A.merge(B, order), True), ogset.merge(ga, gb))
    assert exact_eq(decode(B.merge(A, order), True), ogset.merge(gb, ga))


def test_sorted_and_unsorted_replicas_in_one_batch(env):
    """A batch whose replicas mix ascending lists (merge path) and unsorted ones (lane-0
    walk): each replica is the oracle's merge of its pair."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(77)
    R = 12
    A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, 8000, 40000)
    B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, 8000, 40000)
    want = []
    for r in range(R):
        ta, *ia = gen(rng, int(rng.integers(0, 5000)), runs=r % 3 == 0)
        tb, *ib = gen(rng, int(rng.integers(0, 5000)))
        if r % 4 == 1:                           # unsorted keys: reverse A
            n = len(ta)
            ta = ta[::-1]
            keys, toff, toks = ia
            runs_ = [toks[toff[i]:toff[i + 1]] for i in range(n)][::-1]
            ia = [keys[::-1].copy(), np.concatenate([[0], np.cumsum([len(x) for x in runs_])]).astype(np.uint32),
                  np.concatenate(runs_ + [np.zeros(0, np.uint64)]).astype(np.uint64)]
        A.upload(*ia, replica=r)
        B.upload(*ib, replica=r)
        want.append(oorset.merge(ta, tb))
    M = A.merge(B, order)
    for r in range(R):
        keys, toff, toks = M.download(r)
        from lasp_amd._lib import LIST_REMOVED
        got = [(key_term(int(k)), [(tok_term(int(t) & 63), bool(int(t) & LIST_REMOVED))
                                   for t in toks[int(toff[i]):int(toff[i + 1])]])
               for i, k in enumerate(keys)]
        assert exact_eq(got, want[r]), r


def _bind_want(mod, kind, p, v):
    """lasp_core:bind/3 (lasp_core.erl:291-312): 0 no-op, 1 written, 2 not an inflation."""
    from oracle import lattice as olat
    if exact_eq(p, v):
        return 0, None
    m = mod.merge(p, v)
    return (1 if olat.is_inflation(kind, p, m) else 2), m


def _both_paths(ctx, A, B, order):
    """laspj_list_bind on the rank-indexed path (tried first) and on the merge path
    (LASPJ_TUNE_LIST_WALK 2): (status, downloaded merged list) of each."""
    from lasp_amd import _lib
    out = []
    try:
        for tune in (0, 2):
            ctx.set_tuning(_lib.TUNE_LIST_WALK, tune)
            M, st = A.bind(B, order)
            out.append((int(st[0]), M.download() if st[0] else None))
    finally:
        ctx.set_tuning(_lib.TUNE_LIST_WALK, 0)
    return out


BIND_SIZES = [(0, 0), (0, 700), (5, 0), (1, 1), (300, 40), (2500, 2600), (2990, 2980), (7, 2990)]


@pytest.mark.parametrize("na,nb", BIND_SIZES)
@pytest.mark.parametrize("gs", [False, True])
def test_list_bind_ascending_path(env, na, nb, gs):
    """laspj_list_bind when both lists' keys strictly ascend (k_lbf_prep / k_lbf_write:
    the rank-indexed bind, no merge path): status and merged list as the oracle's
    bind/3, and bit-identical to the merge path's.  The int and the float of one value are
    different slots of equal rank here: orddict:merge keeps the first list's key, and a
    G-Set pair of different slots goes to the merge path (ordsets:union's argument switch
    picks its item)."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(4000 + na * 7 + nb + gs)
    ta, *ia = gen(rng, na, strict=True, unsorted_tokens=True)
    tb, *ib = gen(rng, nb, strict=True, unsorted_tokens=True)
    kind, mod = ("lasp_gset", ogset) if gs else ("lasp_orset", oorset)
    lk = _lib.KIND_GSET_LIST if gs else _lib.KIND_ORSET_LIST
    if gs:
        # G-Set statuses are compared with the oracle over int keys only: the list
        # inflation check compares ranks (laspj.h: equal rank = the same term), which the
        # Store's dictionaries guarantee (codec.EqualTerms); sets:is_subset is =:=
        ints = lambda k: (2 * (k[0] // 2)).astype(np.uint64)             # noqa: E731
        ia, ib = [ints(ia)], [ints(ib)]
        ta = [key_term(int(x)) for x in ia[0]]
        tb = [key_term(int(x)) for x in ib[0]]
    for (p, P), (v, Q) in (((ta, ia), (tb, ib)), ((ta, ia), (ta, ia)), ((tb, ib), (ta, ia))):
        A = engine.ListBatch(ctx, lk).upload(*P)
        B = engine.ListBatch(ctx, lk).upload(*Q)
        (s0, m0), (s2, m2) = _both_paths(ctx, A, B, order)
        w, m = _bind_want(mod, kind, p, v)
        assert s0 == s2 == w, (na, nb, s0, s2, w)
        if w:
            assert all(np.array_equal(x, y) for x, y in zip(m0, m2) if x is not None)
            got = decode(engine.ListBatch(ctx, lk).upload(*m0), gs)
            assert exact_eq(got, m)
    if gs and na and nb:
        # a pair of equal rank from two slots (int v, float v): the merge path's item
        ka = ia[0].copy()
        kb = np.unique(np.concatenate([ib[0], ka[:1] + np.uint64(1)]))
        A = engine.ListBatch(ctx, lk).upload(ka)
        B = engine.ListBatch(ctx, lk).upload(kb)
        (s0, m0), (s2, m2) = _both_paths(ctx, A, B, order)
        assert s0 == s2
        assert all(np.array_equal(x, y) for x, y in zip(m0, m2))


def test_list_bind_ascending_large_and_fallbacks():
    """At the bench's scale (60k-80k-entry lists over 200k ranks, 1-3 tokens per entry
    in any order): the rank-indexed bind equals the merge path bit for bit; a Value whose
    keys descend somewhere, one with a repeated key, and a 3-replica batch with one such
    replica fall back to the merge path (same answer as the merge path's)."""
    from lasp_amd import _lib, engine
    from lasp_amd.orset import context
    ctx = context()
    K = 200_000
    kr = ctx.buffer(4 * K)
    kr.upload(np.arange(K, dtype=np.uint32))
    gr = ctx.buffer(4 * 64 * K)
    gr.upload(np.tile(np.arange(64, dtype=np.uint32), K))
    order = _lib.ListOrder()
    order.krank, order.nkeys, order.grank, order.ntokens = kr.h.value, K, gr.h.value, 64 * K
    rng = np.random.default_rng(9)

    def lst(n, desc=False, dup=False):
        keys = np.sort(rng.choice(K, n, replace=False)).astype(np.uint64)
        if desc:
            keys[n // 2], keys[n // 2 + 1] = keys[n // 2 + 1], keys[n // 2]
        if dup:
            keys[n // 3 + 1] = keys[n // 3]
        cnt = rng.integers(1, 4, n)
        toff = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
        toks = np.concatenate([(64 * int(k) + rng.choice(6, c, replace=False)).astype(np.uint64)
                               for k, c in zip(keys, cnt)])
        toks |= (rng.random(len(toks)) < 0.2).astype(np.uint64) << np.uint64(63)
        return keys, toff, toks

    a, b = lst(60_000), lst(80_000)
    for p, q in ((a, b), (a, a), (b, a), (a, lst(70_000, desc=True)), (a, lst(50_000, dup=True))):
        A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*p)
        B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*q)
        (s0, m0), (s2, m2) = _both_paths(ctx, A, B, order)
        assert s0 == s2
        if s0:
            assert all(np.array_equal(x, y) for x, y in zip(m0, m2))
    # three replicas, the middle one descending
    A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, 3, 80_000, 240_000)
    B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, 3, 80_000, 240_000)
    for r, (p, q) in enumerate(((a, b), (lst(1000), lst(900, desc=True)), (b, a))):
        A.upload(*p, replica=r)
        B.upload(*q, replica=r)
    outs = []
    try:
        for tune in (0, 2):
            ctx.set_tuning(_lib.TUNE_LIST_WALK, tune)
            M, st = A.bind(B, order)
            outs.append((list(st), [M.download(r) for r in range(3)]))
    finally:
        ctx.set_tuning(_lib.TUNE_LIST_WALK, 0)
    assert outs[0][0] == outs[1][0] == [1, 1, 1]
    for x, y in zip(outs[0][1], outs[1][1]):
        assert all(np.array_equal(u, w) for u, w in zip(x, y))
