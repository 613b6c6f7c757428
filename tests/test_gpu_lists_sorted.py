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


def gen(rng, n, runs=False, unsorted_tokens=False):
    """A list with non-decreasing keys: (term list, keys, toff, toks)."""
    vals = np.sort(rng.integers(0, V, n))
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
