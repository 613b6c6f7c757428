"""The list merges for keys that do NOT ascend — the run-jumping walk (merge_runs_replica in
k_merge_tile_scan, laspj_lists.hip) and the chunked walk over the chip (k_merge_spec) — on lists whose keys do NOT
ascend — a non-monotone map's output re-bound (lasp_core.erl:641-667 then :300, merged by
lasp_orset.erl:128-134 / lasp_gset.erl:99-101 over OTP 17's two-finger clauses, SURVEY
Appendix A) — against the oracle's clauses (oracle/otp.py via oracle/orset.py,
oracle/gset.py, oracle/core.py) and against the step-by-step walk it replaced
(LASPJ_TUNE_LIST_WALK 1).

Shapes are chosen for the walk's run structure: reversed lists re-bound with a few
entries added or dropped (one long tie run, then one side's rest), identical descending
lists longer than the 256-rank window and the 1024-rank streaming step, alternating
ascending / descending blocks (long single-side runs in both directions), small key
alphabets (repeated keys everywhere) and random orders (short runs).  Keys use the
1 == 1.0 dictionary of test_gpu_lists_sorted.py, so which of two equal keys a tie keeps
(orddict:merge: the first list's) and the side ordsets:union's argument switch takes are
visible in the output."""

import numpy as np
import pytest

from oracle import core as ocore, gset as ogset, orset as oorset
from oracle.terms import exact_eq

from test_gpu_lists_sorted import NTOK, decode, env, key_term, tok_term  # noqa: F401

pytestmark = pytest.mark.gpu


def _list(rng, vals):
    """An OR-Set list with the given key values (int or float slot at random)."""
    from lasp_amd._lib import LIST_REMOVED
    slots = 2 * np.asarray(vals, np.int64) + rng.integers(0, 2, len(vals))
    toff, toks, terms = [0], [], []
    for s in slots:
        ks = list(rng.choice(NTOK, rng.integers(1, 4), replace=False))
        fl = [bool(rng.integers(0, 2)) for _ in ks]
        toks.extend((64 * int(s) + int(k)) | (LIST_REMOVED if f else 0) for k, f in zip(ks, fl))
        toff.append(len(toks))
        terms.append((key_term(int(s)), [(tok_term(int(k)), f) for k, f in zip(ks, fl)]))
    return terms, slots.astype(np.uint64), np.asarray(toff, np.uint32), \
        np.asarray(toks, np.uint64)


def _edit(rng, vals, n_ins, n_del, V):
    v = list(vals)
    for _ in range(n_del):
        if v:
            v.pop(int(rng.integers(0, len(v))))
    for _ in range(n_ins):
        v.insert(int(rng.integers(0, len(v) + 1)), int(rng.integers(0, V)))
    return v


def shapes(rng):
    V = 3000
    out = []
    desc = list(range(2999, 2999 - 2600, -1))
    out.append(("reversed, identical", desc, list(desc)))
    out.append(("reversed, a few added", desc, _edit(rng, desc, 5, 0, V)))
    out.append(("reversed, a few dropped", desc, _edit(rng, desc, 0, 7, V)))
    out.append(("reversed, edited both", _edit(rng, desc, 3, 3, V), _edit(rng, desc, 4, 2, V)))
    long_desc = list(np.repeat(np.arange(2999, 0, -1), 3))[:8000]
    out.append(("long descending, repeated keys", long_desc, list(long_desc)))
    blocks = []
    for k in range(12):
        b = list(rng.integers(0, V, int(rng.integers(50, 1500))))
        b.sort(reverse=bool(k % 2))
        blocks += b
    blocks2 = list(blocks)
    rng.shuffle(blocks2[:300])
    out.append(("alternating blocks", blocks, blocks2))
    out.append(("alternating blocks vs reversed", blocks, blocks[::-1]))
    out.append(("small alphabet", list(rng.integers(0, 5, 3000)), list(rng.integers(0, 5, 2500))))
    out.append(("random order", list(rng.permutation(V)[:2000]), list(rng.permutation(V)[:2200])))
    out.append(("random vs itself", list(rng.permutation(V)[:1800]), None))
    out.append(("descending vs ascending", desc, sorted(desc)))
    out.append(("one side empty", desc, []))
    out.append(("single entries", [5], [5]))
    return [(name, a, list(a) if b is None else b) for name, a, b in shapes_fix(out)]


def shapes_fix(out):
    return [(n, list(map(int, a)), None if b is None else list(map(int, b))) for n, a, b in out]


def _walks(ctx, fn):
    """fn() with the default walk, the step walk (LASPJ_TUNE_LIST_WALK 1) and the chunked
    walk over the chip (3, k_merge_spec: chunks of 256 rows, so these shapes span up to
    32 chunks); the chunked result must equal the default one."""
    from lasp_amd import _lib
    got = fn()
    try:
        ctx.set_tuning(_lib.TUNE_LIST_WALK, 3)
        chunked = fn()
        ctx.set_tuning(_lib.TUNE_LIST_WALK, 1)
        step = fn()
    finally:
        ctx.set_tuning(_lib.TUNE_LIST_WALK, 0)
    assert exact_eq(chunked, got)
    return got, step


@pytest.mark.parametrize("k", range(13))
def test_unsorted_orset_merge_and_union(env, k):
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(500 + k)
    name, va, vb = shapes(rng)[k]
    ta, *ia = _list(rng, va)
    tb, *ib = _list(rng, vb)
    A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ia)
    B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ib)
    for x, y, tx, ty in ((A, B, ta, tb), (B, A, tb, ta)):
        got, step = _walks(ctx, lambda: decode(x.merge(y, order), False))
        want = oorset.merge(tx, ty)
        assert exact_eq(got, want), name
        assert exact_eq(step, want), name
        got, step = _walks(ctx, lambda: decode(x.union(y, order), False))
        want = ocore.union_body("lasp_orset", tx, ty)
        assert exact_eq(got, want), name
        assert exact_eq(step, want), name


@pytest.mark.parametrize("k", range(13))
def test_unsorted_gset_merge(env, k):
    """ordsets:union with OTP 17's argument switch: a tie emits the item of the side of
    the last single step, visible as int vs float keys."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(900 + k)
    name, va, vb = shapes(rng)[k]
    ta, ka, _o, _t = _list(rng, va)
    tb, kb, _o, _t = _list(rng, vb)
    ga, gb = [t[0] for t in ta], [t[0] for t in tb]
    A = engine.ListBatch(ctx, _lib.KIND_GSET_LIST).upload(ka)
    B = engine.ListBatch(ctx, _lib.KIND_GSET_LIST).upload(kb)
    for x, y, gx, gy in ((A, B, ga, gb), (B, A, gb, ga)):
        got, step = _walks(ctx, lambda: decode(x.merge(y, order), True))
        want = ogset.merge(gx, gy)
        assert exact_eq(got, want), name
        assert exact_eq(step, want), name


def test_unsorted_replicas_batched(env):
    """Many replicas per launch, each its own shape, one wave per replica."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(4242)
    sh = shapes(rng)
    R = len(sh)
    A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, 12000, 40000)
    B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, R, 12000, 40000)
    want = []
    for r, (name, va, vb) in enumerate(sh):
        ta, *ia = _list(rng, va)
        tb, *ib = _list(rng, vb)
        A.upload(*ia, replica=r)
        B.upload(*ib, replica=r)
        want.append(oorset.merge(ta, tb))
    M = A.merge(B, order)
    from lasp_amd._lib import LIST_REMOVED
    for r in range(R):
        keys, toff, toks = M.download(r)
        got = [(key_term(int(k)), [(tok_term(int(t) & 63), bool(int(t) & LIST_REMOVED))
                                   for t in toks[int(toff[i]):int(toff[i + 1])]])
               for i, k in enumerate(keys)]
        assert exact_eq(got, want[r]), sh[r][0]


def test_chunked_walk_bind_at_scale(env):
    """laspj_list_bind of independently shuffled 20k-entry lists (the bench's
    shuffled-each case at 2/5 size): the first bind finds the keys not ascending (the
    rank-indexed path answers 3), marks the lists, and the merge path's chunked walk
    runs; then each bind again.  Statuses and merged lists equal the step walk's, and the
    merged list of one pair equals the oracle's merge."""
    from lasp_amd import _lib, engine
    ctx, order, _keep = env
    rng = np.random.default_rng(77)
    V = 3000
    for name, va, vb in (("shuffled each", list(rng.integers(0, V, 20000)), list(rng.integers(0, V, 19000))),
                         ("reversed", list(range(2999, 0, -1)) * 3, list(range(2999, 0, -1)) * 3),
                         ("random vs sorted", list(rng.integers(0, V, 9000)), sorted(rng.integers(0, V, 9000)))):
        ta, *ia = _list(rng, [int(x) for x in va])
        tb, *ib = _list(rng, [int(x) for x in vb])
        A = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ia)
        B = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*ib)
        outs = []
        for _ in range(2):                                  # first: the fallback; then hinted
            M, st = A.bind(B, order)
            outs.append((int(st[0]), M.download()))
        try:
            ctx.set_tuning(_lib.TUNE_LIST_WALK, 1)
            M, st = A.bind(B, order)
            step = (int(st[0]), M.download())
        finally:
            ctx.set_tuning(_lib.TUNE_LIST_WALK, 0)
        for o in outs:
            assert o[0] == step[0], name
            assert all(np.array_equal(x, y) for x, y in zip(o[1], step[1])), name
        if name == "random vs sorted":
            assert exact_eq(decode(engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*outs[1][1]), False),
                            oorset.merge(ta, tb))
