"""The keyed fused dataflow threshold (laspj_orset_gather_inflation_keyed) against the
oracle lattice on whole objects.

A map / filter / fold pipeline whose output keys repeat across source elements (a
collapsing map X div 3, a fold X -> [X, X + 1] whose lists overlap, ...) binds lists in
which lists:keyfind pairs each Prev entry with the FIRST Cur entry of its key
(lasp_lattice.erl:153-161, 235-253, 277-285), not with the entry at its own position.
Each case runs the reference's bodies (oracle/core.py: map_body / filter_body /
fold_body, lasp_core.erl:641-712, 460-486) and lattice (oracle/lattice.py) on every
replica and compares the device's fused gather + threshold, and its cells, with them.
The CPU test pins the numpy keyfind restatement the full-size config-4 test uses
(tests/test_gpu_configs.py:keyfind_threshold) to the same oracle.
"""

import itertools

import numpy as np
import pytest

from oracle import core as ocore
from oracle import lattice as olat
from oracle.terms import exact_eq

from test_gpu_configs import keyfind_threshold, tok, window_orddict

MAPS = {"div3": lambda x: x // 3, "rem7": lambda x: x % 7, "neg": lambda x: -x,
        "id": lambda x: x}
PREDS = {"drop3": lambda x: x % 3 != 0, "even": lambda x: x % 2 == 0, "all": lambda x: True}
FOLDS = {"fan4": lambda x: [x] * (x % 4), "pair": lambda x: [x, x + 1],
         "trip": lambda x: [x, x, x]}


def pipeline(E, F1, pred, F2):
    """Dictionary-level indexes of map -> filter -> fold over element slots 0..E-1
    (slot e = the int e): fold slot -> mapped slot f, the composed index (empty where
    the filter drops), and the output keys."""
    k1 = np.array([F1(e) for e in range(E)], dtype=np.int64)
    keep = np.array([bool(pred(int(x))) for x in k1])
    f, okeys = [], []
    for e in range(E):
        for v in F2(int(k1[e])):
            f.append(e)
            okeys.append(v)
    f = np.array(f, dtype=np.uint32)
    comp = np.where(keep[f], f, 0xFFFFFFFF).astype(np.uint32)
    return f, comp, np.array(okeys, dtype=np.int64)


def replicas(rng, R, E, T=3):
    p = rng.integers(1, 1 << T, (R, E)).astype(np.uint64)
    p[rng.random((R, E)) < 0.2] = 0
    r = p & rng.integers(0, 1 << T, (R, E)).astype(np.uint64)
    return np.stack([p, r], axis=-1)


def cases(seed, R, E):
    """(Prev, Cur) input replicas: half inflations (Cur = Prev ⊔ X), a quarter
    unrelated, a quarter equal or with extra removals."""
    rng = np.random.default_rng(seed)
    a, x = replicas(rng, R, E), replicas(rng, R, E)
    b = a | x
    q = R // 4
    b[q:2 * q] = x[q:2 * q]
    b[2 * q:3 * q] = a[2 * q:3 * q]
    b[3 * q:, :, 1] = a[3 * q:, :, 0] & (a[3 * q:, :, 1] | np.uint64(1))
    b[3 * q:, :, 0] = a[3 * q:, :, 0]
    return a, b


def oracle_list(cells, F1, pred, F2):
    return ocore.fold_body("lasp_orset", F2, ocore.filter_body(
        "lasp_orset", pred, ocore.map_body("lasp_orset", F1, window_orddict(cells, 0))))


def device_list(cells, f, okeys):
    out = []
    for o, (p, r) in enumerate(cells):
        p, r = int(p), int(r)
        if p:
            se = int(f[o])
            out.append((int(okeys[o]), [(tok(se, k), bool((r >> k) & 1))
                                        for k in range(64) if (p >> k) & 1]))
    return out


def test_keyfind_restatement_matches_oracle():
    """CPU: the numpy keyfind threshold on cells == the oracle lattice on the lists the
    oracle bodies produce, for every pipeline shape."""
    E, R = 30, 16
    for (mn, F1), (pn, pred), (fn, F2) in itertools.product(MAPS.items(), PREDS.items(),
                                                            FOLDS.items()):
        f, comp, okeys = pipeline(E, F1, pred, F2)
        a, b = cases(hash((mn, pn, fn)) % 1000, R, E)
        for i in range(R):
            pa = np.where((comp < E)[:, None], a[i][np.minimum(comp, E - 1)], 0)
            pb = np.where((comp < E)[:, None], b[i][np.minimum(comp, E - 1)], 0)
            la, lb = oracle_list(a[i], F1, pred, F2), oracle_list(b[i], F1, pred, F2)
            assert exact_eq(device_list(pa, f, okeys), la)
            for strict in (False, True):
                want = (olat.is_strict_inflation if strict else olat.is_inflation)(
                    "lasp_orset", la, lb)
                assert keyfind_threshold(pa, pb, comp, okeys, strict) == want, \
                    (mn, pn, fn, i, strict)


@pytest.mark.gpu
@pytest.mark.parametrize("mn,pn,fn", list(itertools.product(MAPS, PREDS, FOLDS)))
def test_keyed_gather_inflation_vs_oracle(mn, pn, fn):
    from lasp_amd.engine import key_chains
    from lasp_amd.orset import context
    ctx = context()
    F1, pred, F2 = MAPS[mn], PREDS[pn], FOLDS[fn]
    E, R = 40, 32
    f, comp, okeys = pipeline(E, F1, pred, F2)
    n_out = len(f)
    a, b = cases(7 + len(mn) * 31 + len(pn) * 7 + len(fn), R, E)
    A, B = ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    A.upload(a.reshape(R, -1))
    B.upload(b.reshape(R, -1))
    chains = key_chains(okeys)
    fa, fb = ctx.orset_batch(R, n_out), ctx.orset_batch(R, n_out)
    empty = ctx.orset_batch(1, n_out)
    first = fa.gather_inflation(A, comp, empty, strict=True, chains=chains)
    got = {s: ctx.orset_batch(R, n_out).gather_inflation(B, comp, fa, strict=s, chains=chains)
           for s in (False, True)}
    fb.gather_inflation(B, comp, fa, strict=True, chains=chains)
    da, db = fa.download(), fb.download()
    for i in range(R):
        la, lb = oracle_list(a[i], F1, pred, F2), oracle_list(b[i], F1, pred, F2)
        assert exact_eq(device_list(da[i], f, okeys), la), i
        assert exact_eq(device_list(db[i], f, okeys), lb), i
        assert first[i] == olat.is_strict_inflation("lasp_orset", [], la), i
        for strict in (False, True):
            want = (olat.is_strict_inflation if strict else olat.is_inflation)(
                "lasp_orset", la, lb)
            assert got[strict][i] == want, (i, strict)
    # a single-replica Prev broadcast over every Cur replica
    bc = ctx.orset_batch(R, n_out).gather_inflation(B, comp, fa.view(0, 1), strict=True,
                                                    chains=chains)
    la = oracle_list(a[0], F1, pred, F2)
    for i in range(R):
        assert bc[i] == olat.is_strict_inflation("lasp_orset", la,
                                                 oracle_list(b[i], F1, pred, F2)), i


@pytest.mark.gpu
def test_keyed_chain_arguments():
    """head / next must come together; a malformed chain (a cycle) ends (forward walks
    only) instead of hanging."""
    from lasp_amd import _lib
    from lasp_amd.orset import context
    ctx = context()
    E = 8
    A, D, P = ctx.orset_batch(2, E), ctx.orset_batch(2, E), ctx.orset_batch(2, E)
    A.fill_synthetic(3)
    idx = np.arange(E, dtype=np.uint32)
    head = np.zeros(E, np.uint32)
    nxt = np.array([3, 0, 1, 2, 7, 6, 5, 0xFFFFFFFF], np.uint32)    # backward links
    D.gather_inflation(A, idx, P, strict=True, chains=(head, nxt))
    L = ctx.L
    b = ctx.buffer(4 * E)
    out = ctx.buffer(2)
    assert L.laspj_orset_gather_inflation_keyed(ctx.h, D.h, A.h, b.h, b.h, None, P.h, 1,
                                                out.h) == _lib.E_INVAL
