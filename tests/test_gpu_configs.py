"""GPU parity at BASELINE.json's configs 1, 3, 4 and 5 (their full workload sizes).

Whole objects at these sizes are far beyond what the list-walking oracle finishes
(its keyfind / `Acc ++` loops are quadratic), so each test combines
  * whole-batch properties that do not depend on size (fused == unfused bit for bit,
    the threshold of the dataflow equal to the inflation of its inputs, convergence of
    a round to the join), and
  * sampled objects x element windows checked against the oracle's own bodies: the
    combinator bodies treat elements one at a time and in list order, so the output for
    a window of input elements is the body applied to that window's sub-orddict.
Inputs are the device's seeded synthetic streams, restated in oracle/laspj_oracle.c
(orc_synth_orset, orc_synth_orset_t) and read here from the oracle side.
"""

import numpy as np
import pytest

from oracle import columnar as orc
from oracle import core as ocore
from oracle.terms import exact_eq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lasp_amd.orset import context
    return context()


def tok(e, k):
    """A 20-byte token for token slot k of element e (slot order = byte order)."""
    return int(e).to_bytes(8, "big") + bytes([k]) + b"\0" * 11


def window_orddict(cells, e0, key=lambda e: e):
    """The sub-orddict of elements [e0, e0 + len(cells)) of a canonical replica."""
    out = []
    for i, (p, r) in enumerate(cells):
        p, r = int(p), int(r)
        if p:
            e = e0 + i
            out.append((key(e), [(tok(e, k), bool((r >> k) & 1)) for k in range(64) if (p >> k) & 1]))
    return out



# ----------------------------------------------------------------------------- config 1

def _cfg1_terms():
    """BASELINE configs[0] / SURVEY.md §8d cfg 1: replica A adds 0..9999 with token tA(e);
    replica B adds them with tB(e) and removes a 10 % subset (seed 1); a second set C of
    10k ints overlaps the first in 5k."""
    n = 10_000
    rng = np.random.default_rng(1)
    removed = set(int(x) for x in rng.choice(n, n // 10, replace=False))
    tA = lambda e: b"A" + e.to_bytes(19, "big")     # noqa: E731
    tB = lambda e: b"B" + e.to_bytes(19, "big")     # noqa: E731
    tC = lambda e: b"C" + e.to_bytes(19, "big")     # noqa: E731
    A = [(e, [(tA(e), False)]) for e in range(n)]
    B = [(e, [(tB(e), e in removed)]) for e in range(n)]
    C = [(e, [(tC(e), False)]) for e in range(n // 2, n // 2 + n)]
    return A, B, C


def test_config1_terms_merge_union_filter():
    """BASELINE configs[0] term for term: lasp_orset:merge/2 of the two 10k-element
    replicas (lasp_orset.erl:128-134) through the drop-in mirror, then the lasp_core
    union (keep-left orddict:merge, lasp_core.erl:602-627) with the second set and
    filter(X rem 2 == 0) (lasp_core.erl:681-712, fun from lasp_filter_test.erl:70) run as
    dataflow processes on the device store and re-run when B is bound; every value is
    compared with the oracle's merge and bodies."""
    from lasp_amd import core as dcore, orset as dorset
    from oracle import orset as oorset, lattice as olat
    A, B, C = _cfg1_terms()
    M = oorset.merge(A, B)
    assert exact_eq(dorset.merge(A, B), M)
    assert exact_eq(dorset.value(M), oorset.value(M))
    from lasp_amd import lattice as dlat
    assert dlat.is_inflation("lasp_orset", A, M) == olat.is_inflation("lasp_orset", A, M)
    assert dlat.is_strict_inflation("lasp_orset", A, M) is True
    even = lambda x: x % 2 == 0                    # noqa: E731
    U = ocore.union_body("lasp_orset", M, C)
    F = ocore.filter_body("lasp_orset", even, U)
    # (the oracle Store's quadratic keyfind inflation takes ~400 s at this size, so the
    # device store is compared with the oracle bodies directly)
    st = dcore.Store(capacity=1 << 15)             # element slots per variable
    _, a = st.declare("lasp_orset")
    _, c = st.declare("lasp_orset")
    _, u = st.declare("lasp_orset")
    _, f = st.declare("lasp_orset")
    st.union(a, c, u)
    st.filter(u, even, f)
    st.bind(a, A)
    st.bind(c, C)
    st.bind(a, B)                                  # bind = merge(A, B): the config's merge
    assert exact_eq(st.value(a), M)
    assert exact_eq(st.value(u), U)
    assert exact_eq(st.value(f), F)
    assert len(U) == 15_000 and len(F) == 7_500


def test_config1_bench_kernels():
    """The calls bench.py's config1_gpu times (one 20k-slot replica pair: join, union,
    filter with the even-slot mask, value/1, is_inflation) against the C orddict
    restatement on the same synthetic replicas (element e = slot e)."""
    n = 20_000
    a, b = ctx_orset(n, 2), ctx_orset(n, 3)
    ctx = a.ctx
    tokens = orc.synth_tokens(n)
    oa = orc.ORDict.from_cells(orc.synth_orset(2, 0, n), tokens)
    ob = orc.ORDict.from_cells(orc.synth_orset(3, 0, n), tokens)
    m = ctx.orset_batch(1, n).join(a, b)
    om = oa.merge(ob)
    assert orc.ORDict.from_cells(m.download()[0], tokens).equal(om)
    u = ctx.orset_batch(1, n).union(a, b)
    assert orc.ORDict.from_cells(u.download()[0], tokens).equal(oa.union(ob))
    keep = np.full(((n + 63) // 64,), 0x5555555555555555, np.uint64)
    f = ctx.orset_batch(1, n).filter(m, keep)
    assert orc.ORDict.from_cells(f.download()[0], tokens).equal(om.filter_even())
    bits = np.unpackbits(m.value_bits()[0].view(np.uint8), bitorder="little")[:n]
    assert np.array_equal(np.nonzero(bits)[0], om.value())
    assert bool(m.is_inflation_of(a)[0]) == om.is_inflation_of(oa) is True
    assert bool(m.is_inflation_of(a, strict=True)[0]) == om.is_strict_inflation_of(oa)
    assert bool(a.is_inflation_of(m)[0]) == oa.is_inflation_of(om)


def ctx_orset(n, seed):
    from lasp_amd.orset import context
    b = context().orset_batch(1, n)
    b.fill_synthetic(seed)
    return b

# ----------------------------------------------------------------------------- config 4

def test_config4_dataflow_full_size(ctx):
    """BASELINE configs[3]: 1024 OR-Set objects x 2^20 int elements x 3 tokens through
    map X -> 2X (riak_test lasp_map_test.erl:70), filter even (lasp_filter_test.erl:70),
    fold X -> [X, X, X] (lasp_fold_test.erl:70) and the {strict, Prev} threshold read of
    the fold output — fused into one gather + inflation pass and checked against the
    four-launch pipeline, the oracle bodies on sampled windows, and the inflation of the
    inputs."""
    from lasp_amd import _lib
    R, E, T = 1024, 1 << 20, 3
    # dictionary level (once per element, host): map m[i] = i (2X keeps list order),
    # filter keeps every mapped slot (2X is even), fold f[o] = o // 3; composite o // 3
    m = np.arange(E, dtype=np.uint32)
    keep = np.full(((E + 63) // 64,), ~np.uint64(0), np.uint64)
    f = np.repeat(np.arange(E, dtype=np.uint32), 3)
    comp = f.copy()
    A, B = ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    A.fill_synthetic(40, token_slots=T)
    B.fill_synthetic(41, token_slots=T)
    B.join(A, B)                                    # B inflates A
    empty = ctx.orset_batch(1, 3 * E)
    foldA = ctx.orset_batch(R, 3 * E)
    first = foldA.gather_inflation(A, comp, empty, strict=True)
    assert first.all()                              # [] -> non-empty: strict ({strict, new()})
    foldB = ctx.orset_batch(R, 3 * E)
    flags = foldB.gather_inflation(B, comp, foldA, strict=True)
    # unfused: gather -> filter -> gather, then the inflation kernel
    mapped = ctx.orset_batch(R, E).gather(B, m)
    filt = ctx.orset_batch(R, E).filter(mapped, keep)
    del mapped
    ref = ctx.orset_batch(R, 3 * E).gather(filt, f)
    assert ref.equal(foldB).all(), "fused fold output differs from the staged pipeline"
    assert np.array_equal(ref.is_inflation_of(foldA, strict=True), flags)
    del ref
    # size-independent: the fold triplicates, map / filter are 1:1 here, so the strict
    # threshold of fold(B) over fold(A) is the strict inflation of B over A
    assert np.array_equal(B.is_inflation_of(A, strict=True), flags)
    assert np.array_equal(foldB.is_inflation_of(foldA, strict=False),
                          np.ones((R,), dtype=bool))
    # stats: 3 x the entries and tokens of the input
    sb, sf = B.stats(), foldB.stats()
    assert np.array_equal(sf, 3 * sb)
    # sampled objects x windows against the oracle bodies (A's stream restated in C)
    dbl = lambda x: 2 * x                # noqa: E731
    even = lambda x: x % 2 == 0          # noqa: E731
    trip = lambda x: [x, x, x]           # noqa: E731
    K = 48
    for rep in (0, 517, R - 1):
        for e0 in (0, 333_333, E - K):
            src = orc.synth_orset_t(40, rep, e0, K, T)
            assert np.array_equal(A.download(rep, 1)[0, e0:e0 + K], src)
            want = ocore.fold_body("lasp_orset", trip, ocore.filter_body(
                "lasp_orset", even, ocore.map_body("lasp_orset", dbl, window_orddict(src, e0))))
            cells = foldA.download(rep, 1)[0, 3 * e0:3 * (e0 + K)]
            got = []
            for o, (p, r) in enumerate(cells):
                p, r = int(p), int(r)
                if p:
                    e = e0 + o // 3
                    got.append((2 * e, [(tok(e, k), bool((r >> k) & 1))
                                        for k in range(64) if (p >> k) & 1]))
            assert exact_eq(got, want), (rep, e0)
    # the kernel refuses aliasing / bad shapes before launching
    with pytest.raises(_lib.LaspjError):
        foldB.gather_inflation(B, comp, foldB)


def keyfind_threshold(prev, cur, src, keys, strict):
    """is_(strict_)inflation(Prev, Cur) (lasp_lattice.erl:153-161, 235-253) of two lists
    held as cells over the same output slots (list order = slot order, present = p != 0),
    slot o carrying key keys[o] and the tokens of source slot src[o]: lists:keyfind's
    first match is the first present Cur slot of each key (np.unique's first index).
    Tokens of different source slots are different terms (fresh tokens)."""
    pp, cp = np.nonzero(prev[:, 0])[0], np.nonzero(cur[:, 0])[0]
    if strict and len(pp) == 0:
        return len(cp) > 0
    uk, fi = np.unique(keys[cp], return_index=True)
    first = cp[fi]
    pos = np.minimum(np.searchsorted(uk, keys[pp]), max(len(uk) - 1, 0))
    found = (uk[pos] == keys[pp]) if len(uk) else np.zeros(len(pp), bool)
    j = first[pos] if len(uk) else np.zeros(len(pp), np.int64)
    same = src[j] == src[pp]
    pc, cc = prev[pp], cur[j]
    ok = found & same & ((pc[:, 0] & ~cc[:, 0]) == 0)
    infl = bool(ok.all())
    if not strict:
        return infl
    changed = bool((found & (~same | (pc[:, 0] != cc[:, 0]) | (pc[:, 1] != cc[:, 1]))).any())
    return infl and (changed or len(pp) < len(cp))


def test_config4_collapsing_pipeline_full_size(ctx):
    """BASELINE configs[3]'s shape with a pipeline whose output keys repeat across source
    elements: map X -> X div 3 (collapsing), filter X rem 3 =/= 0 (drops whole keys), fold
    X -> [X || _ <- lists:seq(1, X rem 4)] (fan-out 0..3), then the {strict, Prev} read —
    through the keyed fused kernel (laspj_orset_gather_inflation_keyed, whose composed
    index has the filter's empty slots).  Checked: cells == the staged gather -> filter ->
    gather pipeline; thresholds == the keyfind restatement above on sampled replicas
    (pinned to the oracle lattice in tests/test_gpu_keyed.py); windows == the oracle
    map / filter / fold bodies."""
    from lasp_amd.engine import key_chains
    R, E, T = 1024, 1 << 20, 3
    e = np.arange(E, dtype=np.int64)
    key1 = e // 3                                    # map: slot e keeps position, key e div 3
    keep1 = key1 % 3 != 0                            # filter on the mapped key
    fan = key1 % 4                                   # fold fan-out per mapped slot
    f = np.repeat(e, fan).astype(np.uint32)          # fold slot -> mapped slot (list order)
    okeys = key1[f]
    comp = np.where(keep1[f], f, 0xFFFFFFFF).astype(np.uint32)
    chains = key_chains(okeys)
    n_out = len(f)
    keepbits = np.packbits(keep1.astype(np.uint8), bitorder="little").view(np.uint64)
    A, B = ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    A.fill_synthetic(42, token_slots=T)
    B.fill_synthetic(43, token_slots=T)
    B.join(A, B)
    empty = ctx.orset_batch(1, n_out)
    foldA = ctx.orset_batch(R, n_out)
    first = foldA.gather_inflation(A, comp, empty, strict=True, chains=chains)
    foldB = ctx.orset_batch(R, n_out)
    flags = foldB.gather_inflation(B, comp, foldA, strict=True, chains=chains)
    flags_ns = ctx.orset_batch(R, n_out).gather_inflation(B, comp, foldA, strict=False,
                                                          chains=chains)
    mapped = ctx.orset_batch(R, E).gather(B, e.astype(np.uint32))
    filt = ctx.orset_batch(R, E).filter(mapped, keepbits)
    del mapped
    ref = ctx.orset_batch(R, n_out).gather(filt, f)
    del filt
    assert ref.equal(foldB).all(), "keyed fused output differs from the staged pipeline"
    del ref
    for rep in (0, 1, 2, 3, 517, R - 1):
        pa, pb = foldA.download(rep, 1)[0], foldB.download(rep, 1)[0]
        assert first[rep] == keyfind_threshold(np.zeros_like(pa), pa, comp, okeys, True)
        assert flags[rep] == keyfind_threshold(pa, pb, comp, okeys, True), rep
        assert flags_ns[rep] == keyfind_threshold(pa, pb, comp, okeys, False), rep
    # a collapsing map makes keyfind compare entries of different source elements, so
    # B over A is rarely an inflation here, unlike the slot-wise reading
    assert not flags_ns.all()
    div3 = lambda x: x // 3                          # noqa: E731
    drop3 = lambda x: x % 3 != 0                     # noqa: E731
    fanf = lambda x: [x] * (x % 4)                   # noqa: E731
    K = 48
    for rep in (0, 517, R - 1):
        for e0 in (0, 333_333, E - K):
            src = orc.synth_orset_t(43, rep, e0, K, T)
            srcA = orc.synth_orset_t(42, rep, e0, K, T)
            merged = [(int(x) | int(y), int(z) | int(w)) for (x, z), (y, w) in zip(src, srcA)]
            want = ocore.fold_body("lasp_orset", fanf, ocore.filter_body(
                "lasp_orset", drop3, ocore.map_body("lasp_orset", div3, window_orddict(merged, e0))))
            lo, hi = np.searchsorted(f, e0), np.searchsorted(f, e0 + K)
            cells = foldB.download(rep, 1)[0, lo:hi]
            got = []
            for o, (p, r) in enumerate(cells):
                p, r = int(p), int(r)
                if p:
                    se = int(f[lo + o])
                    got.append((se // 3, [(tok(se, k), bool((r >> k) & 1))
                                          for k in range(64) if (p >> k) & 1]))
            assert exact_eq(got, want), (rep, e0)


# ----------------------------------------------------------------------------- config 5

def test_config5_intersection_full_size(ctx):
    """BASELINE configs[4] intersection: 1024 pairs of 100k-element OR-Sets with 50 %
    id overlap (L = elements [0, 100k), R = [50k, 150k), T = 3) — every element
    present, as the T-token stream guarantees; sampled pairs x windows against
    intersection_body (keyfind, Cx ++ Cy)."""
    from lasp_amd.codec import Domain, decode_concat
    P, N, D = 1024, 100_000, 150_000
    base_l, base_r = ctx.orset_batch(P, D), ctx.orset_batch(P, D)
    base_l.fill_synthetic(5, token_slots=3)
    base_r.fill_synthetic(6, token_slots=3)
    W = (D + 63) // 64
    ids = np.arange(D)

    def bits(mask):
        b = np.packbits(mask.astype(np.uint8), bitorder="little")
        return np.concatenate([b, np.zeros((8 * W - len(b),), np.uint8)]).view(np.uint64)
    kl, kr = bits(ids < N), bits(ids >= D - N)
    L = ctx.orset_batch(P, D).filter(base_l, kl)
    Rb = ctx.orset_batch(P, D).filter(base_r, kr)
    del base_l, base_r
    sl, sr = L.stats(), Rb.stats()
    assert (sl[:, 0] == N).all() and (sr[:, 0] == N).all()
    X = L.intersection(Rb)
    # whole batch: exactly the 50k common elements of every pair are kept
    vis = X.value_bits()
    assert all(int(np.unpackbits(vis[i].view(np.uint8)).sum()) <= N - (D - N) for i in (0, P - 1))
    K = 40
    for pair in (0, 401, P - 1):
        for e0 in (0, N - (D - N) - K // 2, N - K // 2, D - K):
            lw = orc.synth_orset_t(5, pair, e0, K, 3)
            rw = orc.synth_orset_t(6, pair, e0, K, 3)
            lo = [x for x in window_orddict(lw, e0) if x[0] < N]
            ro = [x for x in window_orddict(rw, e0) if x[0] >= D - N]
            want = ocore.intersection_body("lasp_orset", lo, ro)
            dom = Domain()
            for e in range(e0, e0 + K):
                dom.element_slot(e)
                for k in range(64):
                    dom.token_slot(e - e0, tok(e, k))
            cells = X.download(pair, 1)[0, e0:e0 + K]
            assert exact_eq(decode_concat(dom, cells), want), (pair, e0)


def test_config5_product_full_size(ctx):
    """BASELINE configs[4] product: 100k x 100k OR-Set elements, T = 3 (10^10 cells, 40 GB
    out); sampled rows x column windows against product_body (X-major pairs, tokens
    orset_causal_product = both runs reversed, [Tx, Ty], Dx orelse Dy)."""
    from lasp_amd.codec import Domain, decode_product
    n = 100_000
    l, r = ctx.orset_batch(1, n), ctx.orset_batch(1, n)
    l.fill_synthetic(7, token_slots=3)
    r.fill_synthetic(8, token_slots=3)
    out = l.product(r)
    cw = 32
    for x in (0, 54_321, n - 1):
        lx = orc.synth_orset_t(7, 0, x, 1, 3)
        for y0 in (0, 77_777, n - cw):
            ry = orc.synth_orset_t(8, 0, y0, cw, 3)
            want = ocore.product_body("lasp_orset", window_orddict(lx, x), window_orddict(ry, y0))
            dl, dr = Domain(), Domain()
            dl.element_slot(x)
            for k in range(64):
                dl.token_slot(0, tok(x, k))
            for y in range(y0, y0 + cw):
                s = dr.element_slot(y)
                for k in range(64):
                    dr.token_slot(s, tok(y, k))
            cells = out.download_range((x * n + y0) * 4, cw * 4).view(np.uint32)
            assert exact_eq(decode_product(dl, dr, cells.reshape(1, cw)), want), (x, y0)


# ----------------------------------------------------------------------------- config 3

def test_config3_round_full_size(ctx):
    """BASELINE configs[2] at one rank of eight: the receive buffer of an 8-GPU round
    (8 chunk-major copies of one rank's 2^17-object chunk, each copy the synthetic
    replica stream of rank j = seed 10 + j) joined by reduce_chunks; sampled objects
    are compared token for token with the C restatement's orddict merge fold
    (lasp_update_fsm.erl:189-192 foldl(merge)); then a full-size one-rank
    laspj_antientropy round (64 GiB) leaves the state unchanged (the join of one copy)."""
    from lasp_amd.engine import Comm
    n, E = 8, 4096
    objs = (1 << 20) // n
    recv = ctx.orset_batch(n * objs, E)
    for j in range(n):
        part = _slice(recv, j * objs, objs)
        part.fill_synthetic(10 + j)
    chunk = ctx.orset_batch(objs, E).reduce_chunks(recv, n)
    tokens = orc.synth_tokens(E)
    for o in (0, 12345, objs - 1):
        acc = orc.ORDict.from_cells(orc.synth_orset(10, o, E), tokens)
        for j in range(1, n):
            acc = acc.merge(orc.ORDict.from_cells(orc.synth_orset(10 + j, o, E), tokens))
        got = orc.ORDict.from_cells(chunk.download(o, 1)[0], tokens)
        assert got.equal(acc), o
    del recv, chunk
    comm = Comm(ctx, 1, Comm.unique_id(), 0)
    st, rv = (ctx.orset_batch(1 << 20, E) for _ in range(2))
    st.fill_synthetic(10)
    comm.antientropy(st, rv)
    ctx.synchronize()
    for o in (0, 654_321, (1 << 20) - 1):
        assert np.array_equal(st.download(o, 1)[0], orc.synth_orset(10, o, E))
    comm.close()


def _slice(batch, first, count):
    """A non-owning OR-Set batch over replicas [first, first + count) of `batch`."""
    return batch.view(first, count)
