"""GPU parity of the HIP engine against the oracle (run with -m gpu on an MI355X).

Every engine result is compared bit-for-bit with the C restatement of the reference
(oracle/laspj_oracle.c: orddict merge, keyfind-based inflation, ...) on seeded
synthetic replicas, decoded token for token where the reference returns terms.
"""

import numpy as np
import pytest

from oracle import columnar as orc

pytestmark = pytest.mark.gpu

E = 256          # element slots per replica in the mid-size cases
R = 512          # replicas per batch in the mid-size cases


@pytest.fixture(scope="module")
def ctx():
    from lasp_amd import engine
    c = engine.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def tokens():
    return orc.synth_tokens(E)


def _synth(seed, n, e, base=0):
    return np.stack([orc.synth_orset(seed, base + i, e) for i in range(n)])


def test_fill_synthetic_matches_oracle(ctx):
    b = ctx.orset_batch(R, E)
    b.fill_synthetic(7, replica_base=1000)
    got = b.download()
    assert np.array_equal(got, _synth(7, R, E, 1000))
    g = ctx.gset_batch(64, 1000)          # E not a multiple of 64: padding bits stay 0
    g.fill_synthetic(9, 5)
    want = np.stack([orc.synth_gset(9, 5 + i, 1000) for i in range(64)])
    assert np.array_equal(g.download(), want)


def test_orset_join_token_for_token(ctx, tokens):
    """lasp_orset:merge/2 (lasp_orset.erl:128-134) vs the C orddict merge."""
    a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    c.join(a, b)
    got = c.download()
    ha, hb = a.download(), b.download()
    for i in range(0, R, 37):
        A = orc.ORDict.from_cells(ha[i], tokens)
        B = orc.ORDict.from_cells(hb[i], tokens)
        M = A.merge(B)
        G = orc.ORDict.from_cells(got[i], tokens)
        assert G.equal(M), f"replica {i}"
    # whole-batch property: the columnar join is p|p', r|r'
    assert np.array_equal(got, ha | hb)


def test_orset_join_in_place_and_idempotent(ctx):
    a, b = ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    want = a.download() | b.download()
    a.join(a, b)                       # bind merges in place (lasp_core.erl:300-303)
    assert np.array_equal(a.download(), want)
    a.join(a, a)                       # idempotence
    assert np.array_equal(a.download(), want)
    a.join(a, b)                       # absorbing
    assert np.array_equal(a.download(), want)


def test_orset_join_edge_cases(ctx, tokens):
    """empty, identical, disjoint and all-removed replicas (SURVEY.md §8d cfg 2)."""
    n = 4
    host = np.zeros((n, E, 2), dtype=np.uint64)
    other = np.zeros_like(host)
    full = _synth(4, 1, E)[0]
    host[1] = full                                 # identical
    other[1] = full
    host[2, : E // 2] = full[: E // 2]             # disjoint halves
    other[2, E // 2:] = full[E // 2:]
    host[3] = full
    host[3, :, 1] = full[:, 0]                     # all removed
    other[3] = full
    a, b, c = ctx.orset_batch(n, E), ctx.orset_batch(n, E), ctx.orset_batch(n, E)
    a.upload(host)
    b.upload(other)
    c.join(a, b)
    got = c.download()
    for i in range(n):
        M = orc.ORDict.from_cells(host[i], tokens).merge(orc.ORDict.from_cells(other[i], tokens))
        assert orc.ORDict.from_cells(got[i], tokens).equal(M)
    assert not got[0].any()


def test_orset_value_removed_stats(ctx, tokens):
    b = ctx.orset_batch(R, E)
    b.fill_synthetic(11)
    h = b.download()
    vis = b.value_bits()
    rem = b.value_bits(removed=True)
    st = b.stats()
    for i in range(0, R, 29):
        D = orc.ORDict.from_cells(h[i], tokens)
        want_vis = D.value()
        got_vis = np.nonzero(np.unpackbits(vis[i].view(np.uint8), bitorder="little")[:E])[0]
        assert np.array_equal(got_vis, want_vis)
        assert tuple(int(x) for x in st[i]) == D.stats()
        want_rem = [e for e in range(E) if h[i, e, 1] != 0]
        got_rem = np.nonzero(np.unpackbits(rem[i].view(np.uint8), bitorder="little")[:E])[0]
        assert list(got_rem) == want_rem


def test_orset_inflation_vs_keyfind_oracle(ctx, tokens):
    """is_inflation / is_strict_inflation (lasp_lattice.erl:153-161, 235-253)."""
    n = 64
    prev = _synth(21, n, E)
    cur = prev.copy()
    rng = np.random.default_rng(0)
    for i in range(n):
        kind = i % 6
        if kind == 1:       # merge-style inflation
            cur[i] |= _synth(22, 1, E, i)[0]
        elif kind == 2:     # drop a token -> not an inflation
            e = int(np.nonzero(cur[i, :, 0])[0][0])
            low = cur[i, e, 0] & (~cur[i, e, 0] + np.uint64(1))
            cur[i, e, 0] ^= low
            cur[i, e, 1] &= cur[i, e, 0]
        elif kind == 3:     # remove an element (tombstone all) -> strict inflation
            e = int(np.nonzero(cur[i, :, 0])[0][0])
            cur[i, e, 1] = cur[i, e, 0]
        elif kind == 4:     # un-remove only (flags ignored by is_inflation)
            prev[i, :, 1] = prev[i, :, 0]
        elif kind == 5:     # empty prev
            prev[i] = 0
        if i == n - 1:      # empty both
            prev[i] = 0
            cur[i] = 0
        _ = rng
    P, Cb = ctx.orset_batch(n, E), ctx.orset_batch(n, E)
    P.upload(prev)
    Cb.upload(cur)
    infl = Cb.is_inflation_of(P)
    strict = Cb.is_inflation_of(P, strict=True)
    for i in range(n):
        Dp = orc.ORDict.from_cells(prev[i], tokens)
        Dc = orc.ORDict.from_cells(cur[i], tokens)
        assert infl[i] == Dc.is_inflation_of(Dp), i
        assert strict[i] == Dc.is_strict_inflation_of(Dp), i


def test_orset_threshold_broadcast(ctx, tokens):
    """threshold_met with one threshold against many values (prev replicas = 1)."""
    n = 32
    cur = _synth(31, n, E)
    th = cur[0].copy()
    th[:, 1] = 0
    T, Cb = ctx.orset_batch(1, E), ctx.orset_batch(n, E)
    T.upload(th[None])
    Cb.upload(cur)
    got = Cb.is_inflation_of(T)
    Dt = orc.ORDict.from_cells(th, tokens)
    for i in range(n):
        assert got[i] == orc.ORDict.from_cells(cur[i], tokens).is_inflation_of(Dt)


@pytest.mark.parametrize("e_n", [256, 100, 4096])
def test_orset_reduce_all_kernels(ctx, e_n):
    """Every reduce kernel (LASPJ_TUNE_REDUCE_KERNEL 0 flat sweep for power-of-two
    replica lengths, 1 per-replica segments with a compile-time group, 2 generic) for
    groups 2..5 equals the OR over each group of replicas."""
    from lasp_amd._lib import TUNE_REDUCE_KERNEL
    for group in (2, 3, 4, 5):
        ng = 37
        src = ctx.orset_batch(group * ng, e_n)
        src.fill_synthetic(60 + group)
        hs = src.download()
        want = np.bitwise_or.reduce(hs.reshape(ng, group, e_n, 2), axis=1)
        try:
            for knob in (0, 1, 2):
                ctx.set_tuning(TUNE_REDUCE_KERNEL, knob)
                dst = ctx.orset_batch(ng, e_n)
                dst.reduce_from(src, group)
                assert np.array_equal(dst.download(), want), (group, knob)
        finally:
            ctx.set_tuning(TUNE_REDUCE_KERNEL, 0)


@pytest.mark.parametrize("nchunks", [1, 2, 3, 5, 8])
def test_reduce_chunks_every_kind(ctx, nchunks):
    """laspj_batch_reduce_chunks (the anti-entropy reduce of an all-to-all receive
    buffer) is the kind's join over the chunk-major copies:
    OR for OR-Set cells and G-Set words (odd word counts take the 8-byte kernel), the
    per-actor max for riak_dt_gcounter counts."""
    from lasp_amd._lib import TUNE_REDUCE_KERNEL
    rng = np.random.default_rng(100 + nchunks)
    n = 29
    cases = ((ctx.orset_batch, 100, "or"), (ctx.gset_batch, 100, "or"),     # G-Set: 2 words
             (ctx.gset_batch, 64, "or"),                                   # 29 words: odd
             (ctx.gcounter_batch, 7, "max"), (ctx.gcounter_batch, 8, "max"))
    for make, e_n, op in cases:
        src, dst = make(nchunks * n, e_n), make(n, e_n)
        w = src.words_per_replica
        if op == "max":       # small counts so chunks collide, some equal
            hs = rng.integers(0, 5, size=(nchunks * n, w), dtype=np.uint64)
        else:
            hs = rng.integers(0, 2**63, size=(nchunks * n, w), dtype=np.uint64) * np.uint64(2) \
                + rng.integers(0, 2, size=(nchunks * n, w), dtype=np.uint64)
            if make is ctx.gset_batch and e_n % 64:   # padding bits beyond E stay zero
                hs[:, -1] &= np.uint64((1 << (e_n % 64)) - 1)
        src.upload(hs)
        red = np.maximum.reduce if op == "max" else np.bitwise_or.reduce
        want = red(hs.reshape(nchunks, n, w), axis=0)
        try:
            for knob in (0, 2):    # compile-time chunk count / runtime-count loop
                ctx.set_tuning(TUNE_REDUCE_KERNEL, knob)
                dst.clear()
                dst.reduce_chunks(src, nchunks)
                assert np.array_equal(dst.download_words(), want), (make.__name__, e_n, knob)
        finally:
            ctx.set_tuning(TUNE_REDUCE_KERNEL, 0)


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8])
def test_join_n_every_kind(ctx, n):
    """laspj_batch_join_n (foldl(merge, new(), Replies) over separately held batches —
    the FSM's N-way merge, and the kernel the anti-entropy round reduces with, reading
    the rank's own copy in place) is the kind's join over n sources, with dst a fresh
    batch or aliasing any source; G-Set batches of an odd word count included.  Compared
    with numpy's OR / max, and for OR-Sets with the C orddict merge fold."""
    rng = np.random.default_rng(300 + n)
    R_ = 37
    cases = ((ctx.orset_batch, 100, "or"), (ctx.gset_batch, 100, "or"),
             (ctx.gset_batch, 64, "or"),                                   # 37 words: odd
             (ctx.gcounter_batch, 7, "max"))
    for make, e_n, op in cases:
        srcs = [make(R_, e_n) for _ in range(n)]
        w = srcs[0].words_per_replica
        hs = []
        for b in srcs:
            if op == "max":
                h = rng.integers(0, 5, size=(R_, w), dtype=np.uint64)
            else:
                h = rng.integers(0, 2**63, size=(R_, w), dtype=np.uint64) * np.uint64(2) \
                    + rng.integers(0, 2, size=(R_, w), dtype=np.uint64)
                if make is ctx.orset_batch:
                    h[:, 1::2] &= h[:, 0::2]                  # r within p
                if make is ctx.gset_batch and e_n % 64:
                    h[:, -1] &= np.uint64((1 << (e_n % 64)) - 1)
            b.upload(h)
            hs.append(h)
        red = np.maximum.reduce if op == "max" else np.bitwise_or.reduce
        want = red(np.stack(hs), axis=0)
        dst = make(R_, e_n)
        dst.join_n(srcs)
        assert np.array_equal(dst.download_words(), want), (make.__name__, e_n)
        k = n // 2                                   # in place into one of the sources
        srcs[k].join_n(srcs)
        assert np.array_equal(srcs[k].download_words(), want), (make.__name__, e_n, "alias")
    # OR-Set: the fold of the reference merge over the n replies, token for token
    tokens = orc.synth_tokens(64)
    bs = [ctx.orset_batch(9, 64) for _ in range(n)]
    for j, b in enumerate(bs):
        b.fill_synthetic(40 + j)
    dst = ctx.orset_batch(9, 64).join_n(bs)
    got = dst.download()
    for i in range(9):
        acc = orc.ORDict.from_cells(np.zeros((64, 2), np.uint64), tokens)
        for j in range(n):
            acc = acc.merge(orc.ORDict.from_cells(orc.synth_orset(40 + j, i, 64), tokens))
        assert orc.ORDict.from_cells(got[i], tokens).equal(acc), i


def test_join_n_errors(ctx):
    from lasp_amd._lib import LaspjError
    a, b = ctx.orset_batch(4, 64), ctx.orset_batch(4, 65)
    g = ctx.gset_batch(4, 64)
    for bad in ([a, b], [a, g], [], [a] * 9):
        with pytest.raises(LaspjError):
            ctx.orset_batch(4, 64).join_n(bad)


def test_batch_join_gcounter_is_max(ctx):
    """laspj_batch_join on G-Counter batches is riak_dt_gcounter's merge (per-actor max,
    the same as laspj_gcounter_join), not a bitwise OR of the counts."""
    rng = np.random.default_rng(7)
    a, b, c, d = (ctx.gcounter_batch(33, 9) for _ in range(4))
    ha = rng.integers(0, 6, size=(33, 9), dtype=np.uint64)
    hb = rng.integers(0, 6, size=(33, 9), dtype=np.uint64)
    a.upload(ha)
    b.upload(hb)
    L = ctx.L
    from lasp_amd._lib import check
    check(L.laspj_batch_join(ctx.h, c.h, a.h, b.h), ctx.h)
    d.join(a, b)
    assert np.array_equal(c.download(), np.maximum(ha, hb))
    assert np.array_equal(d.download(), c.download())


def test_orset_equal(ctx):
    a, b = ctx.orset_batch(8, E), ctx.orset_batch(8, E)
    a.fill_synthetic(5)
    b.fill_synthetic(5)
    h = b.download()
    h[3, 7, 1] ^= np.uint64(1) << np.uint64(63)
    b.upload(h)
    eq = a.equal(b)
    assert list(eq) == [True, True, True, False, True, True, True, True]


def test_orset_reduce_fsm_merge(ctx, tokens):
    """foldl(merge, new(), Replies) — lasp_update_fsm.erl:189-192, N=3."""
    groups, N = 50, 3
    src, dst = ctx.orset_batch(groups * N, E), ctx.orset_batch(groups, E)
    src.fill_synthetic(41)
    dst.reduce_from(src, N)
    hs = src.download()
    got = dst.download()
    for g in range(0, groups, 7):
        acc = orc.ORDict.from_cells(np.zeros((E, 2), np.uint64), tokens)
        for j in range(N):
            acc = orc.ORDict.from_cells(hs[g * N + j], tokens).merge(acc)
        assert orc.ORDict.from_cells(got[g], tokens).equal(acc)


def test_orset_apply_ops_vs_python_oracle(ctx):
    """update/3 add_by_token / remove / {update, Ops} (lasp_orset.erl:99-117)."""
    from lasp_amd._lib import OP_ADD, OP_REMOVE, OP_FLAG_NEW_CALL, OPST_APPLIED, \
        OPST_NOT_PRESENT, OPST_ROLLED_BACK
    from oracle import orset as oo
    e_n = 8
    toks = [bytes([k]) * 20 for k in range(64)]
    b = ctx.orset_batch(3, e_n)
    # replica 0: add e1/t3, add e1/t5, remove e1 (one call each), add e1/t3 again
    # replica 1: call {update, [add e2/t0, remove e4]} -> rolled back (e4 absent)
    # replica 2: call {update, [add e4/t1, remove e4]} -> ok (added earlier in call)
    ops = [(0, 1, OP_ADD, 3, OP_FLAG_NEW_CALL), (0, 1, OP_ADD, 5, OP_FLAG_NEW_CALL),
           (0, 1, OP_REMOVE, 0, OP_FLAG_NEW_CALL), (0, 1, OP_ADD, 3, OP_FLAG_NEW_CALL),
           (1, 2, OP_ADD, 0, OP_FLAG_NEW_CALL), (1, 4, OP_REMOVE, 0, 0),
           (2, 4, OP_ADD, 1, OP_FLAG_NEW_CALL), (2, 4, OP_REMOVE, 0, 0)]
    st = b.apply_ops(ops)
    assert list(st) == [OPST_APPLIED] * 4 + [OPST_ROLLED_BACK, OPST_NOT_PRESENT] + [OPST_APPLIED] * 2
    got = b.download()
    # oracle
    s0 = oo.new()
    for op in [("add_by_token", toks[3], 1), ("add_by_token", toks[5], 1), ("remove", 1),
               ("add_by_token", toks[3], 1)]:
        s0 = oo.update(op, None, s0)[1]
    assert oo.update(("update", [("add_by_token", toks[0], 2), ("remove", 4)]), None, [])[0] == "error"
    s2 = oo.update(("update", [("add_by_token", toks[1], 4), ("remove", 4)]), None, [])[1]

    def enc(s):
        out = np.zeros((e_n, 2), np.uint64)
        for elem, tl in s:
            for t, rm in tl:
                k = toks.index(t)
                out[elem, 0] |= np.uint64(1) << np.uint64(k)
                if rm:
                    out[elem, 1] |= np.uint64(1) << np.uint64(k)
        return out
    assert np.array_equal(got[0], enc(s0))
    assert not got[1].any()
    assert np.array_equal(got[2], enc(s2))


def test_orset_union_filter_vs_bodies(ctx):
    """union (lasp_core.erl:616-618) and filter (:681-712) bodies."""
    from oracle import core
    e_n = 70
    toks = [bytes([k]) * 20 for k in range(64)]
    l = _synth(51, 4, e_n)
    r = _synth(52, 4, e_n)
    l[:, ::3] = 0              # some elements only on the right

    def dec(cells):
        out = []
        for e in range(e_n):
            p, rr = int(cells[e, 0]), int(cells[e, 1])
            if p:
                out.append((e, [(toks[k], bool((rr >> k) & 1)) for k in range(64) if (p >> k) & 1]))
        return out
    L, Rb, U, F = (ctx.orset_batch(4, e_n) for _ in range(4))
    L.upload(l)
    Rb.upload(r)
    U.union(L, Rb)
    keep = np.zeros(((e_n + 63) // 64,), np.uint64)
    for e in range(e_n):
        if e % 2 == 0:
            keep[e // 64] |= np.uint64(1) << np.uint64(e % 64)
    F.filter(L, keep)
    gu, gf = U.download(), F.download()
    for i in range(4):
        assert dec(gu[i]) == core.union_body("lasp_orset", dec(l[i]), dec(r[i]))
        assert dec(gf[i]) == core.filter_body("lasp_orset", lambda x: x % 2 == 0, dec(l[i]))


def test_gset_join_inflation_stats(ctx):
    n, e_n = 128, 1000
    a, b, c = (ctx.gset_batch(n, e_n) for _ in range(3))
    a.fill_synthetic(61)
    b.fill_synthetic(62)
    c.join(a, b)
    ha, hb, hc = a.download(), b.download(), c.download()
    for i in range(0, n, 13):
        want = orc.gset_merge(ha[i], hb[i], e_n)
        assert np.array_equal(orc.gset_members(hc[i], e_n), want)
    assert np.array_equal(c.stats(), np.array([len(orc.gset_members(x, e_n)) for x in hc]))
    assert c.is_inflation_of(a).all()
    assert c.is_inflation_of(a, strict=True).all()
    assert not c.is_inflation_of(c, strict=True).any()
    assert c.is_inflation_of(c).all()
    assert c.equal(c).all()


def test_large_join_property(ctx):
    """A 4 GiB-per-operand batch (2^16 replicas x 4096 elements): join equals p|p' on
    sampled replicas regenerated by the oracle, and the join is idempotent."""
    n, e_n = 1 << 16, 4096
    a, b, c = (ctx.orset_batch(n, e_n) for _ in range(3))
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    c.join(a, b)
    for i in (0, 1, 12345, n - 1):
        got = c.download(i, 1)[0]
        want = orc.synth_orset(2, i, e_n) | orc.synth_orset(3, i, e_n)
        assert np.array_equal(got, want)
    assert c.equal(c).all()
    d = ctx.orset_batch(n, e_n)
    d.join(c, a)
    assert d.equal(c).all()


def test_full_size_join_properties(ctx):
    """BASELINE config 2 at its full size (2^20 replicas x 4096 elements x 64 token
    slots, 3 x 64 GiB resident): sampled replicas on both sides of every 4 GiB / 32-bit
    boundary equal lasp_orset:merge/2 of the oracle's orddicts token for token (value,
    stats and inflation too); over the whole batch the join is commutative (B ⊔ A in
    place equals A ⊔ B), idempotent and an inflation of both inputs."""
    n, e_n = 1 << 20, 4096
    toks = orc.synth_tokens(e_n)
    a, b, c = (ctx.orset_batch(n, e_n) for _ in range(3))
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    c.join(a, b)
    assert c.is_inflation_of(a).all() and c.is_inflation_of(b).all()
    vis = c.value_bits()
    st = c.stats()
    for i in (0, 1, (1 << 16) - 1, 1 << 16, 699_051, n - 1):
        A = orc.ORDict.from_cells(orc.synth_orset(2, i, e_n), toks)
        B = orc.ORDict.from_cells(orc.synth_orset(3, i, e_n), toks)
        M = A.merge(B)
        assert orc.ORDict.from_cells(c.download(i, 1)[0], toks).equal(M), f"replica {i}"
        bits = np.unpackbits(vis[i].view(np.uint8), bitorder="little")[:e_n]
        assert np.array_equal(np.nonzero(bits)[0], M.value()), f"value/1 of replica {i}"
        assert tuple(int(x) for x in st[i]) == M.stats(), f"stats/1 of replica {i}"
    b.join(b, a)                                     # in place, operands swapped
    assert b.equal(c).all()
    b.join(b, b)
    assert b.equal(c).all()
    assert not c.is_inflation_of(b, strict=True).any()


def test_orset_product_tiles_and_tails(ctx):
    """Outer-product tiling: EL and ER off the 32..256 x 1024 tiles, several replicas; every
    cell equals {pX8, rX8, pY8, rY8} of its row / column (0 where either is absent)."""
    n, el, er = 3, 130, 1027
    l = _synth(71, n, el)
    r = _synth(72, n, er)
    l &= np.uint64(0x7)          # 3 token slots, as in BASELINE config 5
    r &= np.uint64(0x7)
    L, Rb = ctx.orset_batch(n, el), ctx.orset_batch(n, er)
    L.upload(l)
    Rb.upload(r)
    from lasp_amd._lib import TUNE_PRODUCT_COLS, TUNE_PRODUCT_ROWS
    outs = []
    try:
        for rows, cols in ((32, 0), (64, 2048), (128, 4096), (256, 2048), (0, 0)):
            ctx.set_tuning(TUNE_PRODUCT_ROWS, rows)  # every tile shape; default last
            ctx.set_tuning(TUNE_PRODUCT_COLS, cols)
            P = L.product(Rb)
            outs.append(P.download())
    finally:
        ctx.set_tuning(TUNE_PRODUCT_ROWS, 0)
        ctx.set_tuning(TUNE_PRODUCT_COLS, 0)
    got = outs[-1]
    for o in outs[:-1]:
        assert np.array_equal(o, got)
    lx = np.where(l[:, :, 0] != 0, l[:, :, 0] | (l[:, :, 1] << np.uint64(8)), 0).astype(np.uint32)
    ry = np.where(r[:, :, 0] != 0, (r[:, :, 0] << np.uint64(16)) | (r[:, :, 1] << np.uint64(24)), 0
                  ).astype(np.uint32)
    want = np.where((lx[:, :, None] != 0) & (ry[:, None, :] != 0),
                    lx[:, :, None] | ry[:, None, :], 0).astype(np.uint32)
    assert np.array_equal(got, want)
    vis = P.value_bits()
    live_l = (l[:, :, 0] & ~l[:, :, 1]) != 0
    live_r = (r[:, :, 0] & ~r[:, :, 1]) != 0
    want_vis = (live_l[:, :, None] & live_r[:, None, :]).reshape(n, -1)
    bits = np.unpackbits(vis.view(np.uint8), axis=1, bitorder="little")[:, : el * er].astype(bool)
    assert np.array_equal(bits, want_vis)


def test_orset_product_rejects_wide_token_slots(ctx):
    from lasp_amd import LaspjError
    from lasp_amd._lib import E_RANGE
    L, Rb = ctx.orset_batch(1, 4), ctx.orset_batch(1, 4)
    h = np.zeros((1, 4, 2), np.uint64)
    h[0, 1, 0] = np.uint64(1) << np.uint64(9)      # token slot 9
    L.upload(h)
    Rb.upload(h)
    with pytest.raises(LaspjError) as ei:
        L.product(Rb, wide=False)              # 4-byte cells requested explicitly
    assert ei.value.status == E_RANGE
    assert type(L.product(Rb)).__name__ == "ORSetProductWideBatch"   # automatic choice


def test_orset_intersection_concat(ctx):
    l, r = _synth(81, 8, E), _synth(82, 8, E)
    L, Rb = ctx.orset_batch(8, E), ctx.orset_batch(8, E)
    L.upload(l)
    Rb.upload(r)
    got = L.intersection(Rb).download()
    keep = (l[:, :, 0] != 0) & (r[:, :, 0] != 0)
    want = np.concatenate([l, r], axis=2) * keep[:, :, None].astype(np.uint64)
    assert np.array_equal(got, want)


def test_gset_combinators(ctx):
    """G-Set intersection / filter / product / gather bodies vs oracle lists.  (The G-Set
    union body is `L ++ R`, a list value: tests/test_gpu_lists.py compares it with
    union_body on unsorted and overlapping lists, test_store_random re-binds it.)"""
    from oracle import core
    n, e_n = 4, 150
    a = np.stack([orc.synth_gset(91, i, e_n) for i in range(n)])
    b = np.stack([orc.synth_gset(92, i, e_n) for i in range(n)])
    A, B = ctx.gset_batch(n, e_n), ctx.gset_batch(n, e_n)
    A.upload(a)
    B.upload(b)
    mem = lambda w: [int(x) for x in orc.gset_members(w, e_n)]   # noqa: E731
    I = ctx.gset_batch(n, e_n).intersection(A, B).download()
    keep = np.zeros(((e_n + 63) // 64,), np.uint64)
    for e in range(0, e_n, 3):
        keep[e // 64] |= np.uint64(1) << np.uint64(e % 64)
    Fl = ctx.gset_batch(n, e_n).filter(A, keep).download()
    P = A.product(B).download()
    idx = np.array([e // 2 for e in range(e_n)], np.uint32)          # a map onto slots
    G = ctx.gset_batch(n, e_n).gather(A, idx).download()
    for i in range(n):
        la, lb = mem(a[i]), mem(b[i])
        assert mem(I[i]) == core.intersection_body("lasp_gset", la, lb)
        assert mem(Fl[i]) == core.filter_body("lasp_gset", lambda x: x % 3 == 0, la)
        pairs = [(x, y) for x in range(e_n) for y in range(e_n)
                 if (int(P[i, x, y >> 6]) >> (y & 63)) & 1]
        assert pairs == core.product_body("lasp_gset", la, lb)
        got_g = [o for o in range(e_n) if (int(G[i, o >> 6]) >> (o & 63)) & 1]
        assert got_g == [o for o in range(e_n) if (o // 2) in set(la)]


def test_segmented_reductions_long_replicas(ctx):
    """Replicas longer than one 4096-cell segment (config 4 shape, scaled down): stats,
    equal and (strict) inflation combine per-segment partials exactly."""
    n, e_n = 5, 10_000
    tok = orc.synth_tokens(e_n, 64)
    prev = _synth(101, n, e_n)
    cur = prev.copy()
    cur[1, 9_000, 1] = cur[1, 9_000, 0]              # tombstone far in the last segment
    cur[2, 5_000, 0] = 0                             # drop an element: not an inflation
    cur[2, 5_000, 1] = 0
    cur[3] |= _synth(102, 1, e_n)[0]                 # strict growth
    P, Cb = ctx.orset_batch(n, e_n), ctx.orset_batch(n, e_n)
    P.upload(prev)
    Cb.upload(cur)
    st = Cb.stats()
    eq = Cb.equal(P)
    infl = Cb.is_inflation_of(P)
    strict = Cb.is_inflation_of(P, strict=True)
    for i in range(n):
        Dp, Dc = orc.ORDict.from_cells(prev[i], tok), orc.ORDict.from_cells(cur[i], tok)
        assert tuple(int(x) for x in st[i]) == Dc.stats()
        assert eq[i] == Dc.equal(Dp)
        assert infl[i] == Dc.is_inflation_of(Dp)
        assert strict[i] == Dc.is_strict_inflation_of(Dp)
    # G-Set with more than 4096 words per replica
    g_e = 300_000
    ga, gb = ctx.gset_batch(3, g_e), ctx.gset_batch(3, g_e)
    ga.fill_synthetic(7)
    h = ga.download()
    h2 = h.copy()
    h2[0, 4_500] |= np.uint64(1) << np.uint64(3) if not (h[0, 4_500] >> np.uint64(3)) & np.uint64(1) else np.uint64(0)
    h2[1, 4_600] = 0
    gb.upload(h2)
    assert list(gb.stats()) == [sum(bin(int(w)).count("1") for w in row) for row in h2]
    eqg = gb.equal(ga)
    ig = gb.is_inflation_of(ga)
    sg = gb.is_inflation_of(ga, strict=True)
    for i in range(3):
        sub = not np.any(h[i] & ~h2[i])
        same = np.array_equal(h[i], h2[i])
        assert eqg[i] == same and ig[i] == sub and sg[i] == (sub and not same)


def test_ticketed_reductions_small_batches(ctx):
    """Few replicas, long rows: segments shrink (thousands of waves) and every
    replica's result is produced by its last-arriving segment (a ticket in the
    per-replica record, which it zeroes again) — checked over repeated launches so a
    record left dirty would show; value/1 of a single 20k-slot replica."""
    n, e_n = 3, 20_000
    prev = _synth(111, n, e_n)
    cur = prev | _synth(112, n, e_n)
    cur[1, 19_999, 0] = 0                            # drop an element: not an inflation
    cur[1, 19_999, 1] = 0
    P, Cb = ctx.orset_batch(n, e_n), ctx.orset_batch(n, e_n)
    P.upload(prev)
    Cb.upload(cur)
    tok = orc.synth_tokens(e_n, 64)
    want_i = [orc.ORDict.from_cells(cur[i], tok).is_inflation_of(orc.ORDict.from_cells(prev[i], tok))
              for i in range(n)]
    want_s = [orc.ORDict.from_cells(cur[i], tok).is_strict_inflation_of(
        orc.ORDict.from_cells(prev[i], tok)) for i in range(n)]
    want_st = [orc.ORDict.from_cells(cur[i], tok).stats() for i in range(n)]
    for _ in range(4):
        assert [tuple(int(x) for x in r) for r in Cb.stats()] == want_st
        assert list(Cb.is_inflation_of(P)) == want_i
        assert list(Cb.is_inflation_of(P, strict=True)) == want_s
        assert list(Cb.equal(P)) == [False] * n
        assert list(Cb.equal(Cb)) == [True] * n
    one = ctx.orset_batch(1, e_n)
    one.upload(cur[:1])
    bits = np.unpackbits(one.value_bits()[0].view(np.uint8), bitorder="little")[:e_n]
    live = (cur[0, :, 0] & ~cur[0, :, 1]) != 0
    assert np.array_equal(bits.astype(bool), live)
    # G-Counter: 3 replicas x 10k actors, threshold and inflation over tickets
    g = ctx.gcounter_batch(3, 10_000)
    rng = np.random.default_rng(9)
    hc = rng.integers(0, 1000, (3, 10_000)).astype(np.uint64)
    hc[0, 5] = 7
    g.upload(hc)
    sums = hc.sum(axis=1)
    for _ in range(3):
        assert np.array_equal(g.values(), sums)
        gs = ctx.gset_batch(2, 640_000)
        gs.fill_synthetic(13)
        assert list(gs.stats()) == [sum(bin(int(w)).count("1") for w in row)
                                    for row in gs.download()]
        for t in (int(sums[0]), int(sums[1]) + 1, 0):
            assert list(g.threshold_met(t)) == [t <= int(x) for x in sums]
            assert list(g.threshold_met(t, strict=True)) == [t < int(x) for x in sums]
    g2 = ctx.gcounter_batch(3, 10_000)
    h2 = hc.copy()
    h2[2, 9_999] += np.uint64(1)
    h2[0, 5] = 0
    g2.upload(h2)
    assert list(g2.is_inflation_of(g)) == [False, True, True]
    assert list(g2.is_inflation_of(g, strict=True)) == [False, False, True]


def test_segmented_reductions_large_launch(ctx):
    """More segment items than the ticket limit (5000 replicas x 2 segments): partial
    records are finished by the finalize kernel, which also re-zeroes them — repeated,
    interleaved with ticketed small launches, against numpy restatements of the
    columnar predicates (lasp_lattice.erl:153-161, 235-253; stat/2)."""
    n, e_n = 5000, 5000
    P, Cb = ctx.orset_batch(n, e_n), ctx.orset_batch(n, e_n)
    P.fill_synthetic(121)
    prev = P.download()
    cur = prev.copy()
    cur[::3] |= _synth(122, 1, e_n)[0]                       # growth
    cur[1::7, 4_999, 0] = 0                                  # drop the last element
    cur[1::7, 4_999, 1] = 0
    cur[2::11, 10, 1] = cur[2::11, 10, 0]                    # tombstone
    Cb.upload(cur)
    pp, rp, pc, rc = prev[..., 0], prev[..., 1], cur[..., 0], cur[..., 1]
    viol = ((pp & ~pc) != 0).any(axis=1)
    changed = ((pp != 0) & (pc != 0) & ((pp != pc) | (rp != rc))).any(axis=1)
    npres, ncres = (pp != 0).sum(axis=1), (pc != 0).sum(axis=1)
    want_i = ~viol
    want_s = ~viol & (changed | (npres < ncres))
    want_s |= (npres == 0) & (ncres != 0)
    want_st = np.stack([(pc != 0).sum(axis=1),
                        np.bitwise_count(pc & ~rc).sum(axis=1, dtype=np.int64),
                        np.bitwise_count(rc).sum(axis=1, dtype=np.int64)], axis=1)
    want_eq = (prev == cur).all(axis=(1, 2))
    small = ctx.orset_batch(1, 20_000)
    small.fill_synthetic(5)
    for _ in range(3):
        assert np.array_equal(Cb.is_inflation_of(P), want_i)
        assert np.array_equal(Cb.is_inflation_of(P, strict=True), want_s)
        assert np.array_equal(Cb.equal(P), want_eq)
        assert np.array_equal(Cb.stats().astype(np.int64), want_st)
        assert small.is_inflation_of(small).all() and small.equal(small).all()


def test_gcounter_synthetic_join_value(ctx):
    """Synthetic G-Counter batches (bench data): deterministic, 20-bit counts; the
    join is the per-actor max and value/1 the sum (riak_dt_gcounter merge / value)."""
    a, b, c = (ctx.gcounter_batch(300, 1000) for _ in range(3))
    a.fill_synthetic(5)
    b.fill_synthetic(6)
    ha, hb = a.download(), b.download()
    a.fill_synthetic(5)
    assert np.array_equal(a.download(), ha)
    assert ha.max() < (1 << 20) and not np.array_equal(ha, hb)
    c.join(a, b)
    assert np.array_equal(c.download(), np.maximum(ha, hb))
    assert np.array_equal(c.values(), np.maximum(ha, hb).sum(axis=1))


def test_gcounter_batch_kernels(ctx):
    """riak_dt_gcounter join (per-actor max), value (sum), threshold, inflation, FSM
    reduce, increments — against the oracle's _GCounter restatement."""
    from oracle import core as oc
    from oracle import lattice as ol
    rng = np.random.default_rng(3)
    n, actors = 40, 5000           # > one 4096-word segment per replica
    a = rng.integers(0, 4, (n, actors)).astype(np.uint64) * (rng.random((n, actors)) < 0.3)
    b = rng.integers(0, 4, (n, actors)).astype(np.uint64) * (rng.random((n, actors)) < 0.3)
    b[5] = a[5]
    b[6] = a[6] + np.uint64(1)
    A, B, Cc = (ctx.gcounter_batch(n, actors) for _ in range(3))
    A.upload(a.astype(np.uint64))
    B.upload(b.astype(np.uint64))
    Cc.join(A, B)
    assert np.array_equal(Cc.download(), np.maximum(a, b))
    assert np.array_equal(A.values(), a.sum(axis=1))
    t = int(np.median(a.sum(axis=1)))
    assert list(A.threshold_met(t)) == [t <= int(x) for x in a.sum(axis=1)]
    assert list(A.threshold_met(t, strict=True)) == [t < int(x) for x in a.sum(axis=1)]
    od = lambda row: [(k, int(v)) for k, v in enumerate(row) if v]     # noqa: E731
    infl = B.is_inflation_of(A)
    strict = B.is_inflation_of(A, strict=True)
    for i in range(n):
        assert infl[i] == ol.is_inflation("riak_dt_gcounter", od(a[i]), od(b[i]))
        assert strict[i] == ol.is_strict_inflation("riak_dt_gcounter", od(a[i]), od(b[i]))
        assert oc._GCounter.merge(od(a[i]), od(b[i])) == od(np.maximum(a[i], b[i]))
    assert list(B.equal(A)) == [bool(np.array_equal(a[i], b[i])) for i in range(n)]
    G = ctx.gcounter_batch(n // 4, actors).reduce_from(A, 4)
    assert np.array_equal(G.download(), a.reshape(n // 4, 4, actors).max(axis=1))
    A.increment([(0, 3, 7), (0, 3, 1), (39, 4999, 2)])
    h = A.download()
    assert h[0, 3] == a[0, 3] + 8 and h[39, 4999] == a[39, 4999] + 2


@pytest.mark.parametrize("actors", [2, 64, 1024, 5000, 7])
def test_gcounter_reduce_all_kernels(ctx, actors):
    """The G-Counter FSM reduce (per-actor max over each group) for groups 2..5: the
    flat sweep (power-of-two actor pairs, group <= 4) and the generic kernel
    (LASPJ_TUNE_REDUCE_KERNEL 2, odd actor counts, group 5) agree with numpy."""
    from lasp_amd._lib import TUNE_REDUCE_KERNEL
    rng = np.random.default_rng(actors)
    ng = 37
    for group in (2, 3, 4, 5):
        a = rng.integers(0, 6, (group * ng, actors), dtype=np.uint64)
        a[::7] = np.uint64(2**64 - 1) - a[::7]        # counts above 2^63: unsigned max
        src = ctx.gcounter_batch(group * ng, actors)
        src.upload(a)
        want = a.reshape(ng, group, actors).max(axis=1)
        try:
            for knob in (0, 2):
                ctx.set_tuning(TUNE_REDUCE_KERNEL, knob)
                got = ctx.gcounter_batch(ng, actors).reduce_from(src, group).download()
                assert np.array_equal(got, want), (group, knob)
        finally:
            ctx.set_tuning(TUNE_REDUCE_KERNEL, 0)


def test_abi_error_behaviour(ctx):
    """Shape / kind / range violations come back as status codes with a message and
    leave the batches untouched (the NIF turns them into badarg, which bind swallows:
    lasp_core.erl:308-311); precondition failures come back per op."""
    from lasp_amd import LaspjError
    from lasp_amd import _lib
    L = ctx.L
    a, b = ctx.orset_batch(4, 64), ctx.orset_batch(4, 65)
    g = ctx.gset_batch(4, 64)
    a.fill_synthetic(1)
    before = a.download()
    with pytest.raises(LaspjError) as e:
        a.join(a, b)
    assert e.value.status == _lib.E_SHAPE and "shapes differ" in str(e.value)
    assert L.laspj_orset_join(ctx.h, a.h, a.h, g.h) == _lib.E_KIND
    small = ctx.buffer(3)
    assert L.laspj_orset_equal(ctx.h, a.h, a.h, small.h) == _lib.E_RANGE
    assert L.laspj_orset_reduce(ctx.h, a.h, a.h, 2) == _lib.E_SHAPE
    with pytest.raises(LaspjError) as e:
        a.apply_ops([(9, 0, _lib.OP_ADD, 0, 1)])                  # replica out of range
    assert e.value.status == _lib.E_RANGE
    with pytest.raises(LaspjError):
        a.apply_ops([(2, 0, _lib.OP_ADD, 0, 1), (1, 0, _lib.OP_ADD, 0, 1)])   # unsorted
    with pytest.raises(LaspjError):
        g.apply_ops([(0, 1, _lib.OP_REMOVE, 0, 1)])               # no remove on a G-Set
    assert np.array_equal(a.download(), before)
    assert a.upload(before[:2], first=3) is None if False else True
    with pytest.raises(LaspjError) as e:
        a.upload(before[:2], first=3)                              # replicas 3..4 of 4
    assert e.value.status == _lib.E_RANGE
    # the context stays usable after errors
    c = ctx.orset_batch(4, 64)
    c.join(a, a)
    assert np.array_equal(c.download(), before)


def test_orset_product_wide_any_token_slots(ctx, tokens):
    """Elements with token slots >= 8 take the 32-byte product form automatically; the
    decoded list equals the oracle's product body (descending [Tx, Ty] pairs)."""
    from oracle import core
    from lasp_amd.codec import Domain, decode_product
    toks = [bytes([k]) * 20 for k in range(64)]
    l = [(1, [(toks[k], k % 3 == 0) for k in (0, 9, 40)]), (2, [(toks[5], False)])]
    r = [(7, [(toks[k], False) for k in (2, 63)]), (8, [(toks[11], True)])]
    dl, dr = Domain(), Domain()
    dl.register_orset(l)
    dr.register_orset(r)
    L, Rb = ctx.orset_batch(1, 2), ctx.orset_batch(1, 2)
    L.upload(dl.encode_orset([l], 2))
    Rb.upload(dr.encode_orset([r], 2))
    P = L.product(Rb)
    assert type(P).__name__ == "ORSetProductBatch"          # slots here are < 8
    got = decode_product(dl, dr, P.download()[0])
    assert got == core.product_body("lasp_orset", l, r)
    # now slots beyond 8: cells spread over 64 token slots
    h = np.zeros((1, 2, 2), np.uint64)
    h[0, 0, 0] = np.uint64((1 << 9) | (1 << 40) | 1)
    h[0, 0, 1] = np.uint64(1)
    h[0, 1, 0] = np.uint64(1 << 63)
    L.upload(h)
    P = L.product(Rb)
    assert type(P).__name__ == "ORSetProductWideBatch"
    cells = P.download()[0]
    rr = Rb.download()[0]
    for x in range(2):
        for y in range(2):
            assert list(cells[x, y]) == [int(h[0, x, 0]), int(h[0, x, 1]), int(rr[y, 0]), int(rr[y, 1])]
    vis = P.value_bits()[0]
    # visible: x live in both rows; y = 0 live, y = 1 all tombstoned -> cells 0 and 2
    assert int(vis[0]) & 0xF == 0b0101


def test_orset_product_wide_tiles(ctx):
    """32-byte product over 1024-column tiles: 3 replicas x 37 rows x 2500 columns
    (a tail tile, absent rows and columns): every cell is {pX, rX, pY, rY} or 0."""
    n, el, er = 3, 37, 2500
    l, r = _synth(131, n, el), _synth(132, n, er)
    L, Rb = ctx.orset_batch(n, el), ctx.orset_batch(n, er)
    L.upload(l)
    Rb.upload(r)
    P = L.product(Rb)
    assert type(P).__name__ == "ORSetProductWideBatch"
    got = P.download()
    keep = (l[:, :, None, 0] != 0) & (r[:, None, :, 0] != 0)
    want = np.concatenate([np.broadcast_to(l[:, :, None, :], (n, el, er, 2)),
                           np.broadcast_to(r[:, None, :, :], (n, el, er, 2))], axis=3)
    want = np.where(keep[..., None], want, np.uint64(0))
    assert np.array_equal(got.reshape(n, el, er, 4), want)


def test_concurrent_callers_one_context(ctx):
    """Re-entrancy (vnodes call merge concurrently from many BEAM
    schedulers): 8 host threads share one context, each joining / counting / checking
    inflation on its own batches in a loop (ctypes drops the GIL in every call); every
    result equals the single-threaded one."""
    import threading
    n, e_n, T, iters = 64, 512, 8, 25
    jobs = []
    for t in range(T):
        a, b, c = (ctx.orset_batch(n, e_n) for _ in range(3))
        a.fill_synthetic(200 + t)
        b.fill_synthetic(300 + t)
        c.join(a, b)
        jobs.append((a, b, c, c.download(), c.stats(), c.value_bits()))
    errors = []

    def work(t):
        a, b, c, want, st, vis = jobs[t]
        try:
            for _ in range(iters):
                c.join(a, b)
                if not np.array_equal(c.stats(), st):
                    errors.append((t, "stats"))
                if not c.is_inflation_of(a).all() or not c.is_inflation_of(b).all():
                    errors.append((t, "inflation"))
                if not np.array_equal(c.value_bits(), vis):
                    errors.append((t, "value"))
            if not np.array_equal(c.download(), want):
                errors.append((t, "join"))
        except Exception as e:                      # surfaced below
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(T)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors[:5]


def test_orset_product_diag_matches_product_then_filter(ctx):
    """laspj_orset_product_diag = the product body followed by the filter body with
    fun({X, Y}) -> X =:= Y (lasp_core.erl:499-533, 681-712) on the oracle: random
    OR-Sets over one dictionary (<= 3 token slots per element, tombstones kept), several
    replica pairs; the host decode of each replica's diagonal equals the oracle list."""
    import random
    from lasp_amd.codec import Domain, decode_product_diag
    from lasp_amd.terms import Atom
    from oracle import core, orset
    rng = random.Random(91)
    elems = list(range(0, 60, 3)) + [Atom("a"), Atom("zz"), 1 << 40]
    pool = {i: [bytes([i % 251, k]) * 10 for k in range(3)] for i in range(len(elems))}

    def rand_set(seed):
        toks = iter([t for i in range(len(elems)) for t in pool[i]])
        s = orset.new()
        for i in rng.sample(range(len(elems)), rng.randint(0, len(elems))):
            for t in rng.sample(pool[i], rng.randint(1, 3)):
                s = orset.update(("add_by_token", t, elems[i]), None, s)[1]
            if rng.random() < 0.3:
                s = orset.update(("remove", elems[i]), None, s)[1]
        return s
    pairs = [(rand_set(2 * k), rand_set(2 * k + 1)) for k in range(6)]
    dom = Domain()
    for a, b in pairs:
        dom.register_orset(a)
        dom.register_orset(b)
    E = dom.size + 3
    L, Rb = ctx.orset_batch(len(pairs), E), ctx.orset_batch(len(pairs), E)
    L.upload(dom.encode_orset([a for a, _ in pairs], E))
    Rb.upload(dom.encode_orset([b for _, b in pairs], E))
    D = L.product_diag(Rb)
    cells = D.download().reshape(len(pairs), E, 1)
    same = lambda xy: xy[0] == xy[1] and type(xy[0]) is type(xy[1])   # noqa: E731  (=:=)
    for k, (a, b) in enumerate(pairs):
        want = core.filter_body("lasp_orset", same, core.product_body("lasp_orset", a, b))
        assert decode_product_diag(dom, cells[k]) == want, k
    # shape / kind checks
    from lasp_amd import LaspjError
    from lasp_amd._lib import E_SHAPE
    with pytest.raises(LaspjError) as ei:
        L.product_diag(ctx.orset_batch(len(pairs), E + 1))
    assert ei.value.status == E_SHAPE
