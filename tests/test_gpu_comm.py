"""Anti-entropy behind the C ABI (laspj_comm_*, laspj_antientropy*): RCCL on one GPU.

A one-GPU box can only form one-rank communicators (RCCL refuses one device twice in a
communicator), so these tests pin what a round must do at n = 1 — a round leaves the
join of the single copy, i.e. the state unchanged, through the full all-to-all ->
reduce_chunks -> all-gather path and the G-Counter all-reduce(max) — plus the argument
checks; the n > 1 exchange runs in bench.py on the driver's 8-GPU node, and the plan it
executes (laspj_antientropy_plan) is executed over gloo at world 2, 4 and 8 by
tests/test_dist_gloo.py and on this GPU, every rank's buffers in one context, by
laspj_antientropy_loopback (the round's own step arithmetic and reduce kernel, SEND/RECV
pairs as device copies) below.
Reference: lasp_update_fsm.erl:174-216 (N-way merge + repair)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lasp_amd.orset import context
    return context()


def _comm(ctx):
    from lasp_amd.engine import Comm
    return Comm(ctx, 1, Comm.unique_id(), 0)


def test_orset_round_single_rank(ctx):
    c = _comm(ctx)
    assert (c.rank, c.nranks) == (0, 1)
    R, E = 96, 200
    st, rv, ch, ref = (ctx.orset_batch(R, E) for _ in range(4))
    st.fill_synthetic(41)
    ref.fill_synthetic(41)
    ch.fill_synthetic(77)
    before = ch.download()
    c.antientropy(st, rv, ch)
    c.antientropy(st, rv)                 # chunk is optional: the join is done in place
    ctx.synchronize()
    assert np.array_equal(st.download(), ref.download())
    assert np.array_equal(ch.download(), before)          # chunk left untouched
    c.close()


def test_gset_and_gcounter_rounds_single_rank(ctx):
    from lasp_amd.engine import Comm
    (c,) = Comm.init_all([ctx])          # one process owning its GPUs (here: one)
    g, gr, gc, gref = (ctx.gset_batch(64, 300) for _ in range(4))
    g.fill_synthetic(5)
    gref.fill_synthetic(5)
    Comm.antientropy_group([c], [g], [gr], [gc])
    k, kref = ctx.gcounter_batch(50, 64), ctx.gcounter_batch(50, 64)
    k.fill_synthetic(6)
    kref.fill_synthetic(6)
    c.antientropy(k)                      # all_reduce(max) in place, no scratch
    ctx.synchronize()
    assert np.array_equal(g.download(), gref.download())
    assert np.array_equal(k.download(), kref.download())
    c.close()


def test_round_argument_checks(ctx):
    from lasp_amd import _lib
    c = _comm(ctx)
    st = ctx.orset_batch(8, 16)
    st.fill_synthetic(3)
    before = st.download()
    c.antientropy(st)                       # one rank: no copies to receive, recv optional
    ctx.synchronize()
    assert np.array_equal(st.download(), before)           # the join of one copy
    k = ctx.gcounter_batch(8, 16)
    k.fill_synthetic(4)
    kb = k.download()
    c.antientropy(k)
    ctx.synchronize()
    assert np.array_equal(k.download(), kb)
    with pytest.raises(_lib.LaspjError) as e:
        c.antientropy(st, ctx.orset_batch(8, 16), ctx.orset_batch(4, 16))   # chunk != R/n
    assert e.value.status == _lib.E_SHAPE
    with pytest.raises(_lib.LaspjError) as e:
        c.antientropy(st, ctx.gset_batch(8, 16), ctx.orset_batch(8, 16))
    assert e.value.status == _lib.E_KIND
    with pytest.raises(_lib.LaspjError) as e:
        c.antientropy(st, st)                                  # aliasing
    assert e.value.status == _lib.E_INVAL
    with pytest.raises(_lib.LaspjError) as e:
        c.antientropy(st, st.view(2, 4))                       # overlapping recv
    assert e.value.status == _lib.E_INVAL
    c.close()


def _loopback(ctx, n, state, recv, piece):
    import ctypes as C
    from lasp_amd import _lib
    arr = lambda xs: (C.c_void_p * n)(*[x.h.value for x in xs])    # noqa: E731
    _lib.check(ctx.L.laspj_antientropy_loopback(ctx.h, n, arr(state),
                                                 arr(recv) if recv else None, piece), ctx.h)


@pytest.mark.parametrize("n", [2, 3, 4, 8])
@pytest.mark.parametrize("kind", ["orset", "gset", "gcounter"])
def test_round_steps_loopback(ctx, n, kind):
    """n ranks' plans on one device: after the round every rank holds the join of every
    rank's replica of every object (OR of the words for set bitmaps, per-actor max for
    G-Counters), with pieces small enough that every chunk spans several of them."""
    R = 8 * n * 3
    make = {"orset": lambda: ctx.orset_batch(R, 40), "gset": lambda: ctx.gset_batch(R, 300),
            "gcounter": lambda: ctx.gcounter_batch(R, 24)}[kind]
    state = [make() for _ in range(n)]
    for i, st in enumerate(state):
        st.fill_synthetic(100 + i)
    host = [st.download_words() for st in state]
    want = host[0].copy()
    for h in host[1:]:
        want = np.maximum(want, h) if kind == "gcounter" else want | h
    recv = None
    if kind != "gcounter":
        mk = {"orset": lambda r: ctx.orset_batch(r, 40), "gset": lambda r: ctx.gset_batch(r, 300)}[kind]
        recv = [mk(R // n * (n - 1)) for _ in range(n)]
    _loopback(ctx, n, state, recv, 7)
    ctx.synchronize()
    for i, st in enumerate(state):
        assert np.array_equal(st.download_words(), want), i


def test_round_loopback_recv_size(ctx):
    """recv of exactly (n-1)/n of the objects is accepted, one object fewer refused."""
    from lasp_amd import _lib
    n, R = 4, 16
    state = [ctx.orset_batch(R, 8) for _ in range(n)]
    _loopback(ctx, n, state, [ctx.orset_batch(R // n * (n - 1), 8) for _ in range(n)], 0)
    with pytest.raises(_lib.LaspjError) as e:
        _loopback(ctx, n, state, [ctx.orset_batch(R // n * (n - 1) - 1, 8) for _ in range(n)], 0)
    assert e.value.status == _lib.E_SHAPE
