"""Anti-entropy behind the C ABI (laspj_comm_*, laspj_antientropy*): RCCL on one GPU.

A one-GPU box can only form one-rank communicators (RCCL refuses one device twice in a
communicator), so these tests pin what a round must do at n = 1 — a round leaves the
join of the single copy, i.e. the state unchanged, through the full all-to-all ->
reduce_chunks -> all-gather path and the G-Counter all-reduce(max) — plus the argument
checks; the n > 1 exchange runs in bench.py on the driver's 8-GPU node, and the plan it
executes (laspj_antientropy_plan) is executed over gloo at world 2 and 4 by
tests/test_dist_gloo.py.
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
    c.antientropy(st)                       # one rank: no copies to receive, recv optional
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
