"""Many variables per launch: laspj_batch_bind_many / laspj_batch_inflation_many against
the one-variable kernels, and the Store's batched bind path (bind_many, the batched
{strict, Last} re-checks of the process loop) against sequential binds on the oracle
store (lasp_core.erl:291-312, lasp_process.erl:61-95)."""

import os

import numpy as np
import pytest
from hypothesis import HealthCheck, example, given, settings, strategies as st

from oracle import core as ocore
from oracle import orset as oorset
from oracle.terms import exact_eq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lasp_amd.orset import context
    return context()


def _batches(ctx, kind, n, E, seed):
    mk = {"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[kind]
    out = []
    for i in range(n):
        b = mk(1, E)
        b.fill_synthetic(seed, replica_base=i)
        out.append(b)
    return out


def test_bind_many_matches_single_kernels(ctx):
    """Mixed kinds and shapes in one call; equal pairs are no-ops (status 0), others are
    merged (OR / per-actor max) into dst (status 1)."""
    shapes = [("o", 4096), ("o", 100), ("g", 5000), ("c", 300), ("o", 12000), ("g", 64)]
    curs, vals, dsts, want = [], [], [], []
    for j, (k, E) in enumerate(shapes):
        a = _batches(ctx, k, 1, E, 2 + j)[0]
        b = _batches(ctx, k, 1, E, 30 + j)[0] if j % 3 else a     # every third: equal
        d = {"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[k](1, E)
        curs.append(a)
        vals.append(b)
        dsts.append(d)
        want.append(0 if b is a else 1)
    st = ctx.bind_many(dsts, curs, vals)          # laspj_batch_bind_many_host
    assert list(st) == want
    # the device-buffer form (laspj_batch_bind_many) answers the same into a buffer
    import ctypes as C
    from lasp_amd import _lib
    n = len(curs)
    arr = lambda xs: (C.c_void_p * n)(*[x.h.value for x in xs])  # noqa: E731
    dsts2 = [{"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[k](1, E)
             for k, E in shapes]
    buf = ctx.buffer(n)
    _lib.check(ctx.L.laspj_batch_bind_many(ctx.h, n, arr(dsts2), arr(curs), arr(vals), buf.h),
               ctx.h)
    assert list(buf.download(np.uint8)) == want
    for d, d2, s in zip(dsts, dsts2, st):
        if s:
            assert np.array_equal(d.download_words(), d2.download_words())
    for (k, E), a, b, d, s in zip(shapes, curs, vals, dsts, st):
        if s:
            ref = {"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[k](1, E)
            ref.join(a, b)
            assert np.array_equal(d.download_words(), ref.download_words())
    # in place (dst = cur)
    a, b = _batches(ctx, "o", 1, 777, 5)[0], _batches(ctx, "o", 1, 777, 6)[0]
    ref = ctx.orset_batch(1, 777).join(a, b)
    assert list(ctx.bind_many([a], [a], [b])) == [1]
    assert np.array_equal(a.download_words(), ref.download_words())


def test_inflation_many_matches_single_kernels(ctx):
    pairs = []
    for k, E in (("o", 4096), ("o", 50), ("g", 3000), ("c", 200), ("o", 9000)):
        p = _batches(ctx, k, 1, E, 11)[0]
        q = _batches(ctx, k, 1, E, 12)[0]
        m = {"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[k](1, E)
        m.join(p, q)
        empty = {"o": ctx.orset_batch, "g": ctx.gset_batch, "c": ctx.gcounter_batch}[k](1, E)
        pairs += [(p, m), (m, p), (p, p), (q, m), (empty, p), (p, empty), (empty, empty)]
    for strict in (False, True):
        got = ctx.inflation_many([a for a, _ in pairs], [b for _, b in pairs], strict)
        want = [bool(b.is_inflation_of(a, strict=strict)[0]) for a, b in pairs]
        assert list(got) == want, strict


SET = st.lists(st.tuples(st.sampled_from(["add", "remove"]), st.integers(0, 9)), max_size=10)


@settings(max_examples=20 * int(os.environ.get("LASPJ_SOAK", "1")), deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(st.tuples(st.integers(0, 3), SET), min_size=1, max_size=6))
# a variable named twice ahead of the union's right input: its second pair must land
# before the dataflow runs (a soak found bind_many propagating between the two)
@example([(0, []), (0, [("add", 0)]), (1, [("add", 0)])])
def test_store_bind_many_vs_sequential_oracle(batch):
    """Store.bind_many ends where the oracle ends when it applies the same binds with the
    dataflow deferred until all of them have landed (the interleaving bind_many runs;
    the keep-left union makes the schedule observable, so the oracle runs the same one)."""
    from lasp_amd import core as dcore
    ds, os_ = dcore.Store(capacity=64), ocore.Store()

    def setup(store):
        ids = [store.declare("lasp_orset")[1] for _ in range(6)]
        store.union(ids[0], ids[1], ids[4])
        store.filter(ids[2], lambda x: x % 2 == 0, ids[5])
        return ids
    idd, ido = setup(ds), setup(os_)
    seed = oorset.TokenSource(4)
    terms = []
    for var, ops in batch:
        s = oorset.new()
        for op in ops:
            if op[0] == "add":
                op = ("add_by_token", seed(), op[1])
            r = oorset.update(op, None, s)
            if r[0] == "ok":
                s = r[1]
        terms.append((var, s))
    # every variable starts non-empty so the batched path is the one taken
    for k in range(4):
        first = [(("add_by_token", bytes([k + 1]) * 20, 100 + k))]
        for store, ids in ((ds, idd), (os_, ido)):
            store.update(ids[k], first[0], None)
    ds.bind_many([(idd[v], s) for v, s in terms])
    os_._depth += 1                      # writes first, then one propagation
    try:
        for v, s in terms:
            os_.bind(ido[v], s)
    finally:
        os_._depth -= 1
    os_._propagate()
    for a, b in zip(idd, ido):
        assert exact_eq(ds.value(a), os_.value(b))
    assert ds.ctx.pool_hits > 0


def test_bind_many_generator_and_failure_propagation():
    """bind_many reads a generator of pairs once and still answers every pair; writes
    that landed before a failing pair reach their processes."""
    from lasp_amd import core as dcore
    t1, t2, t3 = (bytes([k]) * 20 for k in (1, 2, 3))
    st_ = dcore.Store(capacity=64)
    _, a = st_.declare("lasp_orset")
    _, m = st_.declare("lasp_orset")
    st_.update(a, ("add_by_token", t1, 1), None)
    st_.map(a, lambda x: x * 2, m)
    res = st_.bind_many(p for p in [(a, [(2, [(t2, False)])])])
    assert [r[1][0] for r in res] == [a]
    assert st_.type_value(m) == [2, 4]
    _, b = st_.declare("lasp_orset")                # empty: bound through bind/3 at once
    _, mb = st_.declare("lasp_orset")
    st_.map(b, lambda x: x + 100, mb)
    with pytest.raises(KeyError):
        st_.bind_many([(b, [(5, [(t3, False)])]), (b"undeclared", [])])
    assert st_.type_value(b) == [5]
    assert st_.type_value(mb) == [105]


def test_bind_many_rejects_overlapping_dsts(ctx):
    """dst[i] may be cur[i] exactly; a dst over another item's cur or val, over its own
    val, or over another dst is refused before any launch (k_bind_many
    would read and write the same words from different waves)."""
    from lasp_amd import _lib
    big = ctx.orset_batch(6, 64)
    big.fill_synthetic(3)
    v = [big.view(k, 1) for k in range(6)]
    before = big.download()
    st = ctx.bind_many([v[0], v[1]], [v[0], v[1]], [v[2], v[3]])      # in place: fine
    assert list(st) == [1, 1]
    for dsts, curs, vals in (([v[1], v[4]], [v[0], v[1]], [v[2], v[3]]),   # dst0 = cur1
                             ([v[3], v[4]], [v[0], v[1]], [v[2], v[3]]),   # dst0 = val1
                             ([v[2], v[4]], [v[0], v[1]], [v[2], v[3]]),   # dst0 = own val
                             ([v[4], v[4]], [v[0], v[1]], [v[2], v[3]])):  # dst0 = dst1
        with pytest.raises(_lib.LaspjError) as e:
            ctx.bind_many(dsts, curs, vals)
        assert e.value.status == _lib.E_INVAL
    after = big.download()
    assert np.array_equal(after[2:], before[2:])          # the refused calls wrote nothing
