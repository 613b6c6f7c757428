"""OR-Sets whose elements carry more than 64 tokens (LASPJ_KIND_ORSET_WIDE,
lasp_amd/csrc/laspj_wide.hip): add_elem mints a fresh token per add and never collects
tombstones (lasp_orset.erl:222-241, 261-262), so an element re-added many times on N = 3
replicas outgrows the 64-bit cell.  Wide cells hold k {p, r} pairs; merge / value / stats /
equal / inflation / update are checked against the oracle (oracle/orset.py,
oracle/lattice.py) on an element re-added 100 times on each of 3 replicas."""

import random

import numpy as np
import pytest

from oracle import lattice as olat
from oracle import orset as oorset

pytestmark = pytest.mark.gpu


def _replicas(seed=1, adds=100, others=20):
    """3 replicas: each adds element 7 `adds` times (a fresh token each, as add_elem
    does), plus other elements; removals now and then (lasp_orset:update/3)."""
    rng = random.Random(seed)
    reps = []
    for r in range(3):
        toks = oorset.TokenSource(1000 * seed + r)
        s = oorset.new()
        for k in range(adds):
            s = oorset.update(("add_by_token", toks(), 7), None, s)[1]
            if k % 17 == 16:
                s = oorset.update(("remove", 7), None, s)[1]
            if k % 5 == 0:
                e = rng.randrange(others)
                s = oorset.update(("add_by_token", toks(), e), None, s)[1]
        reps.append(s)
    return reps


def _ctx():
    from lasp_amd import engine
    return engine.Context(0)


def test_wide_merge_value_stats_match_oracle():
    from lasp_amd.codec import Domain
    ctx = _ctx()
    try:
        reps = _replicas()
        dom = Domain(token_capacity=64 * 16)
        for s in reps:
            dom.register_orset(s)
        k = dom.token_words()
        assert k == 5                                   # 300 tokens on element 7
        E = dom.size + 3
        cells = dom.encode_orset_wide(reps, E, k)
        b = ctx.orset_wide_batch(3, E, k)
        b.upload(cells)
        # foldl(merge, new(), Replies) — the FSM N-way merge (lasp_update_fsm.erl:189-192)
        one = ctx.orset_wide_batch(1, E, k)
        one.reduce_from(b, 3)
        want = oorset.merge(oorset.merge(reps[0], reps[1]), reps[2])
        got = one.download()[0]
        assert dom.decode_orset_wide(got) == want
        # pairwise merge/2
        x, y, z = (ctx.orset_wide_batch(1, E, k) for _ in range(3))
        x.upload(cells[0:1])
        y.upload(cells[1:2])
        z.join(x, y)
        assert dom.decode_orset_wide(z.download()[0]) == oorset.merge(reps[0], reps[1])
        # value/1, value(removed), stats/1
        order = dom.elements.order()
        terms = dom.elements.terms
        for batch, st in ((one, want), (b, reps[0])):
            bits = batch.value_bits()[0]
            vis = [terms[e] for e in order
                   if e < E and (int(bits[e // 64]) >> (e % 64)) & 1]
            assert vis == oorset.value(st)
            rbits = batch.value_bits(removed=True)[0]
            rem = [terms[e] for e in order if e < E and (int(rbits[e // 64]) >> (e % 64)) & 1]
            assert rem == oorset.value2("removed", st)
            s = batch.stats()[0]
            assert [int(v) for v in s] == [oorset.stat("element_count", st),
                                           oorset.stat("adds_count", st),
                                           oorset.stat("removes_count", st)]
        # equal/2 and (strict) inflation, a broadcast prev included
        assert bool(one.equal(one)[0])
        assert not bool(x.equal(one)[0])
        assert bool(one.is_inflation_of(x)[0]) and bool(one.is_inflation_of(x, strict=True)[0])
        assert bool(one.is_inflation_of(one)[0]) and not bool(one.is_inflation_of(one, strict=True)[0])
        assert not bool(x.is_inflation_of(one)[0])
        assert olat.is_strict_inflation("lasp_orset", reps[0], want)
        infl = b.is_inflation_of(one)                     # prev = 1 replica, broadcast
        assert list(infl) == [olat.is_inflation("lasp_orset", want, s) for s in reps]
    finally:
        ctx.close()


def test_wide_update_ops_match_oracle():
    """update/3 on wide cells: add_by_token past token slot 64 (slot bits 8.. in pad),
    remove (every token of the element := true), and a remove of an absent element (the
    precondition error: the call rolled back)."""
    from lasp_amd import _lib
    from lasp_amd.codec import Domain
    ctx = _ctx()
    try:
        dom = Domain(token_capacity=64 * 4)
        toks = oorset.TokenSource(9)
        s = oorset.new()
        b = ctx.orset_wide_batch(1, 8, 4)
        ops_done = 0
        for k in range(150):
            t = toks()
            es = dom.element_slot(3)
            ts = dom.token_slot(es, t)
            st = b.apply_ops([(0, es, _lib.OP_ADD, ts, _lib.OP_FLAG_NEW_CALL)])
            assert list(st) == [0]
            s = oorset.update(("add_by_token", t, 3), None, s)[1]
            if k % 40 == 39:
                st = b.apply_ops([(0, es, _lib.OP_REMOVE, 0, _lib.OP_FLAG_NEW_CALL)])
                assert list(st) == [0]
                s = oorset.update(("remove", 3), None, s)[1]
            ops_done += 1
        e5 = dom.element_slot(5)
        st = b.apply_ops([(0, e5, _lib.OP_REMOVE, 0, _lib.OP_FLAG_NEW_CALL)])
        assert list(st) == [_lib.OPST_NOT_PRESENT]
        assert oorset.update(("remove", 5), None, s)[0] == "error"
        assert dom.token_words() == 3
        got = b.download()[0]
        assert dom.decode_orset_wide(got) == s
        assert b.stats()[0][1] == sum(1 for _e, ts in s for _t, f in ts if not f)
    finally:
        ctx.close()


def test_wide_bind_many_and_rejections():
    """bind_many / inflation_many take wide one-replica batches (the store's bind path);
    entry points without a wide form (union, filter, ...) reject them (LASPJ_E_KIND)."""
    from lasp_amd import _lib
    from lasp_amd.codec import Domain
    ctx = _ctx()
    try:
        reps = _replicas(seed=2, adds=80)
        dom = Domain(token_capacity=64 * 8)
        for s_ in reps:
            dom.register_orset(s_)
        k = dom.token_words()
        E = dom.size
        cells = dom.encode_orset_wide(reps, E, k)
        bs = []
        for i in range(3):
            x = ctx.orset_wide_batch(1, E, k)
            x.upload(cells[i:i + 1])
            bs.append(x)
        dst = ctx.orset_wide_batch(1, E, k)
        st = ctx.bind_many([dst], [bs[0]], [bs[1]])
        assert list(st) == [1]
        assert dom.decode_orset_wide(dst.download()[0]) == oorset.merge(reps[0], reps[1])
        same = ctx.orset_wide_batch(1, E, k)
        same.upload(cells[0:1])
        st = ctx.bind_many([bs[0]], [bs[0]], [same])          # Value0 =:= Value: a no-op
        assert list(st) == [0]
        inf = ctx.inflation_many([bs[0], bs[0]], [dst, bs[0]], strict=True)
        assert list(inf) == [True, False]
        with pytest.raises(_lib.LaspjError):
            dst.union(bs[0], bs[1])
        narrow = ctx.orset_batch(1, E)
        with pytest.raises(_lib.LaspjError):
            narrow.join(narrow, bs[0])
    finally:
        ctx.close()


def test_store_wide_variables_match_oracle_store():
    """lasp_core over the device with elements past 64 tokens (lasp_amd.core.Store): a
    variable moves to wide cells when its value names token slot >= 64 (bind, bind_many,
    update/3), a narrow variable binding a wide value is widened on the device
    (laspj_orset_widen), threshold reads compare across widths, and every value decodes
    to exactly the oracle store's term (oracle/core.py)."""
    from lasp_amd import core as dcore
    from oracle import core as ocore
    from oracle.terms import exact_eq
    reps = _replicas(seed=3, adds=100)
    ds, os_ = dcore.Store(capacity=64), ocore.Store()
    ids = []
    for st in (ds, os_):
        _, a = st.declare("lasp_orset")
        _, b = st.declare("lasp_orset")
        _, c = st.declare("lasp_orset")
        st.bind(b, [(3, [(b"\x01" * 20, False)])])         # narrow cells first
        st.bind(c, [(4, [(b"\x02" * 20, False)])])
        ids.append((a, b, c))
    (ad, bd, cd), (ao, bo, co) = ids
    for s in reps:
        ds.bind(ad, s)
        os_.bind(ao, s)
        assert exact_eq(ds.value(ad), os_.value(ao))
    assert ds.vars[ad].val.token_words == 5
    assert getattr(ds.vars[bd].val, "token_words", 1) == 1
    ds.bind(bd, reps[0])                                   # narrow variable, wide value
    os_.bind(bo, reps[0])
    assert exact_eq(ds.value(bd), os_.value(bo))
    assert ds.vars[bd].val.token_words > 1
    # bind_many: a wide value into a narrow variable and a narrow one into a wide variable
    small = [(3, [(b"\x05" * 20, False)])]
    ds.bind_many([(cd, reps[1]), (ad, small)])
    os_.bind(co, reps[1])
    os_.bind(ao, small)
    assert exact_eq(ds.value(cd), os_.value(co)) and exact_eq(ds.value(ad), os_.value(ao))
    # update/3 on a wide variable, and one minting the 65th token of a narrow variable
    _, nd = ds.declare("lasp_orset")
    _, no = os_.declare("lasp_orset")
    for k in range(70):
        op = ("add_by_token", bytes([9, k]) + bytes(18), 1)
        ds.update(nd, op, None)
        os_.update(no, op, None)
    assert exact_eq(ds.value(nd), os_.value(no))
    assert ds.vars[nd].val.token_words == 2
    for op in [("add_by_token", b"\x09" * 20, 7), ("remove", 7), ("add_by_token", b"\x0a" * 20, 11)]:
        ds.update(ad, op, None)
        os_.update(ao, op, None)
    assert exact_eq(ds.value(ad), os_.value(ao))
    assert ds.type_value(ad) == oorset.value(os_.value(ao))
    # threshold reads across widths: a narrow threshold on a wide value and back
    assert ds.read(ad, small) is not None and os_.read(ao, small) is not None
    assert (ds.read(cd, ("strict", reps[0])) is None) == (os_.read(co, ("strict", reps[0])) is None)
    assert ds.read(ad, ("strict", os_.value(ao))) is None
    # combinator bodies take narrow values only: documented Unsupported
    _, ud = ds.declare("lasp_orset")
    with pytest.raises(dcore.Unsupported):
        ds.union(ad, cd, ud)


def test_module_api_wide_values_match_oracle():
    """lasp_amd.orset (the lasp_orset mirror) on values past 64 tokens per element:
    merge / value / value({tokens, E}) / precondition_context / update / equal / stats on
    wide cells, against oracle/orset.py."""
    from lasp_amd import orset as dorset
    reps = _replicas(seed=4, adds=90)
    m = oorset.merge(reps[0], reps[1])
    assert dorset.merge(reps[0], reps[1]) == m
    assert dorset.merge_many([(reps[0], reps[2]), (reps[1], [])]) == \
        [oorset.merge(reps[0], reps[2]), oorset.merge(reps[1], [])]
    assert dorset.value(m) == oorset.value(m)
    assert dorset.value2(("tokens", 7), m) == oorset.value2(("tokens", 7), m)
    assert dorset.value2("removed", m) == oorset.value2("removed", m)
    assert dorset.precondition_context(m) == oorset.precondition_context(m)
    assert dorset.equal(m, m) and not dorset.equal(m, reps[0])
    assert [v for _k, v in dorset.stats(m)] == [v for _k, v in oorset.stats(m)]
    for op in [("add_by_token", b"\x0b" * 20, 7), ("remove", 7), ("remove", 999)]:
        assert dorset.update(op, None, m) == oorset.update(op, None, m)
