"""Pin the oracle against the reference's own known-answer tests.

Each test cites the reference test it re-runs.  Expected values are copied as data
from those tests; the oracle computes the actual values.
"""

import pytest

from oracle import orset, gset, lattice, core, otp
from oracle.terms import Atom, compare

a, b, c = Atom("a"), Atom("b"), Atom("c")


# ---------------------------------------------------------------- eunit stat tests

def test_orset_stat_kat():
    """src/lasp_orset.erl:273-287 (stat_test)."""
    s = orset.new()
    _, s1 = orset.update(("add", b"foo"), 1, s)
    _, s2 = orset.update(("add", b"foo"), 2, s1)
    _, s3 = orset.update(("add", b"bar"), 3, s2)
    _, s4 = orset.update(("remove", b"foo"), 1, s3)
    assert orset.stats(s) == [("element_count", 0), ("adds_count", 0),
                              ("removes_count", 0), ("waste_pct", 0)]
    assert orset.stat("element_count", s4) == 2
    assert orset.stat("adds_count", s4) == 1
    assert orset.stat("removes_count", s4) == 2
    assert orset.stat("waste_pct", s4) == 67


def test_gset_stat_kat():
    """src/lasp_gset.erl:153-160 (stat_test)."""
    s0 = gset.new()
    _, s1 = gset.update(("add_all", [b"a", b"b1", b"c23", b"d234"]), 1, s0)
    assert gset.stats(s0) == [("element_count", 0), ("max_element_size", 0)]
    assert gset.stats(s1) == [("element_count", 4), ("max_element_size", 15)]
    assert gset.stat("actor_count", s1) is None


# ---------------------------------------------------------------- lattice KATs

def _three(mod, ops=True):
    a1, b1 = mod.new(), mod.new()
    _, a2 = mod.update(("add", 1), a, a1)
    _, b2 = mod.update(("add", 2), b, b1)
    return a1, b1, a2, b2


def test_gset_inflation_kats():
    """src/lasp_lattice.erl:352-382."""
    a1, b1, a2, b2 = _three(gset)
    assert lattice.is_inflation("lasp_gset", a1, b1) is True
    assert lattice.is_inflation("lasp_gset", a1, a2) is True
    assert lattice.is_inflation("lasp_gset", a2, b2) is False
    assert lattice.is_strict_inflation("lasp_gset", a1, b1) is False
    assert lattice.is_strict_inflation("lasp_gset", a1, a2) is True
    assert lattice.is_strict_inflation("lasp_gset", a2, b2) is False


def test_orset_inflation_kats():
    """src/lasp_lattice.erl:531-569."""
    a1, b1, a2, b2 = _three(orset)
    _, a3 = orset.update(("remove", 1), a, a2)
    assert lattice.is_inflation("lasp_orset", a1, b1) is True
    assert lattice.is_inflation("lasp_orset", a1, a2) is True
    assert lattice.is_inflation("lasp_orset", a2, b2) is False
    assert lattice.is_inflation("lasp_orset", a2, a3) is True
    assert lattice.is_strict_inflation("lasp_orset", a1, b1) is False
    assert lattice.is_strict_inflation("lasp_orset", a1, a2) is True
    assert lattice.is_strict_inflation("lasp_orset", a2, b2) is False
    assert lattice.is_strict_inflation("lasp_orset", a2, a3) is True


def test_gcounter_inflation_kats():
    """src/lasp_lattice.erl:386-443 (riak_dt_gcounter clauses, used by the ad counter)."""
    G = core._GCounter
    a1, b1 = G.new(), G.new()
    _, a2 = G.update("increment", a, a1)
    _, a3 = G.update("increment", a, a2)
    _, b2 = G.update("increment", b, b1)
    t = "riak_dt_gcounter"
    assert lattice.is_inflation(t, a1, b1) is True
    assert lattice.is_inflation(t, a2, b1) is False
    assert lattice.is_inflation(t, a1, a2) is True
    assert lattice.is_inflation(t, b1, a2) is True
    assert lattice.is_inflation(t, a2, b2) is False
    assert lattice.is_strict_inflation(t, a1, b1) is False
    assert lattice.is_strict_inflation(t, a2, b1) is False
    assert lattice.is_strict_inflation(t, a1, a2) is True
    assert lattice.is_strict_inflation(t, b1, a2) is True
    assert lattice.is_strict_inflation(t, a2, b2) is False
    assert lattice.is_strict_inflation(t, a2, a2) is False
    assert lattice.is_strict_inflation(t, a2, a3) is True


# ---------------------------------------------------------------- riak_test KATs

@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_union_kat(t):
    """riak_test/lasp_union_test.erl:47-51,67-72."""
    st = core.Store()
    _, s1 = st.declare(t)
    _, s2 = st.declare(t)
    _, s3 = st.declare(t)
    st.update(s1, ("add_all", [1, 2, 3]), a)
    st.update(s2, ("add_all", [a, b, c]), a)
    st.union(s1, s2, s3)
    _, (_, _, v) = st.read(s3, None)
    assert core.type_mod(t).value(v) == [1, 2, 3, a, b, c]


@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_intersection_kat(t):
    """riak_test/lasp_intersection_test.erl:47-51,68-72."""
    st = core.Store()
    _, s1 = st.declare(t)
    _, s2 = st.declare(t)
    _, s3 = st.declare(t)
    st.update(s1, ("add_all", [1, 2, 3, a]), a)
    st.update(s2, ("add_all", [a, b, c, 3]), a)
    st.intersection(s1, s2, s3)
    _, (_, _, v) = st.read(s3, None)
    assert core.type_mod(t).value(v) == [3, a]


@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_product_kat(t):
    """riak_test/lasp_product_test.erl:47-51."""
    st = core.Store()
    _, s1 = st.declare(t)
    _, s2 = st.declare(t)
    _, s3 = st.declare(t)
    st.update(s1, ("add_all", [1, 2, 3]), a)
    st.update(s2, ("add_all", [a, b, c]), a)
    st.product(s1, s2, s3)
    _, (_, _, v) = st.read(s3, None)
    assert core.type_mod(t).value(v) == [(1, a), (1, b), (1, c), (2, a), (2, b), (2, c),
                                          (3, a), (3, b), (3, c)]


def _one_input(t, comb, fun):
    st = core.Store()
    _, s1 = st.declare(t)
    st.update(s1, ("add_all", [1, 2, 3]), a)
    _, s2 = st.declare(t)
    getattr(st, comb)(s1, fun, s2)
    st.update(s1, ("add_all", [4, 5, 6]), a)
    _, (_, _, v1) = st.read(s1)
    _, (_, _, v2) = st.read(s2)
    m = core.type_mod(t)
    return m.value(v1), m.value(v2)


@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_map_kat(t):
    """riak_test/lasp_map_test.erl:47-51,64-76 (fun(X) -> X * 2 end)."""
    assert _one_input(t, "map", lambda x: x * 2) == ([1, 2, 3, 4, 5, 6], [2, 4, 6, 8, 10, 12])


@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_filter_kat(t):
    """riak_test/lasp_filter_test.erl:47-51,70 (fun(X) -> X rem 2 == 0 end)."""
    assert _one_input(t, "filter", lambda x: x % 2 == 0) == ([1, 2, 3, 4, 5, 6], [2, 4, 6])


@pytest.mark.parametrize("t", ["lasp_gset", "lasp_orset"])
def test_fold_kat(t):
    """riak_test/lasp_fold_test.erl:47-51,70 (fun(X) -> [X,X,X] end) — duplicates kept."""
    assert _one_input(t, "fold", lambda x: [x, x, x]) == (
        [1, 2, 3, 4, 5, 6], [1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4, 4, 5, 5, 5, 6, 6, 6])


def test_monotonic_read_kat():
    """riak_test/lasp_monotonic_read_test.erl:46-48,62-86."""
    st = core.Store()
    _, g = st.declare("lasp_gset")
    assert st.read(g, [1, 2, 3]) is None          # blocks
    st.bind(g, [1])
    st.bind(g, [1, 2])
    assert st.read(g, [1, 2, 3]) is None
    st.bind(g, [1, 2, 3])
    assert st.read(g, [1, 2, 3])[1][2] == [1, 2, 3]
    assert st.read(g, [1, 2, 3, 4]) is None
    st.bind(g, [1, 2, 3, 4])
    assert st.read(g, [1, 2, 3, 4])[1][2] == [1, 2, 3, 4]


def test_adcounter_orset_kat():
    """riak_test/lasp_adcounter_orset_test.erl:50-51,57-137: 5 G-Counter ads in an
    OR-Set, 100 views over 5 clients, each ad removed once its threshold-5 read fires;
    the final OR-Set value is []."""
    import random
    st = core.Store()
    _, ads = st.declare("lasp_orset")
    ad_ids = []
    for i in range(5):
        _, ad = st.declare("riak_dt_gcounter", f"ad{i}".encode())  # ids are binaries
        st.update(ads, ("add", ad), None)
        ad_ids.append(ad)
    removed = set()
    rng = random.Random(7)
    for _ in range(100):
        live = orset.value(st.value(ads))
        if not live:
            break
        ad = live[rng.randrange(len(live))]
        st.update(ad, "increment", Atom("client"))
        for x in ad_ids:
            if x not in removed and st.read(x, 5) is not None:   # lasp:read(Ad, 5)
                st.update(ads, ("remove", x), x)
                removed.add(x)
    assert orset.value(st.value(ads)) == []


# ---------------------------------------------------------------- Appendix B traps

def test_gset_union_concatenates():
    """Appendix B item 2: G-Set union = L ++ R (lasp_core.erl:620)."""
    assert core.union_body("lasp_gset", [1, 2, 3], [2, 3, 4]) == [1, 2, 3, 2, 3, 4]


def test_orset_union_keeps_left():
    """Appendix B item 1: common elements keep the left token dict (lasp_core.erl:618)."""
    l = [(1, [(b"t1", False)])]
    r = [(1, [(b"t1", True), (b"t2", False)])]
    assert core.union_body("lasp_orset", l, r) == l


def test_product_tokens_descending():
    """Appendix B item 3: lasp_lattice.erl:303-308."""
    xs = [(b"x1", False), (b"x2", True)]
    ys = [(b"y1", False), (b"y2", False)]
    out = lattice.orset_causal_product(xs, ys)
    assert out == [([b"x2", b"y2"], True), ([b"x2", b"y1"], True),
                   ([b"x1", b"y2"], False), ([b"x1", b"y1"], False)]


def test_orset_is_inflation_ignores_removed():
    """Appendix B item 7."""
    prev = [(1, [(b"t", True)])]
    cur = [(1, [(b"t", False)])]
    assert lattice.is_inflation("lasp_orset", prev, cur) is True


def test_term_order():
    """Appendix A: number < atom < tuple < [] < list < bitstring."""
    seq = [1, 2.5, a, (1,), (0, 0), [], [1], [1, 2], b"", b"a"]
    for x, y in zip(seq, seq[1:]):
        assert compare(x, y) < 0
    assert compare(1, 1.0) == 0


def test_orddict_find_early_exit():
    """Appendix B item 10: orddict:find stops at the first greater key."""
    assert otp.orddict_find(1, [(2, "x"), (1, "y")]) is None


def test_ordsets_union_switch():
    assert otp.ordsets_union([1, 3, 5], [2, 3, 4]) == [1, 2, 3, 4, 5]
    assert otp.ordsets_union([], [1]) == [1]
    assert otp.ordsets_union([1], []) == [1]
