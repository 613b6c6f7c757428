"""lasp_orset_gbtree (src/lasp_orset_gbtree.erl, Lasp's default `?SET`,
include/lasp.hrl:30): the oracle pinned by the reference's own KATs, the OTP gb_trees
restatement's invariants, the host tree builder against the oracle's insert, and
(-m gpu) the device mirror against the oracle.
"""

import random

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from oracle import gbtrees as ogb, lattice as olat, orset as oors, orset_gbtree as ogt
from oracle.terms import exact_eq

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run


def _tok(k: int) -> bytes:
    return bytes([(k * 37 + 11) & 0xFF]) * 19 + bytes([k & 0xFF])


# ---------------------------------------------------------------- reference KATs

def test_gbtree_stat_kat():
    """src/lasp_orset_gbtree.erl:299-314 (stat_test)."""
    s = ogt.new()
    _, s1 = ogt.update(("add", b"foo"), 1, s)
    _, s2 = ogt.update(("add", b"foo"), 2, s1)
    _, s3 = ogt.update(("add", b"bar"), 3, s2)
    _, s4 = ogt.update(("remove", b"foo"), 1, s3)
    assert ogt.stats(s) == [("element_count", 0), ("adds_count", 0),
                            ("removes_count", 0), ("waste_pct", 0)]
    assert ogt.stat("element_count", s4) == 2
    assert ogt.stat("adds_count", s4) == 1
    assert ogt.stat("removes_count", s4) == 2
    assert ogt.stat("waste_pct", s4) == 67


def _kat_states(mod):
    a1, b1 = mod.new(), mod.new()
    _, a2 = mod.update(("add", 1), "a", a1)
    _, b2 = mod.update(("add", 2), "b", b1)
    _, a3 = mod.update(("remove", 1), "a", a2)
    return a1, b1, a2, b2, a3


def test_gbtree_inflation_kats():
    """src/lasp_lattice.erl:573-591 and :593-613."""
    a1, b1, a2, b2, a3 = _kat_states(ogt)
    t = "lasp_orset_gbtree"
    assert olat.is_inflation(t, a1, b1) is True
    assert olat.is_inflation(t, a1, a2) is True
    assert olat.is_inflation(t, a2, b2) is False
    assert olat.is_inflation(t, a2, a3) is True
    assert olat.is_strict_inflation(t, a1, b1) is False
    assert olat.is_strict_inflation(t, a1, a2) is True
    assert olat.is_strict_inflation(t, a2, b2) is False
    assert olat.is_strict_inflation(t, a2, a3) is True
    assert olat.threshold_met(t, a3, ("strict", a2)) is True
    assert olat.threshold_met(t, a3, a2) is True


# ---------------------------------------------------------------- gb_trees restatement

def _height(node):
    if node == ogb.NIL:
        return 0
    return 1 + max(_height(node[2]), _height(node[3]))


@pytest.mark.parametrize("seed", range(6))
def test_gb_trees_insert_invariants(seed):
    """Random-order inserts: in-order walk sorted, sizes right, lookups hit, height
    within the p = 2 bound (height <= 2 log2(size) + 2 after rebalancing), and the
    duplicate insert raises {key_exists, K}."""
    rng = random.Random(seed)
    keys = rng.sample(range(10_000), 400)
    t = ogb.empty()
    for i, k in enumerate(keys):
        t = ogb.insert(k, -k, t)
        assert ogb.size(t) == i + 1
    assert [k for k, _ in ogb.to_list(t)] == sorted(keys)
    assert all(ogb.lookup(k, t) == ("value", -k) for k in keys)
    assert ogb.lookup(-1, t) is None
    import math
    assert _height(t[1]) <= 2 * math.log2(len(keys)) + 2
    with pytest.raises(ogb.KeyExists):
        ogb.insert(keys[0], 0, t)
    t2 = ogb.enter(keys[0], "x", t)
    assert ogb.size(t2) == ogb.size(t) and ogb.get(keys[0], t2) == "x"


def test_host_builder_matches_sorted_inserts():
    """lasp_amd.gbtrees.build_sorted (right-spine, iterative) is the tree the oracle's
    recursive gb_trees:insert/3 builds for ascending keys, for every size to 1200."""
    from lasp_amd import gbtrees as pgb
    for n in range(0, 1200):
        pairs = [(i, i * 3) for i in range(n)]
        b = pgb.build_sorted(pairs)
        assert exact_eq(ogb.from_pairs_by_insert(pairs), b), n
        assert pgb.walk(b) == pairs


def test_merge_output_is_sorted_insert_shape():
    """gb_trees_ext:merge/3 (src/gb_trees_ext.erl:28-57) inserts keys in ascending
    order into empty(): the outer tree and the inner trees of common elements are
    always the ascending-insert shape; an inner tree present on one side only is
    passed through as it was.  So merge of merge-shaped inputs is from_orddict of its
    contents exactly — the shape the device mirror returns."""
    from lasp_amd import gbtrees as pgb
    from lasp_amd.orset_gbtree import from_orddict
    rng = random.Random(5)
    for _ in range(40):
        a, b = _random_tree(rng, 30), _random_tree(rng, 30)
        m = ogt.merge(a, b)
        assert exact_eq(_outer_shape(m), _outer_shape(pgb.build_sorted(ogb.to_list(m))))
        ca, cb = from_orddict(ogt.to_orddict(a)), from_orddict(ogt.to_orddict(b))
        m2 = ogt.merge(ca, cb)
        assert exact_eq(m2, from_orddict(ogt.to_orddict(m2)))


def _outer_shape(t):
    """The tree with every value replaced by 0 (compare outer shapes only)."""
    def strip(n):
        return n if n == ogb.NIL else (n[0], 0, strip(n[2]), strip(n[3]))
    return strip(t[1])


# ---------------------------------------------------------------- content parity with lasp_orset

_ops = st.lists(st.tuples(st.sampled_from(["add", "remove"]), st.integers(0, 12),
                          st.integers(0, 40)), max_size=30)


def _apply(mod, ops, start):
    s = start
    for kind, e, t in ops:
        if kind == "add":
            try:
                s = mod.update(("add_by_token", _tok(t), e), 1, s)[1]
            except ogb.KeyExists:
                pass
        else:
            r = mod.update(("remove", e), 1, s)
            if r[0] == "ok":
                s = r[1]
    return s


def _dedupe(ops):
    """gbtree add of a present token crashes; keep first (element, token) adds only."""
    seen, out = set(), []
    for op in ops:
        if op[0] == "add":
            if (op[1], op[2]) in seen:
                continue
            seen.add((op[1], op[2]))
        out.append(op)
    return out


@settings(max_examples=120 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_ops, _ops)
def test_gbtree_contents_equal_orset(ops_a, ops_b):
    """With distinct tokens the two containers hold the same contents after the same
    updates, and merge / value / stats / inflation agree on them."""
    ops_a, ops_b = _dedupe(ops_a), _dedupe(ops_b)
    ga, gb_ = _apply(ogt, ops_a, ogt.new()), _apply(ogt, ops_b, ogt.new())
    oa, ob = _apply(oors, ops_a, oors.new()), _apply(oors, ops_b, oors.new())
    assert exact_eq(ogt.to_orddict(ga), oa)
    gm, om = ogt.merge(ga, gb_), oors.merge(oa, ob)
    assert exact_eq(ogt.to_orddict(gm), om)
    assert ogt.value(gm) == oors.value(om)
    assert ogt.value2("removed", gm) == oors.value2("removed", om)
    assert ogt.stats(gm) == oors.stats(om)
    for p, c in ((ga, gm), (gm, ga), (ga, gb_)):
        po, co = ogt.to_orddict(p), ogt.to_orddict(c)
        assert olat.is_inflation("lasp_orset_gbtree", p, c) == \
            olat.is_inflation("lasp_orset", po, co)


def test_gbtree_quirks():
    """Reference behaviour the restatement keeps (src/lasp_orset_gbtree.erl):
    duplicate token insert crashes; fragment of an absent element is a one-entry tree
    holding empty(); strict inflation compares token trees by shape."""
    _, s = ogt.update(("add_by_token", _tok(1), 5), 1, ogt.new())
    with pytest.raises(ogb.KeyExists):
        ogt.update(("add_by_token", _tok(1), 5), 1, s)
    frag = ogt.value2(("fragment", 99), s)
    assert exact_eq(frag, (1, (99, ogb.empty(), ogb.NIL, ogb.NIL)))
    # descending token inserts vs the merge-built (ascending) tree: same contents,
    # different shapes -> the reference calls it a strict inflation
    d = ogt.new()
    for k in (3, 2, 1):
        d = ogt.update(("add_by_token", _tok(k), 7), 1, d)[1]
    m = ogt.merge(d, ogt.new())
    assert exact_eq(ogt.to_orddict(d), ogt.to_orddict(m))
    assert ogt.to_orddict(d) == ogt.to_orddict(m)
    shapes_differ = not exact_eq(ogb.get(7, d), ogb.get(7, m))
    assert olat.is_strict_inflation("lasp_orset_gbtree", d, m) is shapes_differ
    assert ogt.equal(d, m) is (not shapes_differ)


# ---------------------------------------------------------------- device mirror (GPU)

def _random_tree(rng, n_ops=25, canonical=False):
    s = ogt.new()
    used = set()
    for _ in range(n_ops):
        e = rng.randint(0, 30)
        if rng.random() < 0.8:
            t = rng.randint(0, 120)
            if (e, t) in used:
                continue
            used.add((e, t))
            s = ogt.update(("add_by_token", _tok(t), e), 1, s)[1]
        else:
            r = ogt.update(("remove", e), 1, s)
            if r[0] == "ok":
                s = r[1]
    if canonical:
        from lasp_amd.orset_gbtree import from_orddict
        s = from_orddict(ogt.to_orddict(s))
    return s


@pytest.mark.gpu
def test_gpu_gbtree_merge_value_stats():
    from lasp_amd import orset_gbtree as dg
    rng = random.Random(11)
    pairs = [(_random_tree(rng), _random_tree(rng)) for _ in range(24)]
    got = dg.merge_many(pairs)
    for (a, b), g in zip(pairs, got):
        want = ogt.merge(a, b)
        # the whole term, shapes included: an element of one operand keeps its token
        # tree as it is (gb_trees_ext:merge/3 inserts Val1 / Val2 itself)
        assert exact_eq(g, want)
        ca, cb = dg.from_orddict(ogt.to_orddict(a)), dg.from_orddict(ogt.to_orddict(b))
        assert exact_eq(dg.merge(ca, cb), ogt.merge(ca, cb))
        assert dg.value(g) == ogt.value(want)
        assert dg.value2("removed", g) == ogt.value2("removed", want)
        assert dg.stats(g) == ogt.stats(want)
        assert dg.equal(g, want) is True
    for e in (0, 5, 31, 99):
        s = pairs[0][0]
        assert exact_eq(dg.value2(("tokens", e), dg.from_orddict(ogt.to_orddict(s))),
                        ogt.value2(("tokens", e), dg.from_orddict(ogt.to_orddict(s))))
        assert exact_eq(dg.value2(("fragment", e), dg.from_orddict(ogt.to_orddict(s))),
                        ogt.value2(("fragment", e), dg.from_orddict(ogt.to_orddict(s))))
    assert exact_eq(dg.merge(dg.new(), dg.new()), ogt.new())


@pytest.mark.gpu
def test_gpu_gbtree_update_errors():
    from lasp_amd import orset_gbtree as dg
    s = dg.new()
    _, s = dg.update(("add_by_token", _tok(1), 5), 1, s)
    _, s = dg.update(("add_by_token", _tok(2), 5), 1, s)
    want = ogt.update(("add_by_token", _tok(2), 5), 1,
                      ogt.update(("add_by_token", _tok(1), 5), 1, ogt.new())[1])[1]
    assert exact_eq(ogt.to_orddict(s), ogt.to_orddict(want))
    with pytest.raises(dg.KeyExists) as ei:
        dg.update(("add_by_token", _tok(1), 5), 1, s)
    assert ei.value.token == _tok(1)
    # the same token twice inside one {update, Ops} call
    with pytest.raises(dg.KeyExists):
        dg.update(("update", [("add_by_token", _tok(9), 6), ("add_by_token", _tok(9), 6)]), 1, s)
    assert dg.update(("remove", 77), 1, s) == ("error", ("precondition", ("not_present", 77)))
    # remove_all stops at the first absent element; the state is unchanged
    r = dg.update(("remove_all", [5, 77]), 1, s)
    assert r == ("error", ("precondition", ("not_present", 77)))
    _, s2 = dg.update(("update", [("add_by_token", _tok(3), 8), ("remove", 8)]), 1, s)
    want2 = ogt.update(("update", [("add_by_token", _tok(3), 8), ("remove", 8)]), 1, want)[1]
    assert exact_eq(s2, want2)                  # the reference's tree, shapes included
    assert dg.value(s2) == ogt.value(want2) == [5]


@pytest.mark.gpu
def test_gpu_gbtree_lattice_kats():
    """src/lasp_lattice.erl:573-613 through the device."""
    from lasp_amd import lattice as dl, orset_gbtree as dg
    a1, b1 = dg.new(), dg.new()
    _, a2 = dg.update(("add", 1), "a", a1)
    _, b2 = dg.update(("add", 2), "b", b1)
    _, a3 = dg.update(("remove", 1), "a", a2)
    t = "lasp_orset_gbtree"
    assert [dl.is_inflation(t, *p) for p in ((a1, b1), (a1, a2), (a2, b2), (a2, a3))] == \
        [True, True, False, True]
    assert [dl.is_strict_inflation(t, *p) for p in ((a1, b1), (a1, a2), (a2, b2), (a2, a3))] == \
        [False, True, False, True]
    assert dl.threshold_met(t, a3, ("strict", a2)) is True


@pytest.mark.gpu
def test_gpu_gbtree_store_matches_oracle_store():
    """Every value a store holds is a merge output (lasp_core.erl:300), built by
    ascending inserts at both levels, so with merge-shaped binds the device store's
    gbtree variable equals the oracle store's as a whole term, shapes included."""
    from lasp_amd import core as dcore
    from oracle import core as ocore
    rng = random.Random(3)
    script = []
    used = set()
    for _ in range(60):
        e = rng.randint(0, 20)
        if rng.random() < 0.75:
            t = rng.randint(0, 90)
            if (e, t) in used:
                continue
            used.add((e, t))
            script.append(("update", ("add_by_token", _tok(t), e)))
        elif rng.random() < 0.5:
            script.append(("update", ("remove", e)))
        else:
            script.append(("bind", _random_tree(rng, 8, canonical=True)))

    def run(store):
        _, v = store.declare("lasp_orset_gbtree")
        vals = []
        for kind, arg in script:
            if kind == "update":
                try:
                    store.update(v, arg, 1)
                except Exception:       # not_present -> badmatch in both stores
                    pass
            else:
                store.bind(v, arg)
            vals.append(store.value(v))
        return vals, store, v

    dvals, ds, dv = run(dcore.Store(capacity=128))
    ovals, os_, ov = run(ocore.Store())
    assert len(dvals) == len(ovals)
    for k, (x, y) in enumerate(zip(dvals, ovals)):
        assert exact_eq(x, y), k
    assert ds.read(dv, ("strict", None))[0] == "ok"
    assert ds.read(dv, ("strict", ds.value(dv))) is None


@pytest.mark.gpu
def test_gpu_gbtree_update_shapes_match_reference():
    """Trees built by update sequences keep the shape their insertion history gives them
    (gb_trees:insert / enter in add_elem, the ordered rebuild in remove_elem,
    src/lasp_orset_gbtree.erl:231-253): after every update the device mirror's state is
    the oracle's state as a whole term; equal/2 (gb_trees_ext:equal compares the inner
    token TREES) and strict inflation (lasp_lattice.erl:217-233, `Ids =/= Ids1` on trees)
    against the state's merge agree with the reference, as do value({tokens, E}),
    value({fragment, E}) and precondition_context/1."""
    from lasp_amd import lattice as dl, orset_gbtree as dg
    T = "lasp_orset_gbtree"
    rng = random.Random(5)
    for trial in range(6):
        d, o, used = dg.new(), ogt.new(), set()
        for _ in range(40):
            e = rng.randint(0, 12)
            if rng.random() < 0.8:
                t = rng.randint(0, 200)
                if (e, t) in used:
                    continue
                used.add((e, t))
                op = ("add_by_token", _tok(t), e)
            else:
                op = ("remove", e)
            rd, ro = dg.update(op, 1, d), ogt.update(op, 1, o)
            assert rd[0] == ro[0]
            if rd[0] == "ok":
                d, o = rd[1], ro[1]
            assert exact_eq(d, o), (trial, op)
        m = ogt.merge(o, ogt.new())
        assert dg.equal(d, m) is ogt.equal(o, m)
        assert dg.equal(d, d) is True
        assert dl.is_strict_inflation(T, d, m) is olat.is_strict_inflation(T, o, m)
        assert dl.is_strict_inflation(T, m, d) is olat.is_strict_inflation(T, m, o)
        for e in range(14):
            assert exact_eq(dg.value2(("tokens", e), d), ogt.value2(("tokens", e), o)), e
            assert exact_eq(dg.value2(("fragment", e), d), ogt.value2(("fragment", e), o)), e
        assert exact_eq(dg.precondition_context(d), ogt.precondition_context(o))
    # tokens added in descending order: merged with new() the element is one-sided and
    # keeps its tree (equal, not strictly inflated); merged with a replica that also
    # holds the element, its tree is rebuilt in ascending order — same contents, another
    # shape: not equal, and a strict inflation (as the reference answers)
    d, o = dg.new(), ogt.new()
    for k in (3, 2, 1):
        d = dg.update(("add_by_token", _tok(k), 7), 1, d)[1]
        o = ogt.update(("add_by_token", _tok(k), 7), 1, o)[1]
    assert exact_eq(d, o)
    m0 = dg.merge(d, dg.new())
    assert exact_eq(m0, ogt.merge(o, ogt.new()))
    assert dg.equal(d, m0) is True and ogt.equal(o, ogt.merge(o, ogt.new())) is True
    assert dl.is_strict_inflation(T, d, m0) is False
    d1 = dg.update(("add_by_token", _tok(1), 7), 1, dg.new())[1]
    o1 = ogt.update(("add_by_token", _tok(1), 7), 1, ogt.new())[1]
    m = dg.merge(d, d1)
    assert exact_eq(m, ogt.merge(o, o1))
    assert dg.equal(d, m) is False and ogt.equal(o, ogt.merge(o, o1)) is False
    assert dl.is_strict_inflation(T, d, m) is True
    assert olat.is_strict_inflation(T, o, ogt.merge(o, o1)) is True
    assert dl.is_inflation(T, d, m) is True


@pytest.mark.gpu
def test_gpu_gbtree_store_shapes_with_update_built_binds():
    """Binding update-built trees (token trees of any shape) and updating in place: the
    device store's variable equals the oracle store's as a whole term after every step
    (gb_trees_ext:merge keeps a one-sided element's tree, rebuilds a shared one), and
    {strict, T} reads agree, shape changes included (lasp_lattice.erl:217-233)."""
    from lasp_amd import core as dcore
    from oracle import core as ocore
    rng = random.Random(17)
    script = []
    used = set()
    for _ in range(70):
        e = rng.randint(0, 15)
        x = rng.random()
        if x < 0.55:
            t = rng.randint(0, 90)
            if (e, t) in used:
                continue
            used.add((e, t))
            script.append(("update", ("add_by_token", _tok(t), e)))
        elif x < 0.7:
            script.append(("update", ("remove", e)))
        else:
            tree = _random_tree(rng, 10)
            for e2, toks in ogt.to_orddict(tree):
                used.update((e2, tt) for tt in range(256)
                            if any(tok == _tok(tt) for tok, _f in toks))
            script.append(("bind", tree))

    def run(store):
        _, v = store.declare("lasp_orset_gbtree")
        vals, reads = [], []
        for kind, arg in script:
            if kind == "update":
                try:
                    store.update(v, arg, 1)
                except Exception:       # not_present / key_exists -> crash in both stores
                    pass
            else:
                store.bind(v, arg)
                reads.append(store.read(v, ("strict", arg)) is not None)
            vals.append(store.value(v))
        return vals, reads

    dvals, dreads = run(dcore.Store(capacity=256))
    ovals, oreads = run(ocore.Store())
    for k, (x, y) in enumerate(zip(dvals, ovals)):
        assert exact_eq(x, y), k
    assert dreads == oreads
