"""Randomised parity (hypothesis) of the device combinator bodies and the device
lasp_core store against the oracle, beyond the fixed golden vectors."""

import os

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

from oracle import core as ocore
from oracle import orset as oorset
from oracle.terms import exact_eq

pytestmark = pytest.mark.gpu

ELEM = st.integers(min_value=-4, max_value=12)
OP = st.one_of(st.tuples(st.just("add"), ELEM), st.tuples(st.just("remove"), ELEM))
SET = st.lists(OP, max_size=14)


def build(ops, seed):
    s = oorset.new()
    toks = oorset.TokenSource(seed)
    for op in ops:
        r = oorset.update(op, None, s, toks)
        if r[0] == "ok":
            s = r[1]
    return s


SOAK = int(os.environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run
SETTINGS = settings(max_examples=40 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(SET, SET)
def test_bodies_random(lops, rops):
    from lasp_amd import orset as do
    from lasp_amd.codec import Domain, SeqOutput, decode_concat, decode_product
    l, r = build(lops, 1), build(rops, 2)
    ctx = do.context()
    dom = Domain()
    dom.register_orset(l)
    dom.register_orset(r)
    E = max(1, dom.size)
    L, R = ctx.orset_batch(1, E), ctx.orset_batch(1, E)
    L.upload(dom.encode_orset([l], E))
    R.upload(dom.encode_orset([r], E))
    U = ctx.orset_batch(1, E).union(L, R)
    assert exact_eq(dom.decode_orset(U.download()[0]), ocore.union_body("lasp_orset", l, r))
    X = L.intersection(R)
    assert exact_eq(decode_concat(dom, X.download()[0]), ocore.intersection_body("lasp_orset", l, r))
    odd = lambda x: x % 2 == 1          # noqa: E731
    F = ctx.orset_batch(1, E).filter(L, dom.keep_bits(odd, E))
    assert exact_eq(dom.decode_orset(F.download()[0]), ocore.filter_body("lasp_orset", odd, l))
    for fun, kind in ((lambda x: -x, "map"), (lambda x: x // 3, "map"),
                      (lambda x: [x, x + 100], "fold"), (lambda x: [] if x % 2 else [x], "fold")):
        so = SeqOutput.map(dom, fun) if kind == "map" else SeqOutput.fold(dom, fun)
        G = ctx.orset_batch(1, max(1, so.size)).gather(L, so.index())
        want = (ocore.map_body if kind == "map" else ocore.fold_body)("lasp_orset", fun, l)
        assert exact_eq(so.decode_orset(G.download()[0]), want)
    # product over per-side dictionaries (token slots < 8 always hold here: <= 14 adds)
    dl, dr = Domain(), Domain()
    dl.register_orset(l)
    dr.register_orset(r)
    PL, PR = ctx.orset_batch(1, max(1, dl.size)), ctx.orset_batch(1, max(1, dr.size))
    PL.upload(dl.encode_orset([l], PL.elements))
    PR.upload(dr.encode_orset([r], PR.elements))
    if all(len(t) <= 8 for _, t in l) and all(len(t) <= 8 for _, t in r):
        P = PL.product(PR)
        assert exact_eq(decode_product(dl, dr, P.download()[0]), ocore.product_body("lasp_orset", l, r))


STEP = st.one_of(
    st.tuples(st.just("update"), st.integers(0, 1), OP),
    st.tuples(st.just("bind"), st.integers(0, 1), SET),
    st.tuples(st.just("gadd"), st.integers(0, 1), st.lists(ELEM, min_size=1, max_size=4)),
    st.tuples(st.just("gbind"), st.integers(0, 1), st.lists(ELEM, max_size=6)))


def _setup(store):
    """Two OR-Set inputs and two G-Set inputs feeding every combinator, including the
    ones whose outputs are not orddicts (intersection, product, a non-monotone map, the
    G-Set `L ++ R` union) and processes chained onto those outputs; every input change
    re-runs them, so each output is re-bound (merged into its previous value) again
    and again."""
    ids = [store.declare("lasp_orset")[1] for _ in range(10)]
    a, b, u, x, p, f, m, fo, mx, ux = ids
    store.union(a, b, u)
    store.intersection(a, b, x)
    store.product(a, b, p)
    store.filter(a, lambda v: v % 2 == 0, f)
    store.map(b, lambda v: v % 3, m)                      # non-monotone, collapsing
    store.fold(a, lambda v: [v, -v], fo)                  # unsorted output keys
    store.map(x, lambda v: -v, mx)                        # chained on a list value
    store.union(m, fo, ux)                                # keep-left merge of lists
    gids = [store.declare("lasp_gset")[1] for _ in range(6)]
    ga, gb, gu, gx, gm, gf = gids
    store.union(ga, gb, gu)                               # L ++ R
    store.intersection(ga, gb, gx)
    store.map(gu, lambda v: v // 2, gm)
    store.filter(gu, lambda v: v > 0, gf)
    return ids, gids


@settings(max_examples=25 * SOAK, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(st.lists(STEP, max_size=10))
def test_store_random(steps):
    """After every step each variable — inputs and every combinator output, list values
    included — decodes to the oracle store's value, term for term."""
    from lasp_amd import core as dcore
    ds, os_ = dcore.Store(capacity=256), ocore.Store(tokens=oorset.TokenSource(9))
    toks = oorset.TokenSource(5)
    (idd, gdd), (ido, gdo) = _setup(ds), _setup(os_)
    for n, step in enumerate(steps):
        kind, var = step[0], step[1]
        if kind == "update":
            op = step[2]
            # deterministic tokens: the same token reaches both stores
            if op[0] == "add":
                op = ("add_by_token", toks(), op[1])
            try:
                os_.update(ido[var], op, None)
            except RuntimeError:
                with pytest.raises(RuntimeError):
                    ds.update(idd[var], op, None)
                continue
            ds.update(idd[var], op, None)
        elif kind == "bind":
            term = build(step[2], 100 + n)
            os_.bind(ido[var], term)
            ds.bind(idd[var], term)
        elif kind == "gadd":
            os_.update(gdo[var], ("add_all", step[2]), None)
            ds.update(gdd[var], ("add_all", step[2]), None)
        else:
            term = sorted(set(step[2]))
            os_.bind(gdo[var], term)
            ds.bind(gdd[var], term)
        for i_d, i_o in list(zip(idd, ido)) + list(zip(gdd, gdo)):
            assert exact_eq(ds.value(i_d), os_.value(i_o)), (step, ds.value(i_d), os_.value(i_o))
        assert len(ds.procs) == len(os_.procs)


def test_store_rebinds_intersection_twice():
    """The VERDICT's example: re-binding an intersection output merges `Cx ++ Cy` lists
    with orddict:merge's two-finger walk and keeps the duplicated token."""
    from lasp_amd import core as dcore
    from oracle.terms import Atom
    ds, os_ = dcore.Store(capacity=64), ocore.Store()
    t = [bytes([i]) * 20 for i in range(8)]
    for st_ in (ds, os_):
        a, b, x = (st_.declare("lasp_orset")[1] for _ in range(3))
        st_.intersection(a, b, x)
        st_.update(a, ("add_by_token", t[3], 1), Atom("a"))
        st_.update(b, ("add_by_token", t[1], 1), Atom("a"))     # x = [{1, [t3, t1]}]
        st_.update(a, ("add_by_token", t[5], 1), Atom("a"))     # new output [t3, t5, t1]
        st_.result = st_.value(x)                               # merged: [t3, t1, t5, t1]
    assert exact_eq(ds.result, os_.result)
    toks = [tok for tok, _f in os_.result[0][1]]
    assert len(toks) != len(set(toks)), "the reference's merge duplicates a token here"


@SETTINGS
@given(SET, ELEM)
def test_value2_and_precondition_context(ops, e):
    """value/2 ({tokens, E}, {fragment, E}, removed) and precondition_context/1 on the
    device against the oracle (lasp_orset.erl:75-97, 147-154, 264-267)."""
    from lasp_amd import orset as do
    s = build(ops, 3)
    for q in (("tokens", e), ("fragment", e), "removed"):
        assert exact_eq(do.value2(q, s), oorset.value2(q, s)), q
    assert exact_eq(do.precondition_context(s), oorset.precondition_context(s))
