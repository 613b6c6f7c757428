"""Host-side G-Counter checks (no GPU): the increment / threshold arguments the mirror
validates before anything reaches the device, against the oracle's riak_dt_gcounter
restatement (oracle/core.py: _GCounter) and lasp_lattice.erl:87-90."""

import math

import pytest
from hypothesis import given, settings, strategies as st

from lasp_amd import gcounter as dg
from oracle import core as ocore, lattice as olat
from oracle.terms import Atom

SOAK = int(__import__("os").environ.get("LASPJ_SOAK", "1"))   # x examples for a soak run

THRESH = st.one_of(
    st.integers(min_value=-(1 << 70), max_value=1 << 70),
    st.floats(allow_nan=False, allow_infinity=True, width=64),
    st.just([]), st.just(Atom("undefined")), st.just(True), st.just(b"x"), st.just((1, 2)))


@settings(max_examples=400 * SOAK, deadline=None)
@given(THRESH, st.integers(min_value=0, max_value=(1 << 64) - 1), st.booleans())
def test_threshold_plan_matches_term_order(t, v, strict):
    """The plan (a constant, or a uint64 `t =< sum` run on the device) agrees with the
    oracle's term-order comparison for every threshold term and count sum."""
    const, dev_t = dg.threshold_plan(t, strict)
    got = const if const is not None else dev_t <= v
    counter = [(Atom("a"), v)] if v else []
    want = olat.threshold_met("riak_dt_gcounter", counter, ("strict", t) if strict else t)
    assert got == want, (t, v, strict)


@pytest.mark.parametrize("op", [("increment", 0), ("increment", -1), ("increment", 1.5),
                                ("increment", True), ("increment", "3"), ("incr", 1),
                                "decrement"])
def test_increment_rejects_bad_amounts(op):
    """riak_dt_gcounter:update takes `increment` or {increment, N}, N > 0 only: the mirror
    raises (function_clause) like the oracle instead of wrapping N into a uint64."""
    with pytest.raises(ValueError):
        dg.increment_amount(op)
    with pytest.raises(ValueError):
        ocore._GCounter.update(op, Atom("a"), [])


def test_increment_amounts_kept_whole():
    assert dg.increment_amount("increment") == 1
    assert dg.increment_amount(("increment", (1 << 32) + 5)) == (1 << 32) + 5
    with pytest.raises(OverflowError):
        dg.increment_amount(("increment", 1 << 64))


def test_threshold_plan_edges():
    assert dg.threshold_plan(-1, False) == (True, None)       # -1 =< 0 always
    assert dg.threshold_plan([], False) == (False, None)      # new() = [] > numbers
    assert dg.threshold_plan(2.5, False) == (None, 3)
    assert dg.threshold_plan(2.5, True) == (None, 3)
    assert dg.threshold_plan(3, True) == (None, 4)
    assert dg.threshold_plan(1 << 64, False) == (False, None)
    assert dg.threshold_plan(-math.inf, True) == (True, None)
