"""riak_dt_gcounter mirror over the engine: the G-Counter the ad counter's threshold
reads use (lasp_lattice.erl:87-90, 169-179, 273-275; riak_test/lasp_adcounter_orset_test).

riak_dt is a third-party dependency that the reference does not vendor; its published
G-Counter is an orddict Actor -> Count with merge = per-actor max and value = sum
(restated in oracle/core.py: _GCounter).  Here actors are slots of a host dictionary
and counts live in HBM (LASPJ_KIND_GCOUNTER).
"""

from __future__ import annotations

from .codec import Domain
from .orset import context


class FunctionClause(ValueError):
    """riak_dt_gcounter:update/3 has no clause for the operation (function_clause)."""


def increment_amount(op) -> int:
    """The N of `increment` / `{increment, N}`: riak_dt_gcounter takes an integer N > 0
    only; counts live in uint64 slots, so N >= 2^64 is refused (OverflowError) rather
    than truncated."""
    if op == "increment":
        return 1
    if isinstance(op, tuple) and len(op) == 2 and op[0] == "increment" and \
            isinstance(op[1], int) and not isinstance(op[1], bool) and op[1] > 0:
        if op[1] >= 1 << 64:
            raise OverflowError(f"increment {op[1]} does not fit a uint64 count")
        return op[1]
    raise FunctionClause(f"riak_dt_gcounter:update({op!r}, ...)")


def threshold_plan(threshold, strict: bool):
    """threshold_met(riak_dt_gcounter, V, T) (lasp_lattice.erl:87-90) is `T =< value(V)`
    (strict: `T < value(V)`) in Erlang term order, value(V) a non-negative integer.
    Returns (const, None) when T alone decides it, else (None, t) with `t =< value(V)`
    to run on the device (t a uint64):
      * a non-number T (atom, list -- new() = [] included --, tuple, binary ...) is
        above every number in term order: never met;
      * integers and floats compare numerically: T =< V iff ceil(T) =< V, and
        T < V iff floor(T) + 1 =< V;
      * t =< 0 is always met; t >= 2^64 is never met by a uint64 sum."""
    import math
    if isinstance(threshold, bool) or not isinstance(threshold, (int, float)):
        return False, None
    if isinstance(threshold, float):
        if math.isnan(threshold):
            return False, None
        if math.isinf(threshold):
            return threshold < 0, None
        t = math.floor(threshold) + 1 if strict else math.ceil(threshold)
    else:
        t = threshold + 1 if strict else threshold
    if t <= 0:
        return True, None
    if t >= 1 << 64:
        return False, None
    return None, t


def _batch(dom: Domain, states):
    for s in states:
        for actor, _n in s:
            dom.element_slot(actor)
    E = max(1, dom.size)
    b = context().gcounter_batch(len(states), E)
    import numpy as np
    host = np.zeros((len(states), E), dtype=np.uint64)
    for i, s in enumerate(states):
        for actor, n in s:
            host[i, dom.element_slot(actor, create=False)] = n
    b.upload(host)
    return b


def _decode(dom: Domain, counts):
    return [(dom.elements.terms[int(a)], int(counts[int(a)]))
            for a in dom.elements.order() if int(counts[int(a)])]


def new():
    return []


def value(c) -> int:
    dom = Domain()
    return int(_batch(dom, [c]).values()[0])


def update(op, actor, c):
    """increment | {increment, N}"""
    n = increment_amount(op)
    dom = Domain()
    dom.element_slot(actor)
    b = _batch(dom, [c])
    b.increment([(0, dom.element_slot(actor, create=False), n)])
    return ("ok", _decode(dom, b.download()[0]))


def merge(a, b):
    dom = Domain()
    A, B = _batch(dom, [a]), None
    B = _batch(dom, [b])
    if A.elements != B.elements:
        A = _batch(dom, [a])
    C = context().gcounter_batch(1, A.elements).join(A, B)
    return _decode(dom, C.download()[0])


def equal(a, b) -> bool:
    dom = Domain()
    A = _batch(dom, [a])
    B = _batch(dom, [b])
    if A.elements != B.elements:
        A = _batch(dom, [a])
    return bool(A.equal(B)[0])
