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
    n = 1 if op == "increment" else op[1]
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
