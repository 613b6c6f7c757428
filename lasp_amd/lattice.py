"""lasp_lattice mirror: threshold_met / is_inflation / is_strict_inflation for the
lasp_orset, lasp_orset_gbtree and lasp_gset clauses (src/lasp_lattice.erl:62-75,
137-161, 212-253, 287-295), computed by the wave64 ballot kernels on the device.

The lasp_orset_gbtree clauses run the lasp_orset kernels on the same cells: inflation
is the same containment test; strict inflation has no `Prev == []` clause
(:217-233), but there an empty Prev makes `NewElements` (size 0 < size Cur) carry the
same answer, so the kernel's special case is immaterial; its `Ids =/= Ids1` also sees
token-tree shapes, which the host adds (orset_gbtree.shapes_differ)."""

from __future__ import annotations

from .codec import Domain
from .orset import context
from . import gset as _gset


def _pair(type_, prev, cur):
    dom = Domain()
    ctx = context()
    if type_ == "lasp_orset_gbtree":
        from .orset_gbtree import to_orddict
        prev, cur, type_ = to_orddict(prev), to_orddict(cur), "lasp_orset"
    if type_ == "lasp_orset":
        dom.register_orset(prev)
        dom.register_orset(cur)
        E = max(1, dom.size)
        P, C = ctx.orset_batch(1, E), ctx.orset_batch(1, E)
        P.upload(dom.encode_orset([prev], E))
        C.upload(dom.encode_orset([cur], E))
        return P, C
    if type_ == "lasp_gset":
        for e in list(prev) + list(cur):
            dom.element_slot(e)
        return _gset._batch(dom, [prev]), _gset._batch(dom, [cur])
    if type_ == "riak_dt_gcounter":
        from . import gcounter as _gc
        dom = Domain()
        P = _gc._batch(dom, [prev])
        C = _gc._batch(dom, [cur])
        if P.elements != C.elements:
            P = _gc._batch(dom, [prev])
        return P, C
    raise ValueError(f"type {type_!r} is not on the device path")


def is_inflation(type_, prev, cur) -> bool:
    """is_inflation/3 — lasp_lattice.erl:97-98."""
    P, C = _pair(type_, prev, cur)
    return bool(C.is_inflation_of(P)[0])


def is_strict_inflation(type_, prev, cur) -> bool:
    """is_strict_inflation/3 — lasp_lattice.erl:105-106.  lasp_orset_gbtree's `Ids =/=
    Ids1` (:217-233) compares token TREES: an element whose tree changed shape is
    changed too (the shapes are host terms; the device compares the contents)."""
    P, C = _pair(type_, prev, cur)
    if bool(C.is_inflation_of(P, strict=True)[0]):
        return True
    if type_ == "lasp_orset_gbtree":
        from .orset_gbtree import shapes_differ
        return shapes_differ(prev, cur) and bool(C.is_inflation_of(P)[0])
    return False


def threshold_met(type_, value, threshold) -> bool:
    """threshold_met/3 — lasp_lattice.erl:62-75: {strict, T} -> strict inflation of T;
    riak_dt_gcounter (:87-90): T =< value(V), strict T < value(V)."""
    if type_ == "riak_dt_gcounter":
        from . import gcounter as _gc
        strict = isinstance(threshold, tuple) and len(threshold) == 2 and \
            threshold[0] == "strict"
        const, t = _gc.threshold_plan(threshold[1] if strict else threshold, strict)
        if const is not None:
            return const
        b = _gc._batch(Domain(), [value])
        return bool(b.threshold_met(t, False)[0])
    if isinstance(threshold, tuple) and len(threshold) == 2 and threshold[0] == "strict":
        return is_strict_inflation(type_, threshold[1], value)
    return is_inflation(type_, threshold, value)
