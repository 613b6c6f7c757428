"""lasp_gset mirror over the MI355X engine (src/lasp_gset.erl signatures).

States are ordsets (ascending lists).  Non-canonical lists — e.g. the `L ++ R` that the
reference's G-Set union combinator binds (lasp_core.erl:620) — raise NonCanonical.
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

from . import _lib, engine
from .codec import Domain
from .orset import context
from .terms import Atom


def _batch(dom: Domain, states: Sequence, E: int = 0) -> engine.GSetBatch:
    for s in states:
        for e in s:
            dom.element_slot(e)
    E = max(1, dom.size, E)
    b = context().gset_batch(len(states), E)
    b.upload(dom.encode_gset(states, E))
    return b


def new():
    """new/0 — lasp_gset.erl:70-72."""
    return []


def value(s):
    """value/1 — lasp_gset.erl:74-76 (ordsets:to_list)."""
    return list(s)


def value2(_query, s):
    """value/2 — lasp_gset.erl:78-81: not implemented in the reference, same as value/1."""
    return value(s)


def update4(op, actor, s, _ctx=None):
    """update/4 — lasp_gset.erl:90-93 (context ignored)."""
    return update(op, actor, s)


def parent_clock(_clock, s):
    """parent_clock/2 — lasp_gset.erl:95-97 (identity)."""
    return s


def to_version(_version, s):
    """to_version/2 — lasp_gset.erl:144-146 (identity)."""
    return s


def update(op, _actor, s):
    """update/3 — lasp_gset.erl:84-88: {add, E} | {add_all, Es} (device set-bit ops)."""
    dom = Domain()
    for e in s:
        dom.element_slot(e)
    if op[0] == "add":
        elems = [op[1]]
    elif op[0] == "add_all":
        elems = list(op[1])
    else:
        raise ValueError(f"function_clause: {op!r}")
    slots = [dom.element_slot(e) for e in elems]
    b = _batch(dom, [s])
    b.apply_ops([(0, es, _lib.OP_ADD, 0, _lib.OP_FLAG_NEW_CALL) for es in slots])
    return ("ok", dom.decode_gset(b.download()[0]))


def merge(a, b):
    """merge/2 — lasp_gset.erl:99-101 (device OR)."""
    return merge_many([(a, b)])[0]


def merge_many(pairs: Sequence[Tuple[list, list]]) -> List[list]:
    if not pairs:
        return []
    dom = Domain()
    for a, b in pairs:
        for e in list(a) + list(b):
            dom.element_slot(e)
    A = _batch(dom, [p[0] for p in pairs])
    B = _batch(dom, [p[1] for p in pairs])
    C = context().gset_batch(len(pairs), A.elements)
    C.join(A, B)
    out = C.download()
    return [dom.decode_gset(out[i]) for i in range(len(pairs))]


def equal(a, b) -> bool:
    """equal/2 — lasp_gset.erl:103-105."""
    dom = Domain()
    for e in list(a) + list(b):
        dom.element_slot(e)
    A, B = _batch(dom, [a]), _batch(dom, [b])
    return bool(A.equal(B)[0])


def stat(name, s):
    """stat/2 — lasp_gset.erl:134-142.  element_count on the device; max_element_size
    is a property of the element terms (erlang:external_size/1), which live on the
    host side of the boundary."""
    if name == "element_count":
        dom = Domain()
        return int(_batch(dom, [s]).stats()[0])
    if name == "max_element_size":
        return max((external_size(e) for e in s), default=0)
    return Atom("undefined")


def stats(s):
    return [(n, stat(n, s)) for n in ("element_count", "max_element_size")]


def external_size(t) -> int:
    """erlang:external_size/1 (OTP 17 estimate; binaries reserve 5 bytes for an
    unaligned tail, which the lasp_gset stat_test pins at 15 for <<"d234">>)."""
    return 1 + _ext(t)


def _ext(t) -> int:
    if isinstance(t, (bytes, bytearray)):
        return 1 + 4 + len(t) + 5
    if isinstance(t, (bool, Atom)):
        name = ("true" if t else "false") if isinstance(t, bool) else str.__str__(t)
        return 3 + len(name.encode())
    if isinstance(t, int):
        return 2 if 0 <= t <= 255 else 5
    if isinstance(t, tuple):
        return (2 if len(t) < 256 else 5) + sum(_ext(x) for x in t)
    if isinstance(t, list):
        return 1 if not t else 5 + sum(_ext(x) for x in t) + 1
    raise TypeError(t)


# --------------------------------------------------------------------------- wire codec

def to_binary(s, tag: int = None) -> bytes:
    """to_binary/1 — lasp_gset.erl:111: <<?TAG, ?V1_VERS, term_to_binary(S)>>,
    assembled on the device from the cells (laspj_gset_etf_write)."""
    from . import etf
    from .engine import ETFDict
    dom = Domain()
    b = _batch(dom, [s])
    E = b.elements
    d = ETFDict(context(), E, *dom.etf_arrays(E, tokens=False))
    return b.to_binaries(d, etf.DT_GSET_TAG if tag is None else tag, etf.V1_VERS)[0]


def to_binary2(vers, s):
    """to_binary/2: version 1 -> {ok, Bin}; else {error, unsupported_version, Vers}."""
    if vers == 1:
        return ("ok", to_binary(s))
    return ("error", "unsupported_version", vers)


def from_binary(b: bytes, tag: int = None):
    """from_binary/1 — lasp_gset.erl:111-128: binary_to_term of the payload after
    <<?TAG, 1>> wrapped in {ok, S};
    {error, unsupported_version, V} or {error, invalid_binary} otherwise."""
    from . import etf
    tag = etf.DT_GSET_TAG if tag is None else tag
    b = bytes(b)
    if len(b) >= 2 and b[0] == tag:
        if b[1] != etf.V1_VERS:
            return ("error", "unsupported_version", b[1])
        state = etf.binary_to_term(b[2:])
        return ("ok", state)
    return ("error", "invalid_binary")
