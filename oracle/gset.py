"""lasp_gset restatement — oracle (TEST INFRASTRUCTURE).  Follows src/lasp_gset.erl."""

from __future__ import annotations

from . import otp


def new():
    """new/0 — lasp_gset.erl:70-72."""
    return otp.ordsets_new()


def value(s):
    """value/1 — lasp_gset.erl:74-76 (ordsets:to_list, the identity)."""
    return otp.ordsets_to_list(s)


def update(op, _actor, s):
    """update/3 — lasp_gset.erl:84-88."""
    if op[0] == "add":
        return ("ok", otp.ordsets_add_element(op[1], s))
    if op[0] == "add_all":
        return ("ok", otp.ordsets_union(s, otp.ordsets_from_list(op[1])))
    raise ValueError(f"function_clause: unknown op {op!r}")


def merge(a, b):
    """merge/2 — lasp_gset.erl:99-101."""
    return otp.ordsets_union(a, b)


def equal(a, b) -> bool:
    """equal/2 — lasp_gset.erl:103-105."""
    from .terms import eq
    return eq(list(a), list(b))


def stat(name, s):
    """stat/2 — lasp_gset.erl:134-142.  max_element_size uses erlang:external_size/1,
    supplied here for the term kinds on this path (ext_size)."""
    if name == "element_count":
        return len(s)
    if name == "max_element_size":
        return otp.ordsets_fold(lambda e, m: max(ext_size(e), m), 0, s)
    return None


def stats(s):
    return [(n, stat(n, s)) for n in ("element_count", "max_element_size")]


def ext_size(t) -> int:
    """erlang:external_size/1 for small ints, atoms and binaries: the 131 version byte
    plus ERTS's *maximum* encoding size estimate.  For a binary the estimate is
    1 tag + 4 length + bytes + 5 (reserved for an unaligned bit-binary), which is what
    the reference KAT pins: max_element_size of <<"d234">> = 15 (lasp_gset.erl:157)."""
    return 1 + _ext_body(t)


def _ext_body(t) -> int:
    from .terms import Atom
    if isinstance(t, (bytes, bytearray)):
        return 1 + 4 + len(t) + 5
    if isinstance(t, bool) or isinstance(t, Atom):
        name = ("true" if t else "false") if isinstance(t, bool) else str.__str__(t)
        return 3 + len(name.encode())       # ATOM_EXT / SMALL_ATOM_UTF8_EXT era: tag+len16
    if isinstance(t, int):
        if 0 <= t <= 255:
            return 2                        # SMALL_INTEGER_EXT
        if -(1 << 31) <= t < (1 << 31):
            return 5                        # INTEGER_EXT
        raise ValueError("bignums are not used on this path")
    if isinstance(t, tuple):
        hdr = 2 if len(t) < 256 else 5
        return hdr + sum(_ext_body(x) for x in t)
    if isinstance(t, list):
        if not t:
            return 1                        # NIL_EXT
        return 5 + sum(_ext_body(x) for x in t) + 1
    raise TypeError(t)
