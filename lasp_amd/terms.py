"""Erlang terms on the host side of the engine (what the NIF receives as ERL_NIF_TERMs).

Python encoding: int/float numbers, `Atom` (str subclass; Python True/False are the
atoms true/false), tuple, list, bytes (binaries).  `term_cmp` is Erlang's standard
term order (number < atom < ref < fun < port < pid < tuple < map < [] < list <
bitstring); the dictionaries order element slots and token slots with it so that
decoded orddicts come out sorted exactly like the reference's (`orddict` keeps keys in
term order).  A NIF would use enif_compare for the same purpose.
"""

from __future__ import annotations

from functools import cmp_to_key


class Atom(str):
    def __repr__(self) -> str:  # pragma: no cover
        return f"'{str.__str__(self)}'"


_RANK_NUM, _RANK_ATOM, _RANK_TUPLE, _RANK_NIL, _RANK_LIST, _RANK_BIN = 0, 1, 6, 8, 9, 10


def _rank(t) -> int:
    if isinstance(t, (bool, Atom)):
        return _RANK_ATOM
    if isinstance(t, (int, float)):
        return _RANK_NUM
    if isinstance(t, tuple):
        return _RANK_TUPLE
    if isinstance(t, list):
        return _RANK_LIST if t else _RANK_NIL
    if isinstance(t, (bytes, bytearray)):
        return _RANK_BIN
    raise TypeError(f"unsupported Erlang term: {t!r}")


def _name(a) -> bytes:
    if isinstance(a, bool):
        return b"true" if a else b"false"
    return str.__str__(a).encode()


def term_cmp(a, b) -> int:
    ra, rb = _rank(a), _rank(b)
    if ra != rb:
        return -1 if ra < rb else 1
    if ra == _RANK_NUM:
        return (a > b) - (a < b)
    if ra == _RANK_ATOM:
        x, y = _name(a), _name(b)
        return (x > y) - (x < y)
    if ra == _RANK_BIN:
        x, y = bytes(a), bytes(b)
        return (x > y) - (x < y)
    if ra == _RANK_NIL:
        return 0
    if ra == _RANK_TUPLE and len(a) != len(b):
        return -1 if len(a) < len(b) else 1
    for x, y in zip(a, b):
        c = term_cmp(x, y)
        if c:
            return c
    return (len(a) > len(b)) - (len(a) < len(b))


term_key = cmp_to_key(term_cmp)


def hkey(t):
    """Hashable key with Erlang `==` semantics (1 and 1.0 collide, as in orddict)."""
    r = _rank(t)
    if r == _RANK_NUM:
        return ("n", t)
    if r == _RANK_ATOM:
        return ("a", _name(t))
    if r == _RANK_BIN:
        return ("b", bytes(t))
    if r == _RANK_TUPLE:
        return ("t",) + tuple(hkey(x) for x in t)
    return ("l",) + tuple(hkey(x) for x in t)


def ekey(t):
    """Hashable key with Erlang `=:=` semantics (1 and 1.0 differ)."""
    r = _rank(t)
    if r == _RANK_NUM:
        return ("f" if isinstance(t, float) else "i", t)
    if r == _RANK_ATOM:
        return ("a", _name(t))
    if r == _RANK_BIN:
        return ("b", bytes(t))
    if r == _RANK_TUPLE:
        return ("t",) + tuple(ekey(x) for x in t)
    return ("l",) + tuple(ekey(x) for x in t)


def same_term(a, b) -> bool:
    """a =:= b for two terms already known to be `==` (equal hkeys)."""
    if a is b:
        return True
    ta = type(a)
    if ta is type(b) and ta in (int, bytes, Atom, str, bool):
        return True
    return ekey(a) == ekey(b)
