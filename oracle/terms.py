"""Erlang term model and standard term order — oracle restatement (TEST INFRASTRUCTURE).

Python encoding of Erlang terms used throughout the oracle and the tests:
  integer / float  -> int / float           (bool is NOT a number here, see below)
  atom             -> Atom (a str subclass); Python True/False are the atoms
                      `true` / `false` (the OR-Set token flags, lasp_orset.erl:131-133)
  tuple            -> tuple
  list / []        -> list
  binary           -> bytes

Term order (Erlang reference manual, restated in SURVEY.md Appendix A):
  number < atom < reference < fun < port < pid < tuple < map < [] < list < bitstring
  * numbers compare arithmetically (1 == 1.0 under `==`, `<`, `>`; different under `=:=`)
  * atoms by name; tuples by size then element-wise; lists element-wise, a proper
    prefix is smaller; binaries byte-wise, a prefix is smaller.
This order is what `orddict` / `ordsets` / `lists:sort` use (otp.py).
"""

from __future__ import annotations


class Atom(str):
    """An Erlang atom (compared by name)."""

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        return f"'{str.__str__(self)}'"


def atom(name: str) -> Atom:
    return Atom(name)


_NUM, _ATOM, _TUPLE, _MAP, _NIL, _LIST, _BIN = 0, 1, 6, 7, 8, 9, 10


def _rank(t) -> int:
    if isinstance(t, (bool, str)):      # any str subclass is an atom (product's too)
        return _ATOM
    if isinstance(t, (int, float)):
        return _NUM
    if isinstance(t, tuple):
        return _TUPLE
    if isinstance(t, dict):
        return _MAP
    if isinstance(t, list):
        return _LIST if t else _NIL
    if isinstance(t, (bytes, bytearray)):
        return _BIN
    raise TypeError(f"not an Erlang term: {t!r}")


def _atom_name(t) -> str:
    if isinstance(t, bool):
        return "true" if t else "false"
    return str.__str__(t)


def compare(a, b) -> int:
    """Erlang term order: -1, 0 or 1 (0 means `a == b`, arithmetic equality)."""
    # Iterative over list spines so 10^5-element lists do not recurse.
    while True:
        ra, rb = _rank(a), _rank(b)
        if ra != rb:
            return -1 if ra < rb else 1
        if ra == _NUM:
            return (a > b) - (a < b)
        if ra == _ATOM:
            na, nb = _atom_name(a).encode(), _atom_name(b).encode()
            return (na > nb) - (na < nb)
        if ra == _BIN:
            ba, bb = bytes(a), bytes(b)
            return (ba > bb) - (ba < bb)
        if ra == _NIL:
            return 0
        if ra == _TUPLE:
            if len(a) != len(b):
                return -1 if len(a) < len(b) else 1
            for x, y in zip(a, b):
                c = compare(x, y)
                if c:
                    return c
            return 0
        if ra == _LIST:
            n = min(len(a), len(b))
            for i in range(n):
                c = compare(a[i], b[i])
                if c:
                    return c
            # compare the remaining tails: [] vs non-empty list
            a, b = a[n:], b[n:]
            continue
        if ra == _MAP:
            raise TypeError("maps are not used on this path")


def lt(a, b) -> bool:
    return compare(a, b) < 0


def gt(a, b) -> bool:
    return compare(a, b) > 0


def eq(a, b) -> bool:
    """Erlang `==` (arithmetic equality)."""
    return compare(a, b) == 0


def exact_eq(a, b) -> bool:
    """Erlang `=:=` (no int/float coercion)."""
    ra, rb = _rank(a), _rank(b)
    if ra != rb:
        return False
    if ra == _NUM:
        return type(a) is type(b) and a == b
    if ra == _ATOM:
        return _atom_name(a) == _atom_name(b)
    if ra == _BIN:
        return bytes(a) == bytes(b)
    if ra == _NIL:
        return True
    if ra in (_TUPLE, _LIST):
        return len(a) == len(b) and all(exact_eq(x, y) for x, y in zip(a, b))
    raise TypeError("maps are not used on this path")


class Key:
    """Sort key wrapper implementing Erlang term order (for sorted())."""

    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def __lt__(self, other: "Key") -> bool:
        return compare(self.t, other.t) < 0

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Key) and compare(self.t, other.t) == 0
