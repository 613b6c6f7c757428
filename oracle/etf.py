"""Erlang external term format — oracle restatement (TEST INFRASTRUCTURE).

`lasp_orset:to_binary/1` (src/lasp_orset.erl:198-200) and `lasp_gset:to_binary/1`
(src/lasp_gset.erl:111-113) are `<<?TAG:8, ?V1_VERS:8, (riak_dt:to_binary(S))/binary>>`
and `riak_dt:to_binary/1` is `term_to_binary/2` (riak_dt is an un-vendored dependency,
rebar.config:7, tag "develop").  This module restates what OTP 17's
`term_to_binary/1,2` emits for the terms on this path (the published external term
format, erts "External Term Format", minor_version 1 — the default from OTP 17 to
OTP 25) and `binary_to_term/1` for the same subset:

  97  SMALL_INTEGER_EXT  0..255            98  INTEGER_EXT   signed 32-bit
  110 SMALL_BIG_EXT      |n| < 2^2040      111 LARGE_BIG_EXT
  70  NEW_FLOAT_EXT      IEEE double, big-endian (minor_version 1)
  100 ATOM_EXT           latin-1 atoms (minor_version 1 never emits the UTF-8 forms for them)
  118 ATOM_UTF8_EXT / 119 SMALL_ATOM_UTF8_EXT  decoded only
  104 SMALL_TUPLE_EXT    arity < 256       105 LARGE_TUPLE_EXT
  106 NIL_EXT            []
  107 STRING_EXT         a proper list of 1..65535 integers in 0..255
  108 LIST_EXT           Length:32, Elements, Tail
  109 BINARY_EXT         Len:32, Data
  80  compressed         UncompressedSize:32, zlib stream  (term_to_binary(T, [{compressed, N}]))

Pinned by the format's published examples (tests/test_etf.py); the compressed form
depends on the zlib build and riak_dt's `binary_compression` setting, so parity of
compressed bytes is unpinned (decoding is exact either way).
"""

from __future__ import annotations

import struct
import zlib

from .terms import Atom, _rank

VERSION = 131


def _enc(t) -> bytes:
    r = _rank(t)
    if r == 1:                                   # atom (Python bools are true/false)
        name = ("true" if t else "false") if isinstance(t, bool) else str.__str__(t)
        try:
            b = name.encode("latin-1")
            return bytes([100]) + struct.pack(">H", len(b)) + b
        except UnicodeEncodeError:
            b = name.encode("utf-8")
            if len(b) < 256:
                return bytes([119, len(b)]) + b
            return bytes([118]) + struct.pack(">H", len(b)) + b
    if r == 0:
        if isinstance(t, float):
            return bytes([70]) + struct.pack(">d", t)
        if 0 <= t <= 255:
            return bytes([97, t])
        if -(1 << 31) <= t < (1 << 31):
            return bytes([98]) + struct.pack(">i", t)
        sign, mag = (1, -t) if t < 0 else (0, t)
        digits = mag.to_bytes((mag.bit_length() + 7) // 8, "little")
        if len(digits) < 256:
            return bytes([110, len(digits), sign]) + digits
        return bytes([111]) + struct.pack(">I", len(digits)) + bytes([sign]) + digits
    if r == 6:                                   # tuple
        body = b"".join(_enc(x) for x in t)
        if len(t) < 256:
            return bytes([104, len(t)]) + body
        return bytes([105]) + struct.pack(">I", len(t)) + body
    if r == 8:                                   # []
        return bytes([106])
    if r == 9:                                   # proper list
        if len(t) < 65536 and all(isinstance(x, int) and not isinstance(x, bool)
                                  and 0 <= x <= 255 for x in t):
            return bytes([107]) + struct.pack(">H", len(t)) + bytes(t)
        return bytes([108]) + struct.pack(">I", len(t)) + b"".join(_enc(x) for x in t) \
            + bytes([106])
    if r == 10:
        return bytes([109]) + struct.pack(">I", len(t)) + bytes(t)
    raise TypeError(f"no external form for {t!r} on this path")


def term_to_binary(t, compressed: int = 0) -> bytes:
    """term_to_binary/1 (compressed = 0) or term_to_binary(T, [{compressed, N}]):
    the zlib form is used only when it is smaller."""
    raw = _enc(t)
    if compressed:
        z = zlib.compress(raw, compressed)
        if len(z) + 5 < len(raw):
            return bytes([VERSION, 80]) + struct.pack(">I", len(raw)) + z
    return bytes([VERSION]) + raw


def _dec(b: bytes, i: int):
    tag = b[i]
    i += 1
    if tag == 97:
        return b[i], i + 1
    if tag == 98:
        return struct.unpack_from(">i", b, i)[0], i + 4
    if tag in (110, 111):
        if tag == 110:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack_from(">I", b, i)[0], i + 4
        sign = b[i]
        v = int.from_bytes(b[i + 1:i + 1 + n], "little")
        return (-v if sign else v), i + 1 + n
    if tag == 70:
        return struct.unpack_from(">d", b, i)[0], i + 8
    if tag in (100, 118):
        n = struct.unpack_from(">H", b, i)[0]
        s = b[i + 2:i + 2 + n].decode("latin-1" if tag == 100 else "utf-8")
        return _atom(s), i + 2 + n
    if tag == 119:
        n = b[i]
        return _atom(b[i + 1:i + 1 + n].decode("utf-8")), i + 1 + n
    if tag in (104, 105):
        if tag == 104:
            n, i = b[i], i + 1
        else:
            n, i = struct.unpack_from(">I", b, i)[0], i + 4
        out = []
        for _ in range(n):
            x, i = _dec(b, i)
            out.append(x)
        return tuple(out), i
    if tag == 106:
        return [], i
    if tag == 107:
        n = struct.unpack_from(">H", b, i)[0]
        return list(b[i + 2:i + 2 + n]), i + 2 + n
    if tag == 108:
        n = struct.unpack_from(">I", b, i)[0]
        i += 4
        out = []
        for _ in range(n):
            x, i = _dec(b, i)
            out.append(x)
        tail, i = _dec(b, i)
        if tail != []:
            raise ValueError("improper list")
        return out, i
    if tag == 109:
        n = struct.unpack_from(">I", b, i)[0]
        return bytes(b[i + 4:i + 4 + n]), i + 4 + n
    raise ValueError(f"badarg: external tag {tag}")


def _atom(s: str):
    if s == "true":
        return True
    if s == "false":
        return False
    return Atom(s)


def binary_to_term(b: bytes):
    """binary_to_term/1 (badarg on anything malformed or with trailing bytes)."""
    b = bytes(b)
    if not b or b[0] != VERSION:
        raise ValueError("badarg")
    if len(b) > 1 and b[1] == 80:
        n = struct.unpack_from(">I", b, 2)[0]
        raw = zlib.decompress(b[6:])
        if len(raw) != n:
            raise ValueError("badarg")
        b = bytes([VERSION]) + raw
    try:
        t, i = _dec(b, 1)
    except (IndexError, struct.error) as e:
        raise ValueError("badarg") from e
    if i != len(b):
        raise ValueError("badarg")
    return t


def to_binary(tag: int, vers: int, state, compressed: int = 0) -> bytes:
    """<<?TAG:8, ?V1_VERS:8, (riak_dt:to_binary(S))/binary>> — lasp_orset.erl:198-200,
    lasp_gset.erl:111-113."""
    return bytes([tag, vers]) + term_to_binary(state, compressed)
