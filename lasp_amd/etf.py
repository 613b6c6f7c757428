"""External term format on the host side of the wire codec.

The device writes whole `to_binary/1` payloads (tag byte, version byte, then the
`term_to_binary/1` image of the orddict / ordset) from the columnar cells; what it
needs from the host is each dictionary term's own external image, which `encode`
produces once per distinct term (never per replica).  `decode` is `binary_to_term/1`
for the subset that appears on this path, used by `from_binary/1` (a NIF gets both
for free from the VM; here they stand in for it).

Encoding follows term_to_binary/1 of OTP 17-25 (minor_version 1): SMALL_INTEGER_EXT /
INTEGER_EXT / SMALL_BIG_EXT / LARGE_BIG_EXT, NEW_FLOAT_EXT, ATOM_EXT for latin-1
atoms, SMALL_TUPLE_EXT / LARGE_TUPLE_EXT, NIL_EXT, STRING_EXT for proper lists of
bytes shorter than 65536, LIST_EXT, BINARY_EXT.
"""

from __future__ import annotations

import struct
import zlib

from .terms import Atom

VERSION = 131
# riak_dt_tags.hrl is not vendored: the NIF passes ?DT_ORSET_TAG /
# ?DT_GSET_TAG from the header it is compiled against; these defaults are the values
# of riak_dt's tag header of that era as best known here (parity unpinned).
DT_ORSET_TAG = 76
DT_GSET_TAG = 82
V1_VERS = 1


class _W:
    __slots__ = ("b",)

    def __init__(self):
        self.b = bytearray()

    def term(self, t):
        b = self.b
        if isinstance(t, bool) or isinstance(t, Atom) or (isinstance(t, str)):
            name = ("true" if t else "false") if isinstance(t, bool) else str.__str__(t)
            try:
                raw = name.encode("latin-1")
                b.append(100)
                b += struct.pack(">H", len(raw))
            except UnicodeEncodeError:
                raw = name.encode("utf-8")
                if len(raw) < 256:
                    b += bytes((119, len(raw)))
                else:
                    b.append(118)
                    b += struct.pack(">H", len(raw))
            b += raw
        elif isinstance(t, int):
            if 0 <= t < 256:
                b += bytes((97, t))
            elif -0x80000000 <= t <= 0x7FFFFFFF:
                b.append(98)
                b += struct.pack(">i", t)
            else:
                mag = abs(t)
                n = (mag.bit_length() + 7) // 8
                if n < 256:
                    b += bytes((110, n))
                else:
                    b.append(111)
                    b += struct.pack(">I", n)
                b.append(1 if t < 0 else 0)
                b += mag.to_bytes(n, "little")
        elif isinstance(t, float):
            b.append(70)
            b += struct.pack(">d", t)
        elif isinstance(t, (bytes, bytearray)):
            b.append(109)
            b += struct.pack(">I", len(t))
            b += t
        elif isinstance(t, tuple):
            if len(t) < 256:
                b += bytes((104, len(t)))
            else:
                b.append(105)
                b += struct.pack(">I", len(t))
            for x in t:
                self.term(x)
        elif isinstance(t, list):
            if not t:
                b.append(106)
            elif len(t) < 65536 and all(type(x) is int and 0 <= x < 256 for x in t):
                b.append(107)
                b += struct.pack(">H", len(t))
                b += bytes(t)
            else:
                b.append(108)
                b += struct.pack(">I", len(t))
                for x in t:
                    self.term(x)
                b.append(106)
        else:
            raise ValueError(f"badarg: no external form for {t!r}")


def encode(t) -> bytes:
    """A term's external image WITHOUT the leading version byte (a fragment)."""
    w = _W()
    w.term(t)
    return bytes(w.b)


def is_byte(t) -> bool:
    """Whether the term is an integer STRING_EXT can carry (0..255)."""
    return type(t) is int and 0 <= t < 256


def term_to_binary(t) -> bytes:
    return bytes((VERSION,)) + encode(t)


class _R:
    __slots__ = ("b", "i")

    def __init__(self, b: bytes, i: int):
        self.b, self.i = b, i

    def take(self, n: int) -> bytes:
        j = self.i + n
        if j > len(self.b):
            raise ValueError("badarg: truncated external term")
        out = self.b[self.i:j]
        self.i = j
        return out

    def u8(self) -> int:
        return self.take(1)[0]

    def u16(self) -> int:
        return struct.unpack(">H", self.take(2))[0]

    def u32(self) -> int:
        return struct.unpack(">I", self.take(4))[0]

    def term(self):
        tag = self.u8()
        if tag == 97:
            return self.u8()
        if tag == 98:
            return struct.unpack(">i", self.take(4))[0]
        if tag == 110 or tag == 111:
            n = self.u8() if tag == 110 else self.u32()
            sign = self.u8()
            v = int.from_bytes(self.take(n), "little")
            return -v if sign else v
        if tag == 70:
            return struct.unpack(">d", self.take(8))[0]
        if tag == 100 or tag == 118 or tag == 119:
            n = self.u8() if tag == 119 else self.u16()
            name = self.take(n).decode("latin-1" if tag == 100 else "utf-8")
            return True if name == "true" else False if name == "false" else Atom(name)
        if tag == 104 or tag == 105:
            n = self.u8() if tag == 104 else self.u32()
            return tuple(self.term() for _ in range(n))
        if tag == 106:
            return []
        if tag == 107:
            return list(self.take(self.u16()))
        if tag == 108:
            n = self.u32()
            out = [self.term() for _ in range(n)]
            if self.u8() != 106:
                raise ValueError("badarg: improper list")
            return out
        if tag == 109:
            return bytes(self.take(self.u32()))
        raise ValueError(f"badarg: external tag {tag}")


def binary_to_term(b: bytes):
    """binary_to_term/1 for this path's terms (plain or zlib-compressed)."""
    b = bytes(b)
    if len(b) < 2 or b[0] != VERSION:
        raise ValueError("badarg: not an external term")
    if b[1] == 80:
        size = struct.unpack_from(">I", b, 2)[0]
        raw = zlib.decompress(b[6:])
        if len(raw) != size:
            raise ValueError("badarg: compressed size mismatch")
        b = bytes((VERSION,)) + raw
    r = _R(b, 1)
    t = r.term()
    if r.i != len(b):
        raise ValueError("badarg: trailing bytes")
    return t
