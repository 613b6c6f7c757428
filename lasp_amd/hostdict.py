"""ctypes view of the native host dictionary (laspj_dict_*, laspj_term_compare): the
NIF-side encoder of include/laspj.h "host dictionary", usable without a GPU."""

from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np

from . import _lib


def pack(payloads: Sequence[bytes]):
    blob = b"".join(payloads)
    offs = np.zeros((len(payloads) + 1,), np.uint64)
    offs[1:] = np.cumsum([len(p) for p in payloads])
    return blob, offs


class NativeDict:
    def __init__(self):
        self.L = _lib.load()
        self.h = C.c_void_p()
        _lib.check(self.L.laspj_dict_create(C.byref(self.h)))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.laspj_dict_destroy(self.h)
            self.h = None

    def add(self, kind: int, payloads: Sequence[bytes], tag: int = -1) -> np.ndarray:
        blob, offs = pack(payloads)
        st = np.zeros((max(1, len(payloads)),), np.int32)
        _lib.check(self.L.laspj_dict_add(self.h, kind, blob, offs.ctypes.data, len(payloads),
                                         tag, st.ctypes.data))
        return st[:len(payloads)]

    def info(self):
        n, eb, tb = C.c_uint32(), C.c_uint64(), C.c_uint64()
        _lib.check(self.L.laspj_dict_info(self.h, C.byref(n), C.byref(eb), C.byref(tb)))
        return n.value, eb.value, tb.value

    def export(self, E: int, tokens: bool = True):
        """(elem_blob, elem_off, elem_order, tok_blob, tok_off, tok_order) — the arrays of
        laspj_etf_dict_create / engine.ETFDict."""
        _n, eb, tb = self.info()
        elem_blob = C.create_string_buffer(max(1, eb))
        elem_off = np.zeros((E + 1,), np.uint32)
        elem_order = np.zeros((E,), np.uint32)
        tok_blob = C.create_string_buffer(max(1, tb)) if tokens else None
        tok_off = np.zeros((64 * E + 1,), np.uint32) if tokens else None
        tok_order = np.zeros((64 * E,), np.uint8) if tokens else None
        _lib.check(self.L.laspj_dict_export(
            self.h, E, elem_blob, elem_off.ctypes.data, elem_order.ctypes.data, tok_blob,
            tok_off.ctypes.data if tokens else None, tok_order.ctypes.data if tokens else None))
        return (elem_blob.raw[:eb], elem_off, elem_order,
                tok_blob.raw[:tb] if tokens else None, tok_off, tok_order)

    def encode(self, kind: int, payloads: Sequence[bytes], E: int, tag: int = -1, out=None):
        blob, offs = pack(payloads)
        wpr = 2 * E if kind == _lib.KIND_ORSET else (E + 63) // 64
        if out is None:
            out = np.zeros((len(payloads), wpr), np.uint64)
        st = np.zeros((max(1, len(payloads)),), np.int32)
        _lib.check(self.L.laspj_dict_encode(self.h, kind, blob, offs.ctypes.data, len(payloads),
                                            tag, E, out.ctypes.data, st.ctypes.data))
        return out, st[:len(payloads)]


def term_compare(a: bytes, b: bytes) -> int:
    L = _lib.load()
    out = C.c_int()
    _lib.check(L.laspj_term_compare(a, len(a), b, len(b), C.byref(out)))
    return out.value
