"""ctypes wrapper over oracle/build/liblaspj_oracle.so — TEST INFRASTRUCTURE ONLY.

The C restatement (laspj_oracle.c) works on the reference's orddict structure; these
helpers feed it columnar replicas (as produced by the engine) and compare results.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# LASPJ_ORACLE_SO selects another build of the same source (the sanitized one, run by
# tests/test_oracle_pin.py in a child process with libasan preloaded)
_SO = os.environ.get("LASPJ_ORACLE_SO") or os.path.join(_HERE, "build", "liblaspj_oracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)
u8p = C.POINTER(C.c_uint8)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        L.orc_synth_orset.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, u64p]
        L.orc_synth_orset_t.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_uint32, u64p]
        L.orc_synth_gset.argtypes = [C.c_uint64, C.c_uint64, C.c_uint32, u64p]
        L.orc_synth_tokens.argtypes = [C.c_uint32, C.c_uint32, u8p]
        L.orc_orset_alloc.argtypes = [C.c_uint32, C.c_uint32]
        L.orc_orset_alloc.restype = C.c_void_p
        L.orc_orset_free.argtypes = [C.c_void_p]
        L.orc_orset_nelem.argtypes = [C.c_void_p]
        L.orc_orset_nelem.restype = C.c_uint32
        L.orc_orset_ntok.argtypes = [C.c_void_p]
        L.orc_orset_ntok.restype = C.c_uint32
        L.orc_orset_from_cells.argtypes = [C.c_uint32, u64p, u8p, C.c_uint32, C.c_void_p]
        L.orc_orset_to_cells.argtypes = [C.c_void_p, C.c_uint32, u8p, C.c_uint32, u64p]
        L.orc_orset_merge.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_orset_equal.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_orset_value.argtypes = [C.c_void_p, i64p]
        L.orc_orset_value.restype = C.c_uint32
        L.orc_orset_stats.argtypes = [C.c_void_p, u64p]
        L.orc_orset_is_inflation.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_orset_is_strict.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_orset_union.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_orset_filter_even.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_gset_from_words.argtypes = [C.c_uint32, u64p, i64p]
        L.orc_gset_from_words.restype = C.c_uint32
        L.orc_gset_merge.argtypes = [i64p, C.c_uint32, i64p, C.c_uint32, i64p]
        L.orc_gset_merge.restype = C.c_uint32
        L.orc_bench_config1.argtypes = [C.c_uint32, C.c_int, C.POINTER(C.c_double),
                                        C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.orc_bench_orset_merge.argtypes = [C.c_uint32, C.c_uint64, C.c_int, C.c_uint32,
                                            C.c_double, C.POINTER(C.c_double), u64p,
                                            C.POINTER(C.c_double)]
        L.orc_bench_config1_ext.argtypes = [C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_double)]
        L.orc_bench_orset_op.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_int, C.c_uint32,
                                          C.c_double, C.POINTER(C.c_double), u64p,
                                          C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _p(a, t=u64p):
    return a.ctypes.data_as(t)


def synth_orset(seed: int, grep: int, E: int) -> np.ndarray:
    """Synthetic OR-Set replica as an (E, 2) uint64 array of {p, r} cells."""
    out = np.empty((E, 2), dtype=np.uint64)
    lib().orc_synth_orset(seed, grep, E, _p(out))
    return out


def synth_orset_t(seed: int, grep: int, e0: int, n: int, T: int) -> np.ndarray:
    """Elements [e0, e0+n) of the T-token stream replica (laspj_batch_fill_synthetic_tokens)
    as an (n, 2) uint64 array."""
    out = np.empty((n, 2), dtype=np.uint64)
    lib().orc_synth_orset_t(seed, grep, e0, n, T, _p(out))
    return out


def synth_gset(seed: int, grep: int, E: int) -> np.ndarray:
    out = np.empty(((E + 63) // 64,), dtype=np.uint64)
    lib().orc_synth_gset(seed, grep, E, _p(out))
    return out


def synth_tokens(E: int, T: int = 64) -> np.ndarray:
    out = np.empty((E, T, 20), dtype=np.uint8)
    lib().orc_synth_tokens(E, T, _p(out, u8p))
    return out


class ORDict:
    """An orddict-form OR-Set replica held by the C restatement."""

    def __init__(self, cap_elem: int, cap_tok: int):
        self.h = lib().orc_orset_alloc(cap_elem, cap_tok)
        if not self.h:
            raise MemoryError

    def __del__(self):
        if getattr(self, "h", None) and lib is not None:   # (module torn down at exit)
            lib().orc_orset_free(self.h)
            self.h = None

    @classmethod
    def from_cells(cls, cells: np.ndarray, tokens: np.ndarray) -> "ORDict":
        E, T = tokens.shape[0], tokens.shape[1]
        cells = np.ascontiguousarray(cells, dtype=np.uint64)
        d = cls(E, E * T)
        if lib().orc_orset_from_cells(E, _p(cells), _p(tokens, u8p), T, d.h) != 0:
            raise ValueError("capacity")
        return d

    def to_cells(self, tokens: np.ndarray) -> np.ndarray:
        E, T = tokens.shape[0], tokens.shape[1]
        out = np.empty((E, 2), dtype=np.uint64)
        if lib().orc_orset_to_cells(self.h, E, _p(tokens, u8p), T, _p(out)) != 0:
            raise ValueError("orddict not expressible over the dictionary")
        return out

    def merge(self, other: "ORDict") -> "ORDict":
        L = lib()
        out = ORDict(L.orc_orset_nelem(self.h) + L.orc_orset_nelem(other.h),
                     L.orc_orset_ntok(self.h) + L.orc_orset_ntok(other.h))
        if L.orc_orset_merge(self.h, other.h, out.h) != 0:
            raise ValueError("capacity")
        return out

    def union(self, other: "ORDict") -> "ORDict":
        """the lasp_orset union body (keep-left orddict:merge)"""
        L = lib()
        out = ORDict(L.orc_orset_nelem(self.h) + L.orc_orset_nelem(other.h),
                     L.orc_orset_ntok(self.h) + L.orc_orset_ntok(other.h))
        if L.orc_orset_union(self.h, other.h, out.h) != 0:
            raise ValueError("capacity")
        return out

    def filter_even(self) -> "ORDict":
        """the filter body with fun(X) -> X rem 2 == 0 end"""
        L = lib()
        out = ORDict(max(1, L.orc_orset_nelem(self.h)), max(1, L.orc_orset_ntok(self.h)))
        if L.orc_orset_filter_even(self.h, out.h) != 0:
            raise ValueError("capacity")
        return out

    def equal(self, other: "ORDict") -> bool:
        return bool(lib().orc_orset_equal(self.h, other.h))

    def value(self) -> np.ndarray:
        n = lib().orc_orset_nelem(self.h)
        keys = np.empty((max(n, 1),), dtype=np.int64)
        k = lib().orc_orset_value(self.h, _p(keys, i64p))
        return keys[:k].copy()

    def stats(self):
        out = np.zeros((3,), dtype=np.uint64)
        lib().orc_orset_stats(self.h, _p(out))
        return tuple(int(x) for x in out)

    def is_inflation_of(self, prev: "ORDict") -> bool:
        return bool(lib().orc_orset_is_inflation(prev.h, self.h))

    def is_strict_inflation_of(self, prev: "ORDict") -> bool:
        return bool(lib().orc_orset_is_strict(prev.h, self.h))


def gset_merge(a_words: np.ndarray, b_words: np.ndarray, E: int) -> np.ndarray:
    """ordsets:union of two integer G-Set replicas given as bitmaps; returns the merged
    ordset (ascending element ids)."""
    L = lib()
    a = np.empty((E,), dtype=np.int64)
    b = np.empty((E,), dtype=np.int64)
    na = L.orc_gset_from_words(E, _p(np.ascontiguousarray(a_words, dtype=np.uint64)), _p(a, i64p))
    nb = L.orc_gset_from_words(E, _p(np.ascontiguousarray(b_words, dtype=np.uint64)), _p(b, i64p))
    out = np.empty((na + nb,), dtype=np.int64)
    n = L.orc_gset_merge(_p(a, i64p), na, _p(b, i64p), nb, _p(out, i64p))
    return out[:n].copy()


def gset_members(words: np.ndarray, E: int) -> np.ndarray:
    a = np.empty((E,), dtype=np.int64)
    n = lib().orc_gset_from_words(E, _p(np.ascontiguousarray(words, dtype=np.uint64)), _p(a, i64p))
    return a[:n].copy()


def bench_orset_merge(E: int, seed: int, threads: int, pairs: int, budget_s: float):
    """Time the C restatement of lasp_orset:merge/2; returns (elements/s, merges, s)."""
    eps = C.c_double()
    merges = C.c_uint64()
    secs = C.c_double()
    rc = lib().orc_bench_orset_merge(E, seed, threads, pairs, budget_s, C.byref(eps),
                                     C.byref(merges), C.byref(secs))
    if rc != 0:
        raise RuntimeError("orc_bench_orset_merge failed")
    return eps.value, merges.value, secs.value


BENCH_OPS = {"merge": 0, "value": 1, "stats": 2, "inflation": 3, "strict_inflation": 4}


def bench_orset_op(op: str, E: int, seed: int, threads: int, pairs: int, budget_s: float):
    """Time one operation of the C restatement (BENCH_OPS) on synthetic replicas;
    returns (element slots/s, calls, s).  Inflation ops test merge(A, B) against A."""
    eps = C.c_double()
    calls = C.c_uint64()
    secs = C.c_double()
    rc = lib().orc_bench_orset_op(BENCH_OPS[op], E, seed, threads, pairs, budget_s,
                                  C.byref(eps), C.byref(calls), C.byref(secs))
    if rc != 0:
        raise RuntimeError("orc_bench_orset_op failed")
    return eps.value, calls.value, secs.value


def bench_config1(n: int = 10_000, iters: int = 200):
    """BASELINE config 1 on the C restatement: (us per merge, union, filter)."""
    m, u, f = C.c_double(), C.c_double(), C.c_double()
    if lib().orc_bench_config1(n, iters, C.byref(m), C.byref(u), C.byref(f)) != 0:
        raise RuntimeError("orc_bench_config1 failed")
    return m.value, u.value, f.value


def bench_config1_ext(n: int = 10_000, iters: int = 200, slow_iters: int = 5):
    """BASELINE config 1 on the C restatement, us per call: merge, union body, filter
    body, value/1, is_inflation(A, merge(A, B)) (quadratic keyfind, slow_iters calls)."""
    out = (C.c_double * 5)()
    if lib().orc_bench_config1_ext(n, iters, slow_iters, out) != 0:
        raise RuntimeError("orc_bench_config1_ext failed")
    return tuple(out)


def bench_config1_merge_threads(n: int, threads: int, budget_s: float) -> float:
    """BASELINE config 1's merge on `threads` host threads at once: wall microseconds per
    merge over all threads (the node-wide rate the batched NIF merges are set against)."""
    out = C.c_double()
    f = lib().orc_bench_config1_merge_threads
    f.argtypes = [C.c_uint32, C.c_int, C.c_double, C.POINTER(C.c_double)]
    if f(n, threads, budget_s, C.byref(out)) != 0:
        raise RuntimeError("orc_bench_config1_merge_threads failed")
    return out.value


def bench_cells_join(cells_per_thread: int, threads: int, budget_s: float) -> float:
    """The device's cell layout joined (d = a | b) on host threads: cells per second
    (a second CPU column for the headline; the reference's algorithm is bench_orset_merge)."""
    out = C.c_double()
    f = lib().orc_bench_cells_join
    f.argtypes = [C.c_uint64, C.c_int, C.c_double, C.POINTER(C.c_double)]
    if f(cells_per_thread, threads, budget_s, C.byref(out)) != 0:
        raise RuntimeError("orc_bench_cells_join failed")
    return out.value
