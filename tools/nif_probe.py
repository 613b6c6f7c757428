#!/usr/bin/env python3
"""One warm NIF-level merge (laspj_orset_etf_merge) of BASELINE config 1's two 10k-element
term_to_binary images, repeated: run it under `rocprofv3 --kernel-trace
--memory-copy-trace --hip-runtime-trace --stats` to see every kernel, copy and HIP call of
the call's single synchronisation, and the library's own stage counters."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402

n = int(os.environ.get("NIF_N", "10000"))
iters = int(os.environ.get("NIF_ITERS", "50"))
ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
ctx = engine.Context(0)
L = ctx.L
from lasp_amd import _lib  # noqa: E402
if os.environ.get("NIF_SEG"):                  # from_binary segment bytes (A/B)
    ctx.set_tuning(_lib.TUNE_ETF_SEG, int(os.environ["NIF_SEG"]))
if os.environ.get("NIF_ETF"):                  # writer variant (A/B; 5: the two-launch merge)
    ctx.set_tuning(_lib.TUNE_ETF_KERNEL, int(os.environ["NIF_ETF"]))
op, on, vd = C.c_void_p(), C.c_uint64(), C.c_int32()


def nif():
    check(L.laspj_orset_etf_merge(ctx.h, pa, len(pa), pb, len(pb), C.byref(op), C.byref(on),
                                  C.byref(vd)), ctx.h)


cold = os.environ.get("NIF_COLD") == "1"     # every call meets one new token
colds = []
for k in range(iters if cold else 0):
    tb2 = list(tb)
    e = 17 * k + 3
    tb2[e] = (e, sorted(tb[e][1] + [(b"N" + (k * 7919 + e).to_bytes(19, "big"), False)]))
    colds.append(etf.term_to_binary(tb2))


def nif_cold(k):
    check(L.laspj_orset_etf_merge(ctx.h, pa, len(pa), colds[k], len(colds[k]), C.byref(op),
                                  C.byref(on), C.byref(vd)), ctx.h)


for _ in range(5):
    nif()
s0 = ctx.nif_stats()
t0 = time.perf_counter()
for k in range(iters):
    nif_cold(k) if cold else nif()
us = (time.perf_counter() - t0) * 1e6 / iters
s1 = ctx.nif_stats()
print(json.dumps({"cold": cold, "us_per_merge": us, "bytes_in": len(pa) + len(pb), "bytes_out": on.value,
                  "stages_us": {k: (s1[k] - s0[k]) / iters / 1e3 for k in s1 if k.startswith("ns_")}}))
