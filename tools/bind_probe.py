#!/usr/bin/env python3
"""One warm resident bind (laspj_var_etf_bind) of BASELINE config 1's 10k-element image B
into a variable holding A ⊔ B, repeated: run it under `rocprofv3 --kernel-trace --stats`
to see every kernel of the call's single synchronisation, and the library's own stage
counters (host staging, enqueue, device wait).  BIND_MANY=n: n variables per call."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402

n = int(os.environ.get("BIND_N", "10000"))
iters = int(os.environ.get("BIND_ITERS", "200"))
many = int(os.environ.get("BIND_MANY", "1"))
ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
ctx = engine.Context(0)
L = ctx.L
if os.environ.get("BIND_SEG"):                 # from_binary segment bytes (A/B)
    from lasp_amd import _lib  # noqa: E402
    ctx.set_tuning(_lib.TUNE_ETF_SEG, int(os.environ["BIND_SEG"]))
vs = [ctx.var("orset") for _ in range(many)]
for v in vs:
    assert v.write(pa) == 0 and v.bind(pb) == (0, 1)
arr_v = (C.c_void_p * many)(*[v.h.value for v in vs])
arr_p = (C.c_char_p * many)(*([pb] * many))
arr_n = (C.c_uint64 * many)(*([len(pb)] * many))
sts, vds = (C.c_int32 * many)(), (C.c_int32 * many)()


def bind():
    check(L.laspj_var_etf_bind_many(ctx.h, many, arr_v, arr_p, arr_n, sts, vds), ctx.h)


for _ in range(5):
    bind()
s0 = ctx.nif_stats()
t0 = time.perf_counter()
for _ in range(iters):
    bind()
us = (time.perf_counter() - t0) * 1e6 / iters
s1 = ctx.nif_stats()
assert all(vds[k] == 0 and sts[k] == 1 for k in range(many))
print(json.dumps({"us_per_call": us, "binds_per_call": many, "us_per_bind": us / many,
                  "bytes_in_per_bind": len(pb),
                  "stages_us": {k: (s1[k] - s0[k]) / iters / 1e3 for k in s1 if k.startswith("ns_")}}))
