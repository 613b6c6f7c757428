#!/usr/bin/env python3
"""NIF-level value/1 (laspj_orset_etf_value) of config 1's 10k-element image and the
G-Set merge (laspj_gset_etf_merge) of two 10k-element ordsets, warm, repeated: the G-Set
writer's single long payload is the answer of both.  Prints us per call and the stages."""
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
ta = [(e, [(b"A" + e.to_bytes(19, "big"), e % 7 == 0)]) for e in range(n)]
ga, gb = list(range(0, 2 * n, 2)), list(range(0, 3 * n, 3))
pa, qa, qb = etf.term_to_binary(ta), etf.term_to_binary(ga), etf.term_to_binary(gb)
ctx = engine.Context(0)
L = ctx.L
op, on, vd = C.c_void_p(), C.c_uint64(), C.c_int32()
calls = {
    "us_orset_value": lambda: L.laspj_orset_etf_value(ctx.h, pa, len(pa), C.byref(op), C.byref(on), C.byref(vd)),
    "us_gset_merge": lambda: L.laspj_gset_etf_merge(ctx.h, qa, len(qa), qb, len(qb), C.byref(op), C.byref(on), C.byref(vd)),
    "us_gset_value": lambda: L.laspj_gset_etf_value(ctx.h, qa, len(qa), C.byref(op), C.byref(on), C.byref(vd)),
}
out = {"n": n}
for name, f in calls.items():
    for _ in range(5):
        check(f(), ctx.h)
    if vd.value != 0:
        raise SystemExit(f"{name}: verdict {vd.value}")
    s0 = ctx.nif_stats()
    t0 = time.perf_counter()
    for _ in range(iters):
        check(f(), ctx.h)
    out[name] = (time.perf_counter() - t0) * 1e6 / iters
    s1 = ctx.nif_stats()
    out[name + "_stages"] = {k: round((s1[k] - s0[k]) / iters / 1e3, 2) for k in s1 if k.startswith("ns_")}
    out[name + "_bytes_out"] = on.value
print(json.dumps(out))
