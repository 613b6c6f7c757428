"""Group commit against bind_many at config 1's shape: 16 threads binding through one
context (bench.py's bind_16thr_1ctx) and one caller's bind_many of the same batch size,
with the NIF counters per device pass — where a group-commit pass spends its time."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402
from oracle import orset as oorset  # noqa: E402

KEYS = ("ns_stage_enqueue", "ns_stage_copy", "ns_device_wait", "ns_answers", "ns_register",
        "ns_rebuild")


def per_pass(a, b):
    p = max(1, b["device_passes"] - a["device_passes"])
    return {"passes": b["device_passes"] - a["device_passes"],
            **{k: round((b[k] - a[k]) / p / 1e3, 1) for k in KEYS}}


def main():
    n = 10_000
    ctx = engine.Context(0)
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
    ref = etf.term_to_binary(oorset.merge(ta, tb))
    s0 = ctx.nif_stats()
    gc = bench._bind_threads(ctx, 16, 60, ref, pb, shared=True)
    s1 = ctx.nif_stats()
    out = {"group_commit": gc, "gc_per_pass_us": per_pass(s0, s1)}
    k = max(1, round(gc["binds_per_pass"]))
    vs = [ctx.var("orset") for _ in range(k)]
    for v in vs:
        v.write(ref)
    arr_v = (C.c_void_p * k)(*[v.h.value for v in vs])
    arr_p = (C.c_char_p * k)(*([pb] * k))
    arr_n = (C.c_uint64 * k)(*([len(pb)] * k))
    sts, vds = (C.c_int32 * k)(), (C.c_int32 * k)()
    check(ctx.L.laspj_var_etf_bind_many(ctx.h, k, arr_v, arr_p, arr_n, sts, vds), ctx.h)
    s2 = ctx.nif_stats()
    t0 = time.perf_counter()
    for _ in range(20):
        check(ctx.L.laspj_var_etf_bind_many(ctx.h, k, arr_v, arr_p, arr_n, sts, vds), ctx.h)
    dt = time.perf_counter() - t0
    s3 = ctx.nif_stats()
    out["bind_many"] = {"batch": k, "us_per_bind": dt * 1e6 / (20 * k),
                        "per_pass_us": per_pass(s2, s3)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
