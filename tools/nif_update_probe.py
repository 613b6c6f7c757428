"""Per-call timing and NIF counters of update/4 and the binds that follow it (config 1's
shape), for finding where an update or a new-token bind spends its time."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402
from oracle import etf as oetf  # noqa: E402
from oracle.terms import Atom  # noqa: E402


def main():
    n = 10_000
    ctx = engine.Context(0)
    L = ctx.L
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
    uv = ctx.var("orset")
    uv.write(pa)
    uv.bind(pb)
    res, vd, nm = C.c_int32(), C.c_int32(), C.c_uint32()
    ei, el, mi = C.c_void_p(), C.c_uint64(), C.c_void_p()
    keys = ("device_passes", "registrations", "image_rebuilds", "image_patches", "ns_register",
            "ns_rebuild", "ns_stage_enqueue", "ns_stage_copy", "ns_device_wait", "ns_answers",
            "dict_resets", "fallbacks", "chain_redo_passes", "device_new_tokens")
    rows = []

    def stats():
        s = ctx.nif_stats()
        return {k: s[k] for k in keys}

    rep, far = uv.replica(), ctx.var("orset")
    _, img0 = uv.read()
    rep.write(img0)
    far.write(img0)
    st = C.c_int32()
    for k in range(12):
        # (LASPJ_PROBE_NEW=1: each update adds a new element — the rebuild path)
        el_ = n + k if os.environ.get("LASPJ_PROBE_NEW") == "1" else 97 * k
        op = oetf.term_to_binary((Atom("add"), el_))
        s0 = stats()
        t0 = time.perf_counter()
        check(L.laspj_var_etf_update(uv.h, op, len(op), C.byref(res), C.byref(ei), C.byref(el),
                                     C.byref(mi), C.byref(nm), C.byref(vd)), ctx.h)
        ctx.synchronize()
        t1 = time.perf_counter()
        s1 = stats()
        _, img = uv.read()
        t2 = time.perf_counter()
        check(L.laspj_var_etf_bind(rep.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        t3 = time.perf_counter()
        s2 = stats()
        check(L.laspj_var_etf_bind(far.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        t4 = time.perf_counter()
        s3 = stats()
        check(L.laspj_var_etf_bind(far.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        t5 = time.perf_counter()
        s4 = stats()
        rows.append({"k": k, "us_update": (t1 - t0) * 1e6, "us_read": (t2 - t1) * 1e6,
                     "us_bind_replica": (t3 - t2) * 1e6, "us_bind_far": (t4 - t3) * 1e6,
                     "us_bind_far_again": (t5 - t4) * 1e6,
                     "d_update": {x: s1[x] - s0[x] for x in keys},
                     "d_replica": {x: s2[x] - s1[x] for x in keys},
                     "d_far": {x: s3[x] - s2[x] for x in keys},
                     "d_far_again": {x: s4[x] - s3[x] for x in keys}})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
