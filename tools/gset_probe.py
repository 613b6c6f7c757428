"""G-Set resident variables at config 1's size (10k elements): per-call time of update/4
adding a new element, a bind of a state carrying one new element, a warm bind — where
every new element is a new dictionary term."""
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
    base = list(range(0, 2 * n, 2))
    v = ctx.var("gset")
    assert v.write(etf.term_to_binary(base)) == 0
    w = v.replica()
    assert w.write(etf.term_to_binary(base)) == 0
    far = ctx.var("gset")
    assert far.write(etf.term_to_binary(base)) == 0
    st, vd = C.c_int32(), C.c_int32()
    keys = ("device_passes", "registrations", "image_rebuilds", "image_patches", "ns_rebuild")
    out = {"update_new": [], "bind_replica": [], "bind_far": [], "stats": []}
    for k in range(8):
        s0 = ctx.nif_stats()
        t0 = time.perf_counter()
        assert v.update(oetf.term_to_binary((Atom("add"), 2 * n + 2 * k + 1)))[0] == 0
        t1 = time.perf_counter()
        _, img = v.read()
        t2 = time.perf_counter()
        check(L.laspj_var_etf_bind(w.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        t3 = time.perf_counter()
        check(L.laspj_var_etf_bind(far.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        t4 = time.perf_counter()
        s1 = ctx.nif_stats()
        out["update_new"].append(round((t1 - t0) * 1e6, 1))
        out["bind_replica"].append(round((t3 - t2) * 1e6, 1))
        out["bind_far"].append(round((t4 - t3) * 1e6, 1))
        out["stats"].append({x: s1[x] - s0[x] for x in keys})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
