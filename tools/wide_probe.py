"""A hot element at config 1's size: 10k elements, one of them re-added (add_elem never
collects a token, lasp_orset.erl:222-241) to 10 tokens (past the element batches' 8) or
past 64 (the namespace's cells become k {p, r} pairs); per-call time of bind (no-op and
written), read, update, against the same calls with every element at 1 token."""
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
from oracle import orset as oorset  # noqa: E402
from oracle.terms import Atom  # noqa: E402


def timed(fn, k=20):
    fn()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    return (time.perf_counter() - t0) * 1e6 / k


def main():
    n = 10_000
    ctx = engine.Context(0)
    L = ctx.L
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
    out = {}
    for mode, adds in (("narrow", 0), ("t10", 9), ("wide", 70)):
        v = ctx.var("orset")
        v.write(pa)
        for k in range(adds):
            assert v.update(oetf.term_to_binary((Atom("add"), 7)))[0] == 0
        _, img = v.read()
        w = v.replica()
        w.write(img)
        st, vd = C.c_int32(), C.c_int32()
        s0 = ctx.nif_stats()
        r = {"bind_noop": timed(lambda: check(L.laspj_var_etf_bind(
                w.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)),
             "read": timed(lambda: w.read()),
             "update": timed(lambda: v.update(oetf.term_to_binary((Atom("add"), 11))), 10)}
        _, img2 = v.read()
        t0 = time.perf_counter()
        check(L.laspj_var_etf_bind(w.h, img2, len(img2), C.byref(st), C.byref(vd)), ctx.h)
        r["bind_written"] = (time.perf_counter() - t0) * 1e6
        r["verdict"] = vd.value
        r["widened"] = ctx.nif_stats()["namespaces_widened"]
        r["rebuilds"] = ctx.nif_stats()["image_rebuilds"] - s0["image_rebuilds"]
        out[mode] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
