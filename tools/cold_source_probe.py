"""A resident bind of one image, warm (the same bytes object each time) against cold (64
copies of it cycled, 30 MB: past the host's caches) — how much of an interleaved bind is
the host reading a cache-cold image into pinned staging."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402
from oracle import orset as oorset  # noqa: E402


def main():
    n = 10_000
    ctx = engine.Context(0)
    L = ctx.L
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    ref = etf.term_to_binary(oorset.merge(ta, tb))
    v = ctx.var("orset")
    v.write(ref)
    st, vd = C.c_int32(), C.c_int32()
    keys = ("ns_stage_enqueue", "ns_stage_copy", "ns_device_wait")

    def bind(img):
        t = time.perf_counter()
        check(L.laspj_var_etf_bind(v.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        return (time.perf_counter() - t) * 1e6

    copies = [bytes(bytearray(ref)) for _ in range(64)]
    out = {}
    for name, seq in (("warm", [ref] * 64), ("cold", copies), ("warm2", [ref] * 64)):
        for img in seq[:8]:
            bind(img)
        s0 = ctx.nif_stats()
        ts = [bind(img) for img in seq]
        s1 = ctx.nif_stats()
        out[name] = {"us": sorted(ts)[32], "per_bind_ns": {x: (s1[x] - s0[x]) / 64 for x in keys}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
