#!/usr/bin/env python3
"""Does the relative placement of the three join operands matter?  Carve A, B, C out of
one allocation at offsets 0, S+skew_b, 2S+skew_c and time the join for several skews."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lasp_amd import engine, _lib  # noqa: E402


class View(engine.ORSetBatch):
    def __init__(self, ctx, ptr, nbytes, R, E):
        self.ctx = ctx
        h = C.c_void_p()
        _lib.check(ctx.L.laspj_batch_wrap(ctx.h, _lib.KIND_ORSET, C.c_void_p(ptr), nbytes, R, E,
                                          C.byref(h)), ctx.h)
        self.h, self.replicas, self.elements = h, R, E
        self.bytes_per_replica, self.nbytes = 16 * E, nbytes


def main():
    R, E = 1 << 20, 4096
    S = 16 * R * E
    ctx = engine.Context(0)
    extra = 64 << 20
    buf = ctx.buffer(3 * S + 2 * extra)
    p = C.c_void_p()
    _lib.check(ctx.L.laspj_buf_device_ptr(buf.h, C.byref(p)))
    base = p.value
    skews = [(0, 0), (256, 512), (4096, 8192), (65536, 131072), (1 << 20, 2 << 20),
             ((2 << 20) + 4096, (4 << 20) + 8192), (8 << 20, 16 << 20), (4096 * 3, 4096 * 5)]
    ev0, ev1 = ctx.event(), ctx.event()
    for sb, sc in skews:
        a = View(ctx, base, S, R, E)
        b = View(ctx, base + S + sb, S, R, E)
        c = View(ctx, base + 2 * S + sc, S, R, E)
        a.fill_synthetic(2)
        b.fill_synthetic(3)
        for _ in range(2):
            c.join(a, b)
        ev0.record()
        for _ in range(8):
            c.join(a, b)
        ev1.record()
        ms = ev0.elapsed_ms(ev1) / 8
        print(json.dumps({"skew_b": sb, "skew_c": sc, "ms": round(ms, 3),
                          "GBps": round(48 * R * E / ms / 1e6, 1)}), flush=True)
        del a, b, c


if __name__ == "__main__":
    main()
