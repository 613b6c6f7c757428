#!/usr/bin/env python3
"""from_binary/1 probe for counter runs: builds the two bench_suite etf workloads
(t64: 4096 x 1024 x 64 token slots, t3: 65536 x 256 x <= 3), writes their payloads on
the device and decodes them `--reps` times with the chosen read kernel
(LASPJ_TUNE_ETF_READ), printing one line per workload with the HIP-event time."""
import argparse
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from lasp_amd import _lib, engine                      # noqa: E402
from lasp_amd.codec import Domain                      # noqa: E402
from lasp_amd.orset import context                     # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--knob", type=int, default=0)
    ap.add_argument("--only", default="t64,t3")
    ap.add_argument("--op", default="read", choices=["read", "write"])
    ap.add_argument("--seg", default="0", help="comma list of LASPJ_TUNE_ETF_SEG values")
    a = ap.parse_args()
    ctx = context()
    L = ctx.L
    for tag, R, E, T in (("t64", 4096, 1024, 64), ("t3", 65536, 256, 3)):
        if tag not in a.only.split(","):
            continue
        b = ctx.orset_batch(R, E)
        if T == 64:
            b.fill_synthetic(9)
        else:
            rng = np.random.default_rng(3)
            h = np.zeros((R, E, 2), np.uint64)
            present = rng.random((R, E)) < 0.9
            h[:, :, 0] = np.where(present, rng.integers(1, 8, (R, E), dtype=np.uint64), 0)
            h[:, :, 1] = h[:, :, 0] & rng.integers(0, 8, (R, E), dtype=np.uint64) & \
                rng.integers(0, 8, (R, E), dtype=np.uint64)
            b.upload(h)
        dom = Domain()
        for e in range(E):
            es = dom.element_slot(e * 1000)
            for k in range(T):
                dom.token_slot(es, hashlib.blake2b(b"%d:%d" % (e, k), digest_size=20).digest())
        d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
        offs = ctx.buffer(8 * (R + 1))
        total = _lib.C.c_uint64()
        _lib.check(L.laspj_orset_etf_size(ctx.h, b.h, d.h, 76, offs.h, _lib.C.byref(total)),
                   ctx.h)
        out = ctx.buffer(total.value)
        _lib.check(L.laspj_orset_etf_write(ctx.h, b.h, d.h, 76, 1, offs.h, out.h), ctx.h)
        back = ctx.orset_batch(R, E)
        stb = ctx.buffer(4 * R)
        ev0, ev1 = ctx.event(), ctx.event()
        if a.op == "write":
            ctx.set_tuning(_lib.TUNE_ETF_KERNEL, a.knob)
            for _ in range(a.reps):
                ev0.record()
                _lib.check(L.laspj_orset_etf_write(ctx.h, b.h, d.h, 76, 1, offs.h, out.h), ctx.h)
                ev1.record()
                ctx.synchronize()
            ctx.set_tuning(_lib.TUNE_ETF_KERNEL, 0)
            _lib.check(L.laspj_orset_etf_read(ctx.h, back.h, d.h, 76, 1, out.h, offs.h, stb.h),
                       ctx.h)
            ok = np.array_equal(back.download(), b.download())
            print(f"{tag} write knob={a.knob} ms={ev0.elapsed_ms(ev1):.3f} payload={total.value} "
                  f"ok={ok}", flush=True)
            del back, stb, out, offs, d, b
            continue
        ctx.set_tuning(_lib.TUNE_ETF_READ, a.knob)
        for seg in [int(x) for x in a.seg.split(",")]:
            ctx.set_tuning(_lib.TUNE_ETF_SEG, seg)
            for _ in range(a.reps):
                ev0.record()
                _lib.check(L.laspj_orset_etf_read(ctx.h, back.h, d.h, 76, 1, out.h, offs.h,
                                                  stb.h), ctx.h)
                ev1.record()
                ctx.synchronize()
            ok = np.array_equal(back.download(), b.download())
            print(f"{tag} knob={a.knob} seg={seg} ms={ev0.elapsed_ms(ev1):.3f} "
                  f"payload={total.value} ok={ok}", flush=True)
        ctx.set_tuning(_lib.TUNE_ETF_READ, 0)
        ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)
        del back, stb, out, offs, d, b


if __name__ == "__main__":
    main()
