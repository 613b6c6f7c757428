#!/usr/bin/env python3
"""Sweep the streaming-kernel knobs of laspj_orset_join at the bench size in one
process (batches allocated once).  Prints one JSON line per variant."""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import engine  # noqa: E402
from lasp_amd._lib import TUNE_STREAM_GRID, TUNE_STREAM_NT, TUNE_STREAM_UNROLL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=1 << 20)
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--grids", default="1024,2048,4096,8192")
    ap.add_argument("--unrolls", default="1,2,4,8")
    ap.add_argument("--nts", default="1,0")
    args = ap.parse_args()
    R, E = args.replicas, args.elements
    ctx = engine.Context(0)
    a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    ev0, ev1 = ctx.event(), ctx.event()
    for nt in [int(x) for x in args.nts.split(",")]:
        for g in [int(x) for x in args.grids.split(",")]:
            for u in [int(x) for x in args.unrolls.split(",")]:
                ctx.set_tuning(TUNE_STREAM_GRID, g)
                ctx.set_tuning(TUNE_STREAM_UNROLL, u)
                ctx.set_tuning(TUNE_STREAM_NT, nt)
                c.join(a, b)
                ev0.record()
                for _ in range(args.steps):
                    c.join(a, b)
                ev1.record()
                ms = ev0.elapsed_ms(ev1) / args.steps
                gbs = 48 * R * E / (ms / 1e3) / 1e9
                print(json.dumps({"nt": nt, "grid": g, "unroll": u, "ms": round(ms, 3),
                                  "GBps": round(gbs, 1)}), flush=True)


if __name__ == "__main__":
    main()
