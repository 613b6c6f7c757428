#!/usr/bin/env python3
"""Launch-shape sweep of the anti-entropy reduce (laspj_batch_reduce_chunks) at N = 8
(8 chunk-major copies of 98304 x 4096-slot objects, 51.5 GB read + 6.4 GB written per
launch) and N = 3 FSM reduce: workgroups per CU x cells per lane x non-temporal."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_suite import timed  # noqa: E402
from lasp_amd import _lib, engine  # noqa: E402

ctx = engine.Context(0)
E, q = 4096, 98304
src, dst = ctx.orset_batch(8 * q, E), ctx.orset_batch(q, E)
src.fill_synthetic(4)
nbytes = 16 * 9 * q * E
if len(sys.argv) > 1 and sys.argv[1] == "ab":
    # interleaved repeats: the default sweep against tiles of 4 cells (64 per CU / all)
    cfgs = {"sweep": (3, 0, 0), "tile4": (0, 0, 0), "tile2": (0, 2, 0), "tile8": (0, 8, 0)}
    res = {k: [] for k in cfgs}
    for _ in range(4):
        for k, (kn, un, gr) in cfgs.items():
            ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, kn)
            ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, un)
            ctx.set_tuning(_lib.TUNE_STREAM_GRID, gr)
            res[k].append(timed(ctx, lambda: dst.reduce_chunks(src, 8), 5))
    for k, v in res.items():
        print(json.dumps({"kernel": k, "ms": [round(x, 3) for x in v],
                          "frac_hbm_best": round(nbytes / (min(v) / 1e3) / 8e12, 4)}), flush=True)
    sys.exit(0)
ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, 3)          # the grid-stride sweep's shapes
for grid_per_cu in (0, 8, 16, 32, 128):
    for unroll in (1, 2):
        for nt in (1, 0):
            ctx.set_tuning(_lib.TUNE_STREAM_GRID, 256 * grid_per_cu)
            ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, unroll)
            ctx.set_tuning(_lib.TUNE_STREAM_NT, nt)
            ms = timed(ctx, lambda: dst.reduce_chunks(src, 8), 5)
            print(json.dumps({"kernel": "reduce_chunks_n8", "grid_per_cu": grid_per_cu or 64,
                              "unroll": unroll, "nt": nt, "ms": round(ms, 3),
                              "frac_hbm": round(nbytes / (ms / 1e3) / 8e12, 4)}), flush=True)
