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
if len(sys.argv) > 1 and sys.argv[1] == "c4":
    # fused config-4 stage (laspj_orset_gather_inflation, 1024 x 2^20 x T=3): grid cap
    import numpy as np
    del src, dst
    O, EE = 1024, 1 << 20
    s4, fold, prev = ctx.orset_batch(O, EE), ctx.orset_batch(O, 3 * EE), ctx.orset_batch(O, 3 * EE)
    s4.fill_synthetic(40, token_slots=3)
    prev.fill_synthetic(41, token_slots=3)
    fidx = ctx.buffer(4 * 3 * EE)
    fidx.upload(np.repeat(np.arange(EE, dtype=np.uint32), 3))
    out = ctx.buffer(O)
    L = ctx.L
    fused = lambda: _lib.check(L.laspj_orset_gather_inflation(ctx.h, fold.h, s4.h, fidx.h, prev.h, 1, out.h), ctx.h)  # noqa: E731
    res = {}
    for _ in range(3):
        for gpc in (0, 64, 128, 100000):
            ctx.set_tuning(_lib.TUNE_STREAM_GRID, min(256 * gpc, 1 << 20))
            res.setdefault(gpc, []).append(timed(ctx, fused, 5))
    for gpc, v in res.items():
        print(json.dumps({"kernel": "gather_inflation", "grid_per_cu": gpc or 32,
                          "ms": [round(x, 3) for x in v],
                          "frac_hbm_best": round(112 * O * EE / (min(v) / 1e3) / 8e12, 4)}), flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "groups":
    # FSM reduce over replica groups (N = 3 OR-Set, N = 4 G-Counter): flat sweep (0) vs
    # one-tile-per-block source-at-a-time (4)
    import numpy as np
    del src, dst
    g = (1 << 20) // 4
    s3, d3 = ctx.orset_batch(3 * g, E), ctx.orset_batch(g, E)
    s3.fill_synthetic(4)
    RG, A = 1 << 20, 1024
    ka, kr = ctx.gcounter_batch(RG, A), ctx.gcounter_batch(RG // 4, A)
    ka.fill_synthetic(7)
    refs = {}
    res = {}
    for _ in range(3):
        for knob in (0, 4):
            ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, knob)
            res.setdefault(("orset_n3", knob), []).append(timed(ctx, lambda: d3.reduce_from(s3, 3), 5))
            refs.setdefault(("o", knob), d3.download_range(0, 1 << 24))
            res.setdefault(("gcounter_n4", knob), []).append(timed(ctx, lambda: kr.reduce_from(ka, 4), 5))
            refs.setdefault(("g", knob), kr.download_range(0, 1 << 24))
    nb = {"orset_n3": 64 * g * E, "gcounter_n4": 10 * RG * A}
    for (k, knob), v in res.items():
        print(json.dumps({"kernel": k, "knob": knob, "ms": [round(x, 3) for x in v],
                          "frac_hbm_best": round(nb[k] / (min(v) / 1e3) / 8e12, 4)}), flush=True)
    print(json.dumps({"same": bool(np.array_equal(refs[("o", 0)], refs[("o", 4)]) and
                                   np.array_equal(refs[("g", 0)], refs[("g", 4)]))}))
    sys.exit(0)
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
