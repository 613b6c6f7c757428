#!/usr/bin/env python3
"""One list bind/3 (laspj_list_bind) of config 5's 50k-entry intersection output,
repeated: run it under `rocprofv3 --kernel-trace --stats` to see the kernels, memsets
and copies of one call and the gaps between them (tools/list_bench.py builds the same
lists)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lasp_amd import _lib, engine  # noqa: E402
from list_bench import cells, identity_order, intersection_list  # noqa: E402

ctx = engine.Context(0)
rng = np.random.default_rng(5)
N, D = 100_000, 150_000
order, keep = identity_order(ctx, D)
common = np.arange(D - N, N)
pl, rl = cells(rng, len(common))
pr, rr = cells(rng, len(common))
old = intersection_list(common, pl, rl, pr, rr)
pr2, rr2 = pr.copy(), rr.copy()
pr2[rng.random(len(common)) < 0.10] |= np.uint64(8)
new = intersection_list(common, pl, rl, pr2, rr2)
a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*old)
b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*new)
for _ in range(3):
    a.bind(b, order)
ctx.synchronize()
it = int(os.environ.get("ITERS", "30"))
t0 = time.perf_counter()
for _ in range(it):
    a.bind(b, order)
print({"us_bind": (time.perf_counter() - t0) * 1e6 / it})
