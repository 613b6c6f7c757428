#!/usr/bin/env python3
"""One list bind/3 (laspj_list_bind) of config 5's 50k-entry intersection output,
repeated: run it under `rocprofv3 --kernel-trace --stats` to see the kernels, memsets
and copies of one call and the gaps between them (tools/list_bench.py builds the same
lists).  SHAPE = sorted (default) | reversed | shuffled_same | shuffled_each; CHUNK =
rows per chunk of the chunked walk (LASPJ_TUNE_LIST_CHUNK, 0 = default); ITERS."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lasp_amd import _lib, engine  # noqa: E402
from list_bench import cells, identity_order, intersection_list  # noqa: E402

ctx = engine.Context(0)
shape = os.environ.get("SHAPE", "sorted")
chunk = int(os.environ.get("CHUNK", "0"))
ctx.set_tuning(_lib.TUNE_LIST_CHUNK, chunk)
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


def perm(l, p):
    runs = [l[2][l[1][i]:l[1][i + 1]] for i in range(len(l[0]))]
    return (l[0][p].copy(), np.concatenate([[0], np.cumsum([len(runs[i]) for i in p])]).astype(np.uint32),
            np.concatenate([runs[i] for i in p]))


n = len(common)
if shape == "reversed":
    old, new = perm(old, np.arange(n)[::-1]), perm(new, np.arange(n)[::-1])
elif shape == "shuffled_same":
    p1 = rng.permutation(n)
    old, new = perm(old, p1), perm(new, p1)
elif shape == "shuffled_each":
    old, new = perm(old, rng.permutation(n)), perm(new, rng.permutation(n))
a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*old)
b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*new)
for _ in range(3):
    a.bind(b, order)
ctx.synchronize()
it = int(os.environ.get("ITERS", "30"))
t0 = time.perf_counter()
for _ in range(it):
    a.bind(b, order)
print(json.dumps({"shape": shape, "chunk": chunk, "us_bind": (time.perf_counter() - t0) * 1e6 / it}),
      flush=True)
