import json, os, sys, time
import numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tools")
from lasp_amd import _lib, engine
from list_bench import cells, identity_order, intersection_list
ctx = engine.Context(0)
rng = np.random.default_rng(5)
N, D = 100_000, 150_000
order, keep = identity_order(ctx, D)
common = np.arange(D - N, N)
pl, rl = cells(rng, len(common)); pr, rr = cells(rng, len(common))
old = intersection_list(common, pl, rl, pr, rr)
pr2, rr2 = pr.copy(), rr.copy()
pr2[rng.random(len(common)) < 0.10] |= np.uint64(8)
rm = rng.random(len(common)) < 0.05
rr2[rm] = pr2[rm]
new = intersection_list(common, pl, rl, pr2, rr2)
def perm(l, p):
    runs = [l[2][l[1][i]:l[1][i + 1]] for i in range(len(l[0]))]
    return (l[0][p].copy(), np.concatenate([[0], np.cumsum([len(runs[i]) for i in p])]).astype(np.uint32), np.concatenate([runs[i] for i in p]))
p1, p2 = rng.permutation(len(common)), rng.permutation(len(common))
o, n = perm(old, p1), perm(new, p2)
ce = max(len(o[0]), len(n[0])); ct = max(len(o[2]), len(n[2]))
for caps in (True, False):
    if caps:
        a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, 1, ce, ct); b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST, 1, ce, ct)
        a.upload(*o, replica=0); b.upload(*n, replica=0)
    else:
        a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*o); b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*n)
    ts = []
    for k in range(12):
        t0 = time.perf_counter(); a.bind(b, order); ctx.synchronize(); ts.append((time.perf_counter() - t0) * 1e6)
    print(json.dumps({"caps": caps, "us": [round(t, 1) for t in ts]}), flush=True)
