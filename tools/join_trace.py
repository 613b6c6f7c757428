#!/usr/bin/env python3
"""Per-launch times of consecutive joins right after allocation (clock ramp check)."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lasp_amd import engine  # noqa: E402

ctx = engine.Context(0)
R, E = 1 << 20, 4096
a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
t0 = time.perf_counter()
a.fill_synthetic(2)
b.fill_synthetic(3)
ctx.synchronize()
fill_s = time.perf_counter() - t0
evs = [ctx.event() for _ in range(41)]
evs[0].record()
for k in range(40):
    c.join(a, b)
    evs[k + 1].record()
ctx.synchronize()
ms = [round(evs[k].elapsed_ms(evs[k + 1]), 2) for k in range(40)]
print(json.dumps({"fill_s": round(fill_s, 3), "per_launch_ms": ms}))
time.sleep(2.0)                   # idle, then again
evs[0].record()
for k in range(10):
    c.join(a, b)
    evs[k + 1].record()
ctx.synchronize()
print(json.dumps({"after_2s_idle_ms": [round(evs[k].elapsed_ms(evs[k + 1]), 2) for k in range(10)]}))
