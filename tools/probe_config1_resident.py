import os, sys, json, time
sys.path.insert(0, os.getcwd())
import bench
from lasp_amd import engine, etf
n = 10_000
ctx = engine.Context(0)
ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
v = ctx.var("orset"); v.write(pa); v.bind(pb); ref = v.read()[1]; v.close()
t0 = time.perf_counter()
out = bench.config1_resident(ctx, pa, pb, ref)
print("total s", time.perf_counter() - t0)
print(json.dumps({k: v for k, v in out.items() if not isinstance(v, dict)}, indent=0))
print(json.dumps(ctx.nif_stats()))
