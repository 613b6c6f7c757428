"""The batched OR-Set join alone (lasp_orset:merge/2, lasp_orset.erl:128-134) for rocprofv3
kernel-trace and PMC passes: `steps` launches of laspj_orset_join over R replicas x E
element slots with k {p, r} pairs per cell (k = 1: BASELINE configs[1], T = 64 token slots;
k = 2: T = 128, LASPJ_KIND_ORSET_WIDE), synthetic operands resident in HBM."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lasp_amd import engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--replicas", type=int, default=1 << 19)
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    ctx = engine.Context(0)
    R, E, k = a.replicas, a.elements, a.k
    mk = (lambda: ctx.orset_batch(R, E)) if k == 1 else (lambda: ctx.orset_wide_batch(R, E, k))
    x, y, z = mk(), mk(), mk()
    x.fill_synthetic(2)
    y.fill_synthetic(3)
    z.join(x, y)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        z.join(x, y)
    ctx.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    algo = 48 * k * R * E
    gbs = algo / (ms / 1e3) / 1e9
    print(f"join k={k} R={R} E={E}: {ms:.3f} ms per launch (host clock), "
          f"{gbs:.1f} GB/s algorithmic = {gbs / 8000:.3f} of 8 TB/s")


if __name__ == "__main__":
    main()
