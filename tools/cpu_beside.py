#!/usr/bin/env python3
"""The reference's CPU path timed beside each device kernel of the core OR-Set rows
(SURVEY.md §8a a1, a2, a6, a9, a10): lasp_orset:merge/2, value/1, stat/2 and the
lasp_lattice inflation / strict-inflation clauses.

CPU: the C restatement (oracle/laspj_oracle.c, kind "port": orddict two-finger
merges, lists:keyfind scans, 20-byte tokens) on all granted host threads for a
bounded time per row.  GPU: the engine kernel at 2^18 replicas x 4096 element slots
x 64 token slots, HIP events on the engine stream.  Both count element slots per
second (E per replica per call).  One JSON line per row."""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lasp_amd import engine  # noqa: E402
from lasp_amd import _lib  # noqa: E402
from oracle import columnar as orc  # noqa: E402  (the timed CPU restatement)


def timed(ctx, fn, steps):
    fn()
    ctx.synchronize()
    e0, e1 = ctx.event(), ctx.event()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    return e0.elapsed_ms(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=1 << 18)
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cpu-budget", type=float, default=3.0)
    a = ap.parse_args()
    try:
        cores = max(1, min(len(os.sched_getaffinity(0)), 16))
    except AttributeError:  # pragma: no cover
        cores = 1
    R, E = a.replicas, a.elements
    ctx = engine.Context(0)
    L = ctx.L
    A, B, C = (ctx.orset_batch(R, E) for _ in range(3))
    A.fill_synthetic(2)
    B.fill_synthetic(3)
    C.join(A, B)
    bits = ctx.buffer(R * ((E + 63) // 64) * 8)
    stats = ctx.buffer(R * 24)
    flags = ctx.buffer(R)
    gpu = {
        "merge": lambda: C.join(A, B),
        "value": lambda: _lib.check(L.laspj_orset_value(ctx.h, A.h, bits.h), ctx.h),
        "stats": lambda: _lib.check(L.laspj_orset_stats(ctx.h, A.h, stats.h), ctx.h),
        "inflation": lambda: _lib.check(
            L.laspj_orset_inflation(ctx.h, A.h, C.h, 0, flags.h), ctx.h),
        "strict_inflation": lambda: _lib.check(
            L.laspj_orset_inflation(ctx.h, A.h, C.h, 1, flags.h), ctx.h),
    }
    for op, fn in gpu.items():
        ms = timed(ctx, fn, a.steps)
        g = R * E / (ms / 1e3)
        # the quadratic keyfind clauses need far fewer replicas to fill the budget
        pairs = 2
        c, calls, secs = orc.bench_orset_op(op, E, 2, cores, pairs, a.cpu_budget)
        print(json.dumps({
            "row": op, "gpu_elements_per_s": g, "gpu_ms": round(ms, 3),
            "gpu_workload": f"{R} replicas x {E} slots x 64 token slots",
            "cpu_elements_per_s": c, "cpu_cores": cores, "cpu_kind": "port",
            "cpu_calls": calls, "cpu_s": round(secs, 2), "gpu_over_cpu": g / c,
        }), flush=True)


if __name__ == "__main__":
    main()
