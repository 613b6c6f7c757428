#!/usr/bin/env python3
"""Per-kernel and per-config measurements beyond bench.py's headline line.

Each line: kernel / workload, average launch time from HIP events on the engine's
stream, algorithmic bytes per launch (DESIGN.md §4 per-unit figures x units) and the
fraction of the 8 TB/s HBM peak.  Workloads:
  kernels at BASELINE config 2 size (2^20 replicas x 4096 slots unless noted);
  config 4: ad-counter dataflow map -> filter -> fold -> strict threshold over 1024
            OR-Set objects x 1M int elements x 3 tokens;
  config 5: intersection (1024 pairs x 150k slots, 50 % id overlap) and product
            (100k x 100k, 3 tokens: 4 B per cell written).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import engine  # noqa: E402
from lasp_amd import _lib  # noqa: E402

PEAK = 8000.0


def timed(ctx, fn, steps, warmup=3):
    for _ in range(warmup):
        fn()
    ctx.synchronize()
    e0, e1 = ctx.event(), ctx.event()
    e0.record()
    for _ in range(steps):
        fn()
    e1.record()
    return e0.elapsed_ms(e1) / steps


def report(name, ms, nbytes, units, unit_name, **extra):
    gbs = nbytes / (ms / 1e3) / 1e9
    d = {"kernel": name, "ms": round(ms, 4), "algorithmic_bytes": int(nbytes),
         "GBps": round(gbs, 1), "frac_hbm": round(gbs / PEAK, 4),
         unit_name: units / (ms / 1e3)}
    d.update(extra)
    print(json.dumps(d), flush=True)


def ctx_cus(ctx) -> int:
    return 256          # MI355X: 256 CUs (the grid knob takes workgroups)


def kernels(ctx, R, E, steps):
    a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    cells = R * E
    W = (E + 63) // 64
    report("orset_join", timed(ctx, lambda: c.join(a, b), steps), 48 * cells, cells, "cells_per_s")
    bits = ctx.buffer(R * W * 8)
    L = ctx.L
    report("orset_value", timed(ctx, lambda: _lib.check(L.laspj_orset_value(ctx.h, a.h, bits.h)), steps),
           16 * cells + R * W * 8, cells, "cells_per_s")
    ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, 8)      # value with 8 words in flight per lane
    report("orset_value_u8", timed(ctx, lambda: _lib.check(L.laspj_orset_value(ctx.h, a.h, bits.h)), steps),
           16 * cells + R * W * 8, cells, "cells_per_s")
    ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, 0)
    st = ctx.buffer(R * 24)
    report("orset_stats", timed(ctx, lambda: _lib.check(L.laspj_orset_stats(ctx.h, a.h, st.h)), steps),
           16 * cells + R * 24, cells, "cells_per_s")
    o = ctx.buffer(R)
    for strict in (0, 1):
        c.join(a, b)
        report(f"orset_inflation_strict{strict}",
               timed(ctx, lambda: _lib.check(L.laspj_orset_inflation(ctx.h, a.h, c.h, strict, o.h)), steps),
               32 * cells + R, cells, "cells_per_s")
    report("orset_equal", timed(ctx, lambda: _lib.check(L.laspj_orset_equal(ctx.h, a.h, c.h, o.h)), steps),
           32 * cells + R, cells, "cells_per_s")
    report("orset_union", timed(ctx, lambda: c.union(a, b), steps), 48 * cells, cells, "cells_per_s")
    keep = ctx.buffer(W * 8)
    keep.upload(np.full((W,), 0x5555555555555555, np.uint64))
    report("orset_filter", timed(ctx, lambda: _lib.check(L.laspj_orset_filter(ctx.h, c.h, a.h, keep.h)), steps),
           32 * cells, cells, "cells_per_s")
    idx = ctx.buffer(4 * E)
    idx.upload(np.arange(E, dtype=np.uint32)[::-1].copy())
    report("orset_gather", timed(ctx, lambda: _lib.check(L.laspj_orset_gather(ctx.h, c.h, a.h, idx.h)), steps),
           32 * cells, cells, "cells_per_s")
    del c
    # FSM N-way merge: groups of N=3 replicas (lasp_update_fsm.erl:189-192)
    g = R // 4
    src = ctx.orset_batch(3 * g, E)
    dst = ctx.orset_batch(g, E)
    src.fill_synthetic(4)
    for knob, name in ((0, "orset_reduce_n3"), (1, "orset_reduce_n3_segments"),
                       (2, "orset_reduce_n3_generic")):
        ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, knob)
        report(name, timed(ctx, lambda: dst.reduce_from(src, 3), steps),
               64 * g * E, g * E, "dst_cells_per_s")
    ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, 0)
    for grp in (2, 4):
        src2 = ctx.orset_batch(grp * (g // 2), E)
        dst2 = ctx.orset_batch(g // 2, E)
        report(f"orset_reduce_n{grp}_half", timed(ctx, lambda: dst2.reduce_from(src2, grp), steps),
               16 * (grp + 1) * (g // 2) * E, (g // 2) * E, "dst_cells_per_s")
        del src2, dst2
    # the same N = 3 fold with the replies laid out chunk-major (reply j of every group
    # contiguous, as the anti-entropy receive buffer is): laspj_batch_reduce_chunks
    report("orset_reduce_chunks_n3", timed(ctx, lambda: dst.reduce_chunks(src, 3), steps),
           64 * g * E, g * E, "dst_cells_per_s")
    del src, dst, a, b
    # the anti-entropy reduce at N = 8 (gossip round on 8 GPUs: 8 chunk-major copies)
    q = (3 * g) // 8
    src8, dst8 = ctx.orset_batch(8 * q, E), ctx.orset_batch(q, E)
    for knob, name in ((0, "orset_reduce_chunks_n8"), (2, "orset_reduce_chunks_n8_loop")):
        ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, knob)
        report(name, timed(ctx, lambda: dst8.reduce_chunks(src8, 8), steps),
               16 * 9 * q * E, q * E, "dst_cells_per_s")
    ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, 0)
    if os.environ.get("REDUCE_SWEEP"):
        # launch shape of the N = 8 reduce: grid (workgroups per CU) x cells per lane x NT
        for grid_per_cu in (8, 16, 32, 64, 128):
            for unroll in (1, 2):
                for nt in (1, 0):
                    ctx.set_tuning(_lib.TUNE_STREAM_GRID, ctx_cus(ctx) * grid_per_cu)
                    ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, unroll)
                    ctx.set_tuning(_lib.TUNE_STREAM_NT, nt)
                    report(f"orset_reduce_chunks_n8_g{grid_per_cu}_u{unroll}_nt{nt}",
                           timed(ctx, lambda: dst8.reduce_chunks(src8, 8), steps),
                           16 * 9 * q * E, q * E, "dst_cells_per_s")
        ctx.set_tuning(_lib.TUNE_STREAM_GRID, 0)
        ctx.set_tuning(_lib.TUNE_STREAM_UNROLL, 0)
        ctx.set_tuning(_lib.TUNE_STREAM_NT, -1)
    del src8, dst8
    h = R // 2                      # CONCAT output is 32 B per cell: half the replicas
    a2, b2 = ctx.orset_batch(h, E), ctx.orset_batch(h, E)
    a2.fill_synthetic(2)
    b2.fill_synthetic(3)
    x = a2.intersection(b2)
    report("orset_intersection", timed(ctx, lambda: _lib.check(
        L.laspj_orset_intersection(ctx.h, x.h, a2.h, b2.h)), steps), 64 * h * E, h * E, "cells_per_s")
    del x, a2, b2
    # G-Set at the same element count
    ga, gb, gc = (ctx.gset_batch(R, E) for _ in range(3))
    ga.fill_synthetic(5)
    gb.fill_synthetic(6)
    report("gset_join", timed(ctx, lambda: gc.join(ga, gb), steps), 24 * R * W, R * E, "elements_per_s")
    del ga, gb, gc
    # the same join at 16x the replicas (8 GiB per operand): the 0.3 ms launch above is
    # short enough for launch and tail to show; this one is the steady-state rate
    RL_ = 16 * R
    ga, gb, gc = (ctx.gset_batch(RL_, E) for _ in range(3))
    ga.fill_synthetic(5)
    gb.fill_synthetic(6)
    report("gset_join_16x", timed(ctx, lambda: gc.join(ga, gb), steps), 24 * RL_ * W, RL_ * E,
           "elements_per_s")
    del ga, gb, gc
    # riak_dt_gcounter (the ad counter's threshold counter): 2^20 replicas x 1024 actors
    RG, A = 1 << 20, 1024
    ka, kb, kc = (ctx.gcounter_batch(RG, A) for _ in range(3))
    ka.fill_synthetic(7)
    kb.fill_synthetic(8)
    n8 = RG * A * 8
    report("gcounter_join_max", timed(ctx, lambda: kc.join(ka, kb), steps), 3 * n8, RG * A,
           "actor_slots_per_s")
    sums = ctx.buffer(RG * 8)
    report("gcounter_value", timed(ctx, lambda: _lib.check(
        L.laspj_gcounter_value(ctx.h, kc.h, sums.h), ctx.h), steps), n8 + RG * 8, RG * A,
        "actor_slots_per_s")
    og = ctx.buffer(RG)
    report("gcounter_threshold", timed(ctx, lambda: _lib.check(
        L.laspj_gcounter_threshold(ctx.h, kc.h, 1 << 29, 0, og.h), ctx.h), steps), n8 + RG,
        RG * A, "actor_slots_per_s")
    report("gcounter_inflation", timed(ctx, lambda: _lib.check(
        L.laspj_gcounter_inflation(ctx.h, ka.h, kc.h, 0, og.h), ctx.h), steps), 2 * n8 + RG,
        RG * A, "actor_slots_per_s")
    # FSM N = 4 reduce of counters (per-actor max): flat sweep vs the generic kernel
    kr = ctx.gcounter_batch(RG // 4, A)
    for knob, name in ((0, "gcounter_reduce_n4"), (2, "gcounter_reduce_n4_generic")):
        ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, knob)
        report(name, timed(ctx, lambda: kr.reduce_from(ka, 4), steps), n8 + n8 // 4,
               (RG // 4) * A, "dst_slots_per_s")
    ctx.set_tuning(_lib.TUNE_REDUCE_KERNEL, 0)
    del kr
    del ka, kb, kc


def ops(ctx, steps):
    """update/3 throughput: 1M single-op calls spread over 2^20 replicas."""
    R, E = 1 << 20, 64
    b = ctx.orset_batch(R, E)
    rng = np.random.default_rng(0)
    n = 1 << 20
    reps = np.sort(rng.integers(0, R, n))
    arr = (_lib.Op * n)()
    el = rng.integers(0, E, n)
    sl = rng.integers(0, 64, n)
    kd = np.where(rng.random(n) < 0.8, _lib.OP_ADD, _lib.OP_REMOVE)
    for k in range(n):
        arr[k].replica, arr[k].element, arr[k].kind = int(reps[k]), int(el[k]), int(kd[k])
        arr[k].slot, arr[k].flags = int(sl[k]), 1
    st = np.zeros((n,), np.int32)
    ptr = st.ctypes.data_as(_lib.C.POINTER(_lib.C.c_int32))
    t0 = time.perf_counter()
    for _ in range(steps):
        _lib.check(ctx.L.laspj_orset_apply_ops(ctx.h, b.h, arr, n, ptr), ctx.h)
    dt = (time.perf_counter() - t0) / steps
    print(json.dumps({"kernel": "orset_apply_ops", "ms": round(dt * 1e3, 3), "ops": n,
                      "ops_per_s": n / dt, "note": "host->device op upload + status download included"}),
          flush=True)


def config4(ctx, objects, elements, steps):
    """BASELINE configs[3]: 1024 OR-Set objects x 2^20 int elements x T = 3 tokens
    (laspj_batch_fill_synthetic_tokens) through map X -> 2X, filter even, fold
    X -> [X, X, X] and the {strict, Prev} threshold read of the fold output.  The
    dictionary-level work (each fun evaluated once per element, composing the indexes)
    is host-side and not timed.
      staged: gather (map) -> filter -> gather (fold) -> strict inflation, every stage's
              output written: 16+16 + 16+16 + 16+48 + 48+48 = 224 B per input element
              (+ index / keep reads);
      fused:  laspj_orset_gather_inflation with the composed index o -> o // 3: src read
              once (16 B; each cell feeds 3 fold slots from cache), fold written (48 B),
              Prev read (48 B) = 112 B per input element.  The map / filter outputs are
              the same gather of src with their own indexes; they are produced on demand,
              not per step."""
    E, T = elements, 3
    src = ctx.orset_batch(objects, E)
    src.fill_synthetic(40, token_slots=T)
    mapped = ctx.orset_batch(objects, E)
    filt = ctx.orset_batch(objects, E)
    fold = ctx.orset_batch(objects, 3 * E)
    prev = ctx.orset_batch(objects, 3 * E)
    prev.fill_synthetic(41, token_slots=T)
    L = ctx.L
    ident = ctx.buffer(4 * E)
    ident.upload(np.arange(E, dtype=np.uint32))       # X -> 2X is monotone: slot order kept
    keep = ctx.buffer(((E + 63) // 64) * 8)
    keep.upload(np.full(((E + 63) // 64,), ~np.uint64(0), np.uint64))   # 2X is even
    fidx = ctx.buffer(4 * 3 * E)
    fidx.upload(np.repeat(np.arange(E, dtype=np.uint32), 3))
    out = ctx.buffer(objects)

    def staged():
        _lib.check(L.laspj_orset_gather(ctx.h, mapped.h, src.h, ident.h), ctx.h)
        _lib.check(L.laspj_orset_filter(ctx.h, filt.h, mapped.h, keep.h), ctx.h)
        _lib.check(L.laspj_orset_gather(ctx.h, fold.h, filt.h, fidx.h), ctx.h)
        _lib.check(L.laspj_orset_inflation(ctx.h, prev.h, fold.h, 1, out.h), ctx.h)
    cells = objects * E
    ms = timed(ctx, staged, steps)
    report("config4_dataflow", ms, 224 * cells, cells, "input_elements_per_s",
           objects=objects, elements=E, token_slots=T,
           stages="gather 32B + filter 32B + fold-gather 64B + strict inflation 96B per input element")
    del mapped, filt

    def fused():
        _lib.check(L.laspj_orset_gather_inflation(ctx.h, fold.h, src.h, fidx.h, prev.h, 1,
                                                  out.h), ctx.h)
    ms = timed(ctx, fused, steps)
    report("config4_dataflow_fused", ms, 112 * cells, cells, "input_elements_per_s",
           objects=objects, elements=E, token_slots=T,
           stages="src 16B read once + fold 48B written + Prev 48B read per input element")


def config5(ctx, steps):
    # intersection: 1024 pairs over a 150k-slot dictionary, each side 100k elements
    # L = elements [0, 100k), R = [50k, 150k): 100k-element sets (every element present,
    # T = 3 tokens) with 50 % id overlap, as tests/test_gpu_configs.py checks them
    P, E, N = 1024, 150_000, 100_000
    bl, br = ctx.orset_batch(P, E), ctx.orset_batch(P, E)
    bl.fill_synthetic(5, token_slots=3)
    br.fill_synthetic(6, token_slots=3)
    ids = np.arange(E)

    def bits(mask):
        b = np.packbits(mask.astype(np.uint8), bitorder="little")
        return np.concatenate([b, np.zeros((8 * ((E + 63) // 64) - len(b),), np.uint8)]).view(np.uint64)
    l = ctx.orset_batch(P, E).filter(bl, bits(ids < N))
    r = ctx.orset_batch(P, E).filter(br, bits(ids >= E - N))
    del bl, br
    x = l.intersection(r)
    L = ctx.L
    report("config5_intersection", timed(ctx, lambda: _lib.check(
        L.laspj_orset_intersection(ctx.h, x.h, l.h, r.h), ctx.h), steps),
        64 * P * E, P * E, "slots_per_s", pairs=P, slots=E)
    del x
    # the fused product + filter({X, Y} -> X =:= Y) variant over the same pairs: 32 B
    # read + 4 B written per slot instead of 1e10 product cells per pair
    dg = engine.ORSetProductBatch(ctx, P, E, 1)
    report("config5_product_diag", timed(ctx, lambda: _lib.check(
        L.laspj_orset_product_diag(ctx.h, dg.h, l.h, r.h), ctx.h), steps),
        36 * P * E, P * E, "slots_per_s", pairs=P, slots=E)
    del dg, l, r
    # product: 100k x 100k, T = 3 token slots
    n = 100_000
    pl, pr = ctx.orset_batch(1, n), ctx.orset_batch(1, n)
    pl.fill_synthetic(7, token_slots=3)
    pr.fill_synthetic(8, token_slots=3)
    out = engine.ORSetProductBatch(ctx, 1, n, n)
    for rows, cols in ((0, 0), (64, 0), (128, 0), (0, 2048), (0, 4096), (128, 4096)):
        ctx.set_tuning(_lib.TUNE_PRODUCT_ROWS, rows)     # 0 = default tile (256 x 1024)
        ctx.set_tuning(_lib.TUNE_PRODUCT_COLS, cols)
        ms = timed(ctx, lambda: pl.product(pr, out), steps)
        tag = (f"_rows{rows}" if rows else "") + (f"_cols{cols}" if cols else "")
        report("config5_product" + tag, ms, 4 * n * n + 32 * n, n * n, "cells_per_s",
               el=n, er=n)
    ctx.set_tuning(_lib.TUNE_PRODUCT_ROWS, 0)
    ctx.set_tuning(_lib.TUNE_PRODUCT_COLS, 0)
    del out, pl, pr
    # wide form (token slots >= 8: 32-byte cells {pX, rX, pY, rY}), 30k x 30k x 64 slots
    m = 30_000
    wl, wr = ctx.orset_batch(1, m), ctx.orset_batch(1, m)
    wl.fill_synthetic(7)
    wr.fill_synthetic(8)
    wout = engine.ORSetProductWideBatch(ctx, 1, m, m)
    ms = timed(ctx, lambda: wl.product(wr, wout), steps)
    report("config5_product_wide_30k", ms, 32 * m * m + 32 * m, m * m, "cells_per_s", el=m, er=m)


def etf(ctx, steps):
    """to_binary/1 payloads of whole batches: the size pass
    (cells read + a device scan) and the write pass (cells read, payload written).
    Shapes: (a) 4096 replicas x 1024 slots x 64 token slots (synthetic cells, ~32
    tokens per element); (b) 65536 replicas x 256 slots x <= 3 tokens.  Tokens are
    20-byte binaries, elements integers (SMALL_INTEGER_EXT / INTEGER_EXT images)."""
    import hashlib
    from lasp_amd.codec import Domain
    L = ctx.L
    steps = max(steps, 20)                    # ~1 ms kernels: average over more launches
    for tag, R, E, T in (("t64", 4096, 1024, 64), ("t3", 65536, 256, 3)):
        b = ctx.orset_batch(R, E)
        if T == 64:
            b.fill_synthetic(9)
        else:
            rng = np.random.default_rng(3)
            h = np.zeros((R, E, 2), np.uint64)
            present = rng.random((R, E)) < 0.9
            h[:, :, 0] = np.where(present, rng.integers(1, 8, (R, E), dtype=np.uint64), 0)
            h[:, :, 1] = h[:, :, 0] & rng.integers(0, 8, (R, E), dtype=np.uint64) & \
                rng.integers(0, 8, (R, E), dtype=np.uint64)
            b.upload(h)
        dom = Domain()
        for e in range(E):
            es = dom.element_slot(e * 1000)
            for k in range(T):
                dom.token_slot(es, hashlib.blake2b(b"%d:%d" % (e, k), digest_size=20).digest())
        d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
        offs = ctx.buffer(8 * (R + 1))
        total = _lib.C.c_uint64()
        size_ms = timed(ctx, lambda: _lib.check(L.laspj_orset_etf_size(
            ctx.h, b.h, d.h, 76, offs.h, _lib.C.byref(total)), ctx.h), steps)
        out = ctx.buffer(total.value)
        cells = R * E
        report(f"orset_etf_size_{tag}", size_ms, 16 * cells + 16 * R, cells, "cells_per_s",
               replicas=R, elements=E)
        # record kernel (default for uniform token images), then the staging kernels
        variants = ((0, "write"), (1, "write_staging"))
        if os.environ.get("ETF_WINDOWS"):
            variants += ((2, "write_w16k"), (3, "write_w20k"), (4, "write_lanes"),
                         (5, "write_elem"))
        for knob, name in variants:
            ctx.set_tuning(_lib.TUNE_ETF_KERNEL, knob)
            ms = timed(ctx, lambda: _lib.check(L.laspj_orset_etf_write(
                ctx.h, b.h, d.h, 76, 1, offs.h, out.h), ctx.h), steps)
            report(f"orset_etf_{name}_{tag}", ms, 16 * cells + total.value, cells,
                   "cells_per_s", replicas=R, elements=E, payload_bytes=total.value,
                   payload_GBps=round(total.value / (ms / 1e3) / 1e9, 1))
        ctx.set_tuning(_lib.TUNE_ETF_KERNEL, 0)
        # from_binary: the payloads just written, decoded back into a batch
        _lib.check(L.laspj_orset_etf_write(ctx.h, b.h, d.h, 76, 1, offs.h, out.h), ctx.h)
        back = ctx.orset_batch(R, E)
        stb = ctx.buffer(4 * R)
        # 0: default (element batches at <= 8 token slots), 2: record batches only
        for knob, name in ((0, "read"), (2, "read_records")) if T <= 8 else ((0, "read"),):
            ctx.set_tuning(_lib.TUNE_ETF_READ, knob)
            ms = timed(ctx, lambda: _lib.check(L.laspj_orset_etf_read(
                ctx.h, back.h, d.h, 76, 1, out.h, offs.h, stb.h), ctx.h), steps)
            report(f"orset_etf_{name}_{tag}", ms, 16 * cells + total.value, cells,
                   "cells_per_s", replicas=R, elements=E, payload_bytes=total.value,
                   payload_GBps=round(total.value / (ms / 1e3) / 1e9, 1))
        ctx.set_tuning(_lib.TUNE_ETF_READ, 0)
        del back, stb
        del out, offs, d, b
    # G-Set to_binary / from_binary (lasp_gset.erl:111-113, 122-128): 65536 replicas x 1024
    # integer elements (SMALL_INTEGER_EXT / INTEGER_EXT images), ~50 % present: LIST_EXT
    R, E = 65536, 1024
    g = ctx.gset_batch(R, E)
    g.fill_synthetic(12)
    dom = Domain()
    for e in range(E):
        dom.element_slot(e)
    d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
    offs = ctx.buffer(8 * (R + 1))
    total = _lib.C.c_uint64()
    size_ms = timed(ctx, lambda: _lib.check(L.laspj_gset_etf_size(
        ctx.h, g.h, d.h, 82, offs.h, _lib.C.byref(total)), ctx.h), steps)
    W = (E + 63) // 64
    report("gset_etf_size", size_ms, 8 * W * R + 8 * R, R * E, "elements_per_s", replicas=R,
           elements=E)
    out = ctx.buffer(total.value)
    ms = timed(ctx, lambda: _lib.check(L.laspj_gset_etf_write(
        ctx.h, g.h, d.h, 82, 1, offs.h, out.h), ctx.h), steps)
    report("gset_etf_write", ms, 8 * W * R + total.value, R * E, "elements_per_s", replicas=R,
           elements=E, payload_bytes=total.value,
           payload_GBps=round(total.value / (ms / 1e3) / 1e9, 1))
    back = ctx.gset_batch(R, E)
    stb = ctx.buffer(4 * R)
    ms = timed(ctx, lambda: _lib.check(L.laspj_gset_etf_read(
        ctx.h, back.h, d.h, 82, 1, out.h, offs.h, stb.h), ctx.h), steps)
    same = bool(np.array_equal(back.download(), g.download())) and \
        not stb.download(np.int32, count=R).any()
    report("gset_etf_read", ms, 8 * W * R + total.value, R * E, "elements_per_s", replicas=R,
           elements=E, payload_bytes=total.value,
           payload_GBps=round(total.value / (ms / 1e3) / 1e9, 1), round_trip_equal=same)


def weak(ctx, steps):
    """The kernels VERDICT r2 found at 0.60-0.70 of the HBM roofline, alone, for PMC
    passes (tools/gpu_pmc_weak.sh): config 4 fused, config 5 intersection and product
    diag, the N = 8 anti-entropy reduce, and the G-Set join at 8 GiB operands."""
    L = ctx.L
    # config 4 fused (as config4(): composed index o -> o // 3, strict threshold)
    objects, E = 1024, 1 << 20
    src = ctx.orset_batch(objects, E)
    src.fill_synthetic(40, token_slots=3)
    fold, prev = ctx.orset_batch(objects, 3 * E), ctx.orset_batch(objects, 3 * E)
    prev.fill_synthetic(41, token_slots=3)
    fidx = ctx.buffer(4 * 3 * E)
    fidx.upload(np.repeat(np.arange(E, dtype=np.uint32), 3))
    out = ctx.buffer(objects)
    report("config4_dataflow_fused", timed(ctx, lambda: _lib.check(
        L.laspj_orset_gather_inflation(ctx.h, fold.h, src.h, fidx.h, prev.h, 1, out.h), ctx.h),
        steps), 112 * objects * E, objects * E, "input_elements_per_s")
    del src, fold, prev
    # config 5 intersection and product diag (as config5())
    P, E5, N = 1024, 150_000, 100_000
    bl, br = ctx.orset_batch(P, E5), ctx.orset_batch(P, E5)
    bl.fill_synthetic(5, token_slots=3)
    br.fill_synthetic(6, token_slots=3)
    ids = np.arange(E5)

    def bits(mask):
        b = np.packbits(mask.astype(np.uint8), bitorder="little")
        return np.concatenate([b, np.zeros((8 * ((E5 + 63) // 64) - len(b),), np.uint8)]).view(np.uint64)
    l = ctx.orset_batch(P, E5).filter(bl, bits(ids < N))
    r = ctx.orset_batch(P, E5).filter(br, bits(ids >= E5 - N))
    del bl, br
    x = l.intersection(r)
    report("config5_intersection", timed(ctx, lambda: _lib.check(
        L.laspj_orset_intersection(ctx.h, x.h, l.h, r.h), ctx.h), steps),
        64 * P * E5, P * E5, "slots_per_s")
    del x
    dg = engine.ORSetProductBatch(ctx, P, E5, 1)
    report("config5_product_diag", timed(ctx, lambda: _lib.check(
        L.laspj_orset_product_diag(ctx.h, dg.h, l.h, r.h), ctx.h), steps),
        36 * P * E5, P * E5, "slots_per_s")
    del dg, l, r
    # anti-entropy reduce at N = 8
    E8, q = 4096, (3 * (1 << 18)) // 8
    src8, dst8 = ctx.orset_batch(8 * q, E8), ctx.orset_batch(q, E8)
    report("orset_reduce_chunks_n8", timed(ctx, lambda: dst8.reduce_chunks(src8, 8), steps),
           16 * 9 * q * E8, q * E8, "dst_cells_per_s")
    del src8, dst8
    # the REDUCE step of an 8-GPU anti-entropy round at config 3 (laspj_antientropy_plan):
    # the rank's own 2^17-object chunk (8 GiB) joined in place with the 7 received copies
    # (recv: 56 GiB) — k_reduce_ptrs<8>, 8 x 16 B read + 16 B written per dst cell
    Q = 1 << 17
    own, recv = ctx.orset_batch(Q, E8), ctx.orset_batch(7 * Q, E8)
    own.fill_synthetic(10)
    recv.fill_synthetic(11)
    srcs = [own] + [recv.view(j * Q, 1 * Q) for j in range(7)]
    report("ae_reduce_in_place_n8", timed(ctx, lambda: own.join_n(srcs), steps),
           16 * 9 * Q * E8, Q * E8, "dst_cells_per_s")
    del own, recv, srcs
    # G-Set join, 8 GiB per operand
    RL_, EG = 16 << 20, 4096
    ga, gb, gc = (ctx.gset_batch(RL_, EG) for _ in range(3))
    ga.fill_synthetic(5)
    gb.fill_synthetic(6)
    W = (EG + 63) // 64
    report("gset_join_16x", timed(ctx, lambda: gc.join(ga, gb), steps), 24 * RL_ * W, RL_ * EG,
           "elements_per_s")


def ceilings(ctx, steps):
    """What plain streams of a given read:write mix reach at a given size on this box:
    the yardstick for kernels whose operands are a few GiB.  join =
    2 reads : 1 write (k_or16), copy = 1 : 1 (precondition_context: p & ~r, r = 0), read =
    value/1 (a bitmap written), each at total traffic ~6, 12, 24, 48, 96 GB."""
    L = ctx.L
    E = 4096
    for gib in (2, 4, 8, 16, 32, 64):
        R = gib << 30 >> 16                        # replicas of 64 KiB: `gib` GiB per operand
        a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
        a.fill_synthetic(2)
        b.fill_synthetic(3)
        cells = R * E
        report(f"ceiling_join_{gib}g", timed(ctx, lambda: c.join(a, b), steps), 48 * cells, cells,
               "cells_per_s", operand_gib=gib, mix="2R:1W")
        if gib == 64:                  # the headline's operand size: join only
            del a, b, c
            continue
        report(f"ceiling_copy_{gib}g", timed(ctx, lambda: _lib.check(
            L.laspj_orset_precondition_context(ctx.h, c.h, a.h), ctx.h), steps), 32 * cells,
            cells, "cells_per_s", operand_gib=gib, mix="1R:1W")
        bits = ctx.buffer(R * (E // 64) * 8)
        report(f"ceiling_read_{gib}g", timed(ctx, lambda: _lib.check(
            L.laspj_orset_value(ctx.h, a.h, bits.h), ctx.h), steps), 16 * cells + R * E // 8,
            cells, "cells_per_s", operand_gib=gib, mix="1R")
        del a, b, c, bits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=1 << 20)
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--only", default="kernels,ops,config4,config5,etf")
    a = ap.parse_args()
    ctx = engine.Context(0)
    todo = a.only.split(",")
    if "kernels" in todo:
        kernels(ctx, a.replicas, a.elements, a.steps)
    if "ops" in todo:
        ops(ctx, 3)
    if "config4" in todo:
        config4(ctx, 1024, 1 << 20, a.steps)
    if "config5" in todo:
        config5(ctx, a.steps)
    if "etf" in todo:
        etf(ctx, a.steps)
    if "weak" in todo:
        weak(ctx, a.steps)
    if "ceilings" in todo:
        ceilings(ctx, a.steps)


if __name__ == "__main__":
    main()
