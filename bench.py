#!/usr/bin/env python3
"""Headline benchmark: batched OR-Set join (lasp_orset:merge/2) on MI355X.

Workload (BASELINE.json configs[1], SURVEY.md §8d cfg 2): per GPU, 2^20 replica pairs
x 4096 element slots x 64 token slots, synthetic.  One step = one
`laspj_orset_join` launch computing C = A ⊔ B over the whole batch (3 x 64 GiB
resident in HBM).  Multi-GPU: one process per GPU, each joins its own replica shard
(no data-path collective; weak scaling); a gloo barrier + max-over-ranks brackets the
timed region.

Output: one JSON line (rank 0).  `roofline.achieved` = 48 algorithmic bytes per
(replica, element) join x cells per launch / average launch time measured with HIP
events on the engine's stream; `roofline.traffic` = HBM bytes per launch from the
rocprofv3 PMC passes committed under profiles/ (null if absent);  `cpu_baseline` =
the C restatement of lasp_orset:merge/2 (oracle/laspj_oracle.c, kind "port") timed on
this host's cores on a bounded sample.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "merged lattice elements/sec (node) + % HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_JOIN = 48         # read 2 x 16 B cells, write 16 B


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--replicas", type=int, default=1 << 20, help="replica pairs per GPU")
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--wide-replicas", type=int, default=1 << 19,
                    help="replicas of the T = 128 join leg (0: skip it)")
    ap.add_argument("--list-leg", type=int, default=1,
                    help="1: time config 5's list re-bind and the Store update (rank 0, N=1)")
    ap.add_argument("--cpu-budget", type=float, default=12.0,
                    help="seconds of CPU baseline work (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="check the launch (ranks, world size) and exit before any GPU work")
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--unroll", type=int, default=0)
    ap.add_argument("--nt", type=int, default=-1)
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r06_pmc_join.json"),
                    help="PMC summary giving HBM traffic per join launch")
    ap.add_argument("--antientropy", choices=["auto", "on", "off"], default="auto",
                    help="config-3 gossip anti-entropy leg (auto: when N > 1)")
    ap.add_argument("--ae-objects", type=int, default=1 << 20,
                    help="objects per GPU for the anti-entropy leg: BASELINE config 3, "
                         "2^20 x 4096 = 64 GiB of state (+ 64 GiB receive buffer)")
    ap.add_argument("--ae-rounds", type=int, default=3)
    ap.add_argument("--gc-objects", type=int, default=1 << 22,
                    help="G-Counters per GPU for the all_reduce(MAX) leg (x 64 actors x 8 B)")
    ap.add_argument("--ae-timeout", type=float, default=240.0,
                    help="seconds before a stuck anti-entropy leg is abandoned (the "
                         "headline line is still printed)")
    return ap.parse_args()


XGMI_LINK_GBS = 153.0        # per link per direction


def _uid(rank):
    """A communicator id made on rank 0 and handed to every rank over the gloo group
    (the NIF would send it over Erlang distribution)."""
    import torch.distributed as dist
    from lasp_amd.engine import Comm
    box = [Comm.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def _sampled_join_ok(ctx, state, make, join, seed0, world, objects):
    """Objects spread over every chunk: the state after a round must equal the join of
    all ranks' synthetic replicas of that object (computed here from the streams)."""
    import numpy as np
    picks = sorted({int(x) for x in np.linspace(0, objects - 1, 16)})
    exp, tmp = make(), make()
    for o in picks:
        exp.clear()
        for r in range(world):
            tmp.fill_synthetic(seed0 + r, replica_base=o)
            join(exp, exp, tmp)
        if not np.array_equal(state.download(o, 1), exp.download()):
            return False
    return True


def antientropy_leg(ctx, args, rank, world, barrier):
    """BASELINE config 3 through the C ABI (laspj_antientropy, RCCL over xGMI): every
    rank holds one replica of `objects` OR-Sets; a round (all-to-all -> HIP OR of the
    copies -> all-gather, all on the engine stream) leaves every rank with the join of
    all ranks' replicas."""
    import torch
    import torch.distributed as dist
    from lasp_amd.engine import Comm
    comm = Comm(ctx, world, _uid(rank), rank)
    O, E = args.ae_objects, args.elements
    st = ctx.orset_batch(O, E)
    # the peers' copies of this rank's chunk: (n-1)/n of the state (none at n = 1)
    rv = ctx.orset_batch(O // world * (world - 1), E) if world > 1 else None
    st.fill_synthetic(10 + rank)
    ctx.synchronize()
    comm.antientropy(st, rv)                     # warm-up round (RCCL connection setup)
    ctx.synchronize()
    ok = _sampled_join_ok(ctx, st, lambda: ctx.orset_batch(1, E),
                          lambda d, a, b: d.join(a, b), 10, world, O)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.ae_rounds):
        comm.antientropy(st, rv)
    ctx.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, 0.0 if ok else 1.0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per_round = float(t[0].item()) / args.ae_rounds
    S = st.nbytes
    xgmi = 2.0 * (world - 1) / world * S / per_round / 1e9 if world > 1 else 0.0
    out = {
        "workload": "gossip anti-entropy (BASELINE configs[2]) via laspj_antientropy: "
                    "RCCL all-to-all + HIP OR (own chunk joined in place) + RCCL "
                    "all-gather, all on the engine stream (laspj_antientropy_plan's "
                    "steps; a one-rank round has no step)",
        "hbm_bytes_per_round": (S + S // world) if world > 1 else 0,
        "objects_per_gpu": O, "elements": E, "state_bytes_per_gpu": S,
        "rounds": args.ae_rounds, "ms_per_round": per_round * 1e3,
        "merged_elements_per_s": (world - 1) * O * E / per_round,
        "xgmi_GBps_per_gpu": xgmi,
        "frac_mesh": xgmi / (XGMI_LINK_GBS * 7), "frac_ring": xgmi / XGMI_LINK_GBS,
        "converged": t[1].item() == 0.0,
    }
    del st, rv
    out["gcounter"] = gcounter_leg(ctx, args, rank, world, barrier, comm)
    comm.close()
    return out


def gcounter_leg(ctx, args, rank, world, barrier, comm):
    """G-Counter anti-entropy: one RCCL all_reduce(max) on uint64 counts per round
    (riak_dt_gcounter's join is the per-actor max); afterwards sampled counters must be
    the max over every rank's synthetic replica, and threshold reads run on the result."""
    import torch
    import torch.distributed as dist
    O, A = args.gc_objects, 64
    gc = ctx.gcounter_batch(O, A)
    gc.fill_synthetic(20 + rank)
    comm.antientropy(gc)
    ctx.synchronize()
    ok = _sampled_join_ok(ctx, gc, lambda: ctx.gcounter_batch(1, A),
                          lambda d, a, b: d.join(a, b), 20, world, O)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.ae_rounds):
        comm.antientropy(gc)
    ctx.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    reached = int(gc.threshold_met(64 * (1 << 19)).sum())     # threshold reads after gossip
    t = torch.tensor([wall, 0.0 if ok else 1.0], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    per_round = float(t[0].item()) / args.ae_rounds
    busbw = 2.0 * (world - 1) / world * gc.nbytes / per_round / 1e9 if world > 1 else 0.0
    return {
        "workload": "G-Counter anti-entropy: RCCL all_reduce(max) on uint64 counts",
        "objects_per_gpu": O, "actors": A, "state_bytes_per_gpu": gc.nbytes,
        "ms_per_round": per_round * 1e3, "converged": t[1].item() == 0.0,
        "threshold_objects": reached,
        "merged_counts_per_s": (world - 1) * O * A / per_round,
        "xgmi_GBps_per_gpu": busbw,
    }


def host_cores() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, 16))       # the GPU box grants 16 CPUs per GPU


def cpu_baseline(elements: int, budget: float):
    from oracle import columnar as orc    # cpu_baseline leg: the oracle is the timed port
    cores = host_cores()
    eps, merges, secs = orc.bench_orset_merge(elements, 2, cores, 2, budget)
    m, u, f, v, infl = orc.bench_config1_ext(10_000, 200, 5)
    m_threads = orc.bench_config1_merge_threads(10_000, cores, 2.0)
    # a second column: the device's own cell layout OR-ed on the same cores (bounded by
    # host DRAM bandwidth, not by the orddict walk)
    per_thread = 1 << 22                 # 4M cells = 64 MiB per array per thread
    col = orc.bench_cells_join(per_thread, cores, min(3.0, budget / 4))
    return {
        "value": eps, "unit": "merged elements/s", "cores": cores, "kind": "port",
        "sample": (f"C restatement of lasp_orset:merge/2 (nested orddict two-finger merge, "
                   f"20-byte tokens) on {cores} threads x 2 synthetic replica pairs "
                   f"(E={elements}, T<=64), {merges} merges in {secs:.1f} s"),
        "columnar": {"value": col, "unit": "merged elements/s", "cores": cores,
                     "sample": (f"the GPU's {{p, r}} cell layout joined d = a | b on {cores} "
                                f"threads, {per_thread} cells (3 x 64 MiB) per thread, "
                                f"~{min(3.0, budget / 4):.0f} s")},
        "config1": {"workload": "2 replicas x 10k elements (BASELINE configs[0]), 1 thread",
                    "us_merge": m, "us_union": u, "us_filter": f, "us_value": v,
                    "us_inflation": infl,
                    # lasp_core:bind/3 (lasp_core.erl:298-304) does both: Merged = merge(Value0,
                    # Value), then is_inflation(Value0, Merged) — the keyfind walk above
                    "us_bind": m + infl,
                    "us_merge_all_cores_per_merge": m_threads,
                    "all_cores": cores},
    }


def config1_gpu(ctx):
    """BASELINE configs[0] on the device: one 10k-slot replica pair; per-call latency of
    merge, the union body, the filter body, value/1 and is_inflation (launch + kernel,
    inputs resident)."""
    import numpy as np
    n, iters = 10_000, 200
    a, b, c = ctx.orset_batch(1, 2 * n), ctx.orset_batch(1, 2 * n), ctx.orset_batch(1, 2 * n)
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    keep = ctx.buffer(((2 * n + 63) // 64) * 8)
    keep.upload(np.full(((2 * n + 63) // 64,), 0x5555555555555555, np.uint64))
    bits = ctx.buffer(((2 * n + 63) // 64) * 8)
    flag = ctx.buffer(1)
    L = ctx.L
    from lasp_amd._lib import check
    out = {}
    c.join(a, b)
    for name, fn in (("merge", lambda: c.join(a, b)), ("union", lambda: c.union(a, b)),
                     ("filter", lambda: check(L.laspj_orset_filter(ctx.h, c.h, a.h, keep.h))),
                     ("value", lambda: check(L.laspj_orset_value(ctx.h, c.h, bits.h))),
                     ("inflation", lambda: check(L.laspj_orset_inflation(ctx.h, a.h, c.h, 0,
                                                                          flag.h)))):
        fn()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        ctx.synchronize()
        out["us_" + name] = (time.perf_counter() - t0) * 1e6 / iters
    out["workload"] = "1 replica pair x 20k element slots, inputs resident in HBM"
    # the same merge as the NIF pays it: two term_to_binary/1 payloads of 10k-element
    # orddicts (built untimed, their terms registered untimed) -> upload -> device
    # from_binary -> k_or16 -> device to_binary -> download of the merged payload
    from lasp_amd import _lib, etf
    from lasp_amd.engine import ETFDict
    from lasp_amd.hostdict import NativeDict
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
    nd = NativeDict()
    nd.add(_lib.KIND_ORSET, [pa, pb])
    E = nd.info()[0]
    d = ETFDict(ctx, E, *nd.export(E))
    na, nb, nc = ctx.orset_batch(1, E), ctx.orset_batch(1, E), ctx.orset_batch(1, E)
    host = np.zeros((2, 2 * E), np.uint64)

    def e2e_host_encode():
        cells, st = nd.encode(_lib.KIND_ORSET, [pa, pb], E, out=host)
        na.upload(cells[0])
        nb.upload(cells[1])
        nc.join(na, nb)
        return nc.to_binaries(d)[0]

    # the NIF's path when the dictionary already holds every term:
    # the two payloads go to the device as they are and are decoded there
    # (laspj_orset_etf_read); only a payload with a term the dictionary lacks
    # (LASPJ_DEC_UNKNOWN_TERM) would take laspj_dict_add + laspj_dict_encode.  Buffers
    # are the NIF's, allocated once.
    import ctypes as C
    blob = np.frombuffer(pa + pb, np.uint8)
    offs = np.array([0, len(pa), len(pa) + len(pb)], np.uint64)
    pay, poff = ctx.buffer(len(blob)), ctx.buffer(24)
    ab = ctx.orset_batch(2, E)
    a0, b0 = ab.view(0, 1), ab.view(1, 1)
    stb, oo = ctx.buffer(8), ctx.buffer(16)
    ob = ctx.buffer(len(blob) + 64)            # a merge is never longer than both inputs
    total = C.c_uint64()

    def e2e():
        pay.upload(blob)
        poff.upload(offs)
        check(L.laspj_orset_etf_read(ctx.h, ab.h, d.h, -1, 1, pay.h, poff.h, stb.h), ctx.h)
        check(L.laspj_orset_join(ctx.h, nc.h, a0.h, b0.h), ctx.h)
        check(L.laspj_orset_etf_size(ctx.h, nc.h, d.h, -1, oo.h, C.byref(total)), ctx.h)
        check(L.laspj_orset_etf_write(ctx.h, nc.h, d.h, -1, 1, oo.h, ob.h), ctx.h)
        if stb.download(np.int32, count=2).any():
            raise RuntimeError("config1 e2e: a payload did not decode")
        return ob.download(np.uint8, count=total.value).tobytes()

    ref = e2e_host_encode()
    if e2e() != ref:
        raise RuntimeError("config1 e2e: device-decode path differs from the host encoder")
    for name, fn in (("us_merge_native_end_to_end", e2e),
                     ("us_merge_native_host_encode", e2e_host_encode)):
        fn()
        t0 = time.perf_counter()
        for _ in range(20):
            fn()
        out[name] = (time.perf_counter() - t0) * 1e6 / 20
    # the NIF-level entry point (laspj_orset_etf_merge, laspj_nif.hip): the same two
    # images in host memory -> the merged image in pinned host memory, one C call with one
    # host synchronisation (the context's own dictionary, warmed by the first call); and
    # n queued merges in one call (laspj_orset_etf_merge_many), per merge
    op, on, vd = C.c_void_p(), C.c_uint64(), C.c_int32()

    def nif():
        check(L.laspj_orset_etf_merge(ctx.h, pa, len(pa), pb, len(pb), C.byref(op),
                                      C.byref(on), C.byref(vd)), ctx.h)

    nif()
    if vd.value != 0 or C.string_at(op, on.value) != ref:
        raise RuntimeError("config1: the NIF entry point's merge differs from the host encoder")
    nif()
    t0 = time.perf_counter()
    for _ in range(50):
        nif()
    out["us_merge_nif"] = (time.perf_counter() - t0) * 1e6 / 50
    # value/1 of B's image (lasp_orset.erl:67-73: its answer is a G-Set image) and the
    # lasp_gset merge of config 1's two integer sets (10k each, 5k overlap:
    # lasp_gset.erl:99-101) through the NIF entry points, warm
    gva = [e for e, toks in tb if any(not f for _t, f in toks)]
    ga, gb = list(range(n)), list(range(n // 2, n + n // 2))
    qa, qb = etf.term_to_binary(ga), etf.term_to_binary(gb)
    for name, fn, want in (
            ("us_value_nif", lambda: L.laspj_orset_etf_value(ctx.h, pb, len(pb), C.byref(op),
                                                             C.byref(on), C.byref(vd)),
             etf.term_to_binary(gva)),
            ("us_gset_merge_nif", lambda: L.laspj_gset_etf_merge(ctx.h, qa, len(qa), qb, len(qb),
                                                                 C.byref(op), C.byref(on),
                                                                 C.byref(vd)),
             etf.term_to_binary(list(range(n + n // 2))))):
        check(fn(), ctx.h)
        if vd.value != 0 or C.string_at(op, on.value) != want:
            raise RuntimeError("config1: %s answered wrongly" % name)
        t0 = time.perf_counter()
        for _ in range(50):
            check(fn(), ctx.h)
        out[name] = (time.perf_counter() - t0) * 1e6 / 50
    nm = 32
    arr_a = (C.c_char_p * nm)(*([pa] * nm))
    arr_b = (C.c_char_p * nm)(*([pb] * nm))
    len_a = (C.c_uint64 * nm)(*([len(pa)] * nm))
    len_b = (C.c_uint64 * nm)(*([len(pb)] * nm))
    outs, olens, vds = (C.c_void_p * nm)(), (C.c_uint64 * nm)(), (C.c_int32 * nm)()

    def nif_many():
        check(L.laspj_orset_etf_merge_many(ctx.h, nm, arr_a, len_a, arr_b, len_b, outs, olens,
                                           vds), ctx.h)

    nif_many()
    if any(vds[k] for k in range(nm)) or C.string_at(outs[nm - 1], olens[nm - 1]) != ref:
        raise RuntimeError("config1: merge_many differs from the host encoder")
    t0 = time.perf_counter()
    for _ in range(5):
        nif_many()
    out["us_merge_nif_many_per_merge"] = (time.perf_counter() - t0) * 1e6 / (5 * nm)
    out["nif_many_batch"] = nm
    # an update/3 between binds mints a token (lasp_orset.erl:222-230, 261-262): the
    # merge then meets one term its dictionary lacks — registration, device images
    # rebuilt, a second device pass
    cold = []
    sc0 = ctx.nif_stats()
    for k in range(5):
        tb2 = list(tb)
        e = 17 * k + 3
        tb2[e] = (e, sorted(tb[e][1] + [(b"N" + (k * 7919 + e).to_bytes(19, "big"), False)]))
        pb2 = etf.term_to_binary(tb2)
        t0 = time.perf_counter()
        check(L.laspj_orset_etf_merge(ctx.h, pa, len(pa), pb2, len(pb2), C.byref(op),
                                      C.byref(on), C.byref(vd)), ctx.h)
        cold.append((time.perf_counter() - t0) * 1e6)
        if vd.value != 0:
            raise RuntimeError("config1: a merge with a new token fell back")
    out["us_merge_nif_new_token"] = sorted(cold)[len(cold) // 2]
    sc1 = ctx.nif_stats()
    # where a cold merge's time goes (host clock, averaged over the 5): the first device
    # pass that meets the new term, registering both operands' terms, rebuilding the device
    # images, the second pass
    out["nif_new_token_stages_us"] = {k: (sc1[k] - sc0[k]) / 5e3 for k in
                                      ("ns_stage_enqueue", "ns_device_wait", "ns_register",
                                       "ns_rebuild")}
    nif()
    st0 = ctx.nif_stats()
    for _ in range(20):
        nif()
    st1 = ctx.nif_stats()
    out["nif_stats"] = st1
    # where one warm NIF merge's time goes (host clock, averaged over 20 calls)
    out["nif_stages_us"] = {k: (st1[k] - st0[k]) / 20e3 for k in
                            ("ns_stage_copy", "ns_stage_enqueue", "ns_device_wait",
                             "ns_answers")}
    # where the device-decode path's time goes (one call, synchronised per stage)
    stages = {}
    t0 = time.perf_counter()
    pay.upload(blob)
    poff.upload(offs)
    t1 = time.perf_counter()
    check(L.laspj_orset_etf_read(ctx.h, ab.h, d.h, -1, 1, pay.h, poff.h, stb.h), ctx.h)
    ctx.synchronize()
    t2 = time.perf_counter()
    check(L.laspj_orset_join(ctx.h, nc.h, a0.h, b0.h), ctx.h)
    ctx.synchronize()
    t3 = time.perf_counter()
    check(L.laspj_orset_etf_size(ctx.h, nc.h, d.h, -1, oo.h, C.byref(total)), ctx.h)
    check(L.laspj_orset_etf_write(ctx.h, nc.h, d.h, -1, 1, oo.h, ob.h), ctx.h)
    ctx.synchronize()
    t4 = time.perf_counter()
    stb.download(np.int32, count=2)
    ob.download(np.uint8, count=total.value)
    t5 = time.perf_counter()
    for k, (u, v) in zip(("upload", "from_binary", "join", "to_binary", "download"),
                         ((t0, t1), (t1, t2), (t2, t3), (t3, t4), (t4, t5))):
        stages[k] = (v - u) * 1e6
    out["end_to_end_stages_us"] = stages
    out["end_to_end"] = ("2 x 10k-element term_to_binary payloads (%d B): upload + device "
                         "from_binary + join + device to_binary + download of the %d-byte "
                         "merged payload; us_merge_native_host_encode: host dictionary encode "
                         "instead of the device decoder" % (len(blob), total.value))
    out.update(config1_resident(ctx, pa, pb, ref))
    return out


def config1_resident(ctx, pa: bytes, pb: bytes, ref: bytes):
    """bind/3 with `#dv.value` resident on the device (laspj_var_etf_bind, lasp_core.erl:
    291-312): Value0 = A ⊔ B stays in HBM, each bind ships only the incoming 10k-element
    image B, decodes it, decides `Value0 =:= Value` and merges in one kernel, and reads
    back a status.  Single binds on one context, 32 binds per call, and 16 contexts (one
    per BEAM scheduler) binding at once from 16 threads on the one GPU."""
    import ctypes as C
    import threading
    from lasp_amd._lib import check
    from lasp_amd import engine
    L = ctx.L
    out = {}
    var = ctx.var("orset")
    if var.write(pa) != 0 or var.bind(pb) != (0, 1) or var.read() != (0, ref):
        raise RuntimeError("config1: the resident bind differs from the merge")
    st, vd = C.c_int32(), C.c_int32()

    def vbind(v=var):
        check(L.laspj_var_etf_bind(v.h, pb, len(pb), C.byref(st), C.byref(vd)), ctx.h)

    vbind()
    t0 = time.perf_counter()
    for _ in range(50):
        vbind()
    out["us_bind_nif"] = (time.perf_counter() - t0) * 1e6 / 50
    if (vd.value, st.value) != (0, 1) or var.read() != (0, ref):
        raise RuntimeError("config1: resident bind answered wrongly")
    # the C call alone, as us_merge_nif (the answer stays in pinned memory for
    # enif_binary_to_term; var.read() above copied it into a Python bytes to check it)
    rout, rlen, rvd = C.c_void_p(), C.c_uint64(), C.c_int32()
    t0 = time.perf_counter()
    for _ in range(20):
        check(L.laspj_var_etf_read(var.h, C.byref(rout), C.byref(rlen), C.byref(rvd)), ctx.h)
    out["us_read_nif"] = (time.perf_counter() - t0) * 1e6 / 20
    if rvd.value != 0 or C.string_at(rout, rlen.value) != ref:
        raise RuntimeError("config1: resident read answered wrongly")
    nm = 32
    vs = [ctx.var("orset") for _ in range(nm)]
    for v in vs:
        v.write(ref)
    arr_v = (C.c_void_p * nm)(*[v.h.value for v in vs])
    arr_p = (C.c_char_p * nm)(*([pb] * nm))
    arr_n = (C.c_uint64 * nm)(*([len(pb)] * nm))
    sts, vds = (C.c_int32 * nm)(), (C.c_int32 * nm)()

    def vbind_many():
        check(L.laspj_var_etf_bind_many(ctx.h, nm, arr_v, arr_p, arr_n, sts, vds), ctx.h)

    vbind_many()
    t0 = time.perf_counter()
    for _ in range(5):
        vbind_many()
    out["us_bind_nif_many_per_bind"] = (time.perf_counter() - t0) * 1e6 / (5 * nm)
    if any(vds[k] or sts[k] != 1 for k in range(nm)):
        raise RuntimeError("config1: bind_many answered wrongly")
    # update/4 on the resident variable (laspj_var_etf_update, lasp_core.erl:283-287): {add, E}
    # of a known element mints a token (unique/1), registers it in the variable's namespace,
    # patches the device images and sets the token's bit — the update ships only the op
    from lasp_amd import etf as oetf           # (the op images are built untimed)
    from lasp_amd.terms import Atom
    res, vd2, nmint = C.c_int32(), C.c_int32(), C.c_uint32()
    eimg, elen, mint = C.c_void_p(), C.c_uint64(), C.c_void_p()
    uv = ctx.var("orset")
    uv.write(ref)
    add_ops = [oetf.term_to_binary((Atom("add"), e)) for e in range(0, 10_000, 97)]
    rm_ops = [oetf.term_to_binary((Atom("remove"), e)) for e in range(5, 10_000, 89)]

    def vupdate(img):
        check(L.laspj_var_etf_update(uv.h, img, len(img), C.byref(res), C.byref(eimg),
                                     C.byref(elen), C.byref(mint), C.byref(nmint), C.byref(vd2)),
              ctx.h)
        if vd2.value != 0 or res.value != 0:
            raise RuntimeError("config1: update/4 answered wrongly")

    stage_keys = ("device_passes", "registrations", "image_rebuilds", "image_patches",
                  "ns_register", "ns_rebuild", "ns_stage_enqueue", "ns_device_wait")

    def stats_delta(a, b, k):
        return {x: (b[x] - a[x]) / k if x.startswith("ns_") else b[x] - a[x] for x in stage_keys}

    vupdate(add_ops[0])
    ctx.synchronize()
    su0 = ctx.nif_stats()
    t0 = time.perf_counter()
    for img in add_ops[1:51]:
        vupdate(img)
    ctx.synchronize()
    out["us_update_nif"] = (time.perf_counter() - t0) * 1e6 / 50
    out["update_stages"] = stats_delta(su0, ctx.nif_stats(), 50)
    t0 = time.perf_counter()
    for img in rm_ops[:50]:
        vupdate(img)
    out["us_update_nif_remove"] = (time.perf_counter() - t0) * 1e6 / 50
    # the bind that meets a freshly minted token: a replica in the variable's namespace
    # (laspj_var_create_replica) binds the updated state — the token is known; a variable of
    # its own namespace (another node's replica) binds it — a token its dictionary has not
    # seen, taken by the decoder in the same pass (registered after it, the device images
    # patched on the next call)
    rep = uv.replica()
    far = ctx.var("orset")
    _, img0 = uv.read()
    rep.write(img0)
    far.write(img0)
    times_rep, times_far = [], []
    sc0 = ctx.nif_stats()
    for k in range(10):
        vupdate(add_ops[60 + k])
        _, img = uv.read()
        for v, acc in ((rep, times_rep), (far, times_far)):
            t0 = time.perf_counter()
            check(L.laspj_var_etf_bind(v.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
            acc.append((time.perf_counter() - t0) * 1e6)
            if (vd.value, st.value) != (0, 1):
                raise RuntimeError("config1: the bind of an updated state answered wrongly")
    sc1 = ctx.nif_stats()
    out["new_token_stages"] = stats_delta(sc0, sc1, 10)
    out["new_token_samples_us"] = {"replica": [round(x, 1) for x in times_rep],
                                   "far": [round(x, 1) for x in times_far]}
    if rep.read() != uv.read() or far.read() != uv.read():
        raise RuntimeError("config1: replicas did not converge")
    out["us_bind_nif_replica_update"] = sorted(times_rep)[len(times_rep) // 2]
    out["us_bind_nif_new_token"] = sorted(times_far)[len(times_far) // 2]
    out["bind_new_token_passes"] = (sc1["device_passes"] - sc0["device_passes"]) / 10
    for v in (rep, far, uv):
        v.close()
    # update/4 adding an element the namespace has never held: a new dictionary term, so
    # the namespace's device images are rebuilt (the rank-indexed tables)
    nv = ctx.var("orset")
    if nv.write(pa) != 0:
        raise RuntimeError("config1: write answered wrongly")
    times_ne = []
    for k in range(9):
        op = oetf.term_to_binary((Atom("add"), 1_000_000 + k))
        t0 = time.perf_counter()
        check(L.laspj_var_etf_update(nv.h, op, len(op), C.byref(res), C.byref(eimg),
                                     C.byref(elen), C.byref(mint), C.byref(nmint), C.byref(vd2)),
              ctx.h)
        ctx.synchronize()
        times_ne.append((time.perf_counter() - t0) * 1e6)
        if vd2.value != 0 or res.value != 0:
            raise RuntimeError("config1: update/4 of a new element answered wrongly")
    out["us_update_nif_new_element"] = sorted(times_ne)[len(times_ne) // 2]
    nv.close()
    # lasp_core:union/7's body re-run over resident variables of one namespace
    # (laspj_var_union): l = A, r = B, out := merge(out, keep-left(l, r)) — nothing crosses
    # PCIe but the status (the image route: var_read of both, the body, var_bind)
    ul = ctx.var("orset")
    ur, uo = ul.replica(), ul.replica()
    if ul.write(pa) != 0 or ur.write(pb) != 0 or uo.union(ul, ur) != (0, 1):
        raise RuntimeError("config1: var_union answered wrongly")
    ust, uvd = C.c_int32(), C.c_int32()
    t0 = time.perf_counter()
    for _ in range(50):
        check(L.laspj_var_union(uo.h, ul.h, ur.h, C.byref(ust), C.byref(uvd)), ctx.h)
    out["us_var_union"] = (time.perf_counter() - t0) * 1e6 / 50
    if (uvd.value, ust.value) != (0, 0) or uo.read() != ul.read():     # out =:= keep-left = A
        raise RuntimeError("config1: var_union answered wrongly")
    for v in (ul, ur, uo):
        v.close()
    # schedulers: a context and a variable each, binding B in a loop (4 = the box's
    # hardware queues per process, GPU_MAX_HW_QUEUES; 16 = one per BEAM scheduler)
    for nthreads in (4, 16):
        out[f"bind_{nthreads}ctx"] = _bind_threads(ctx, nthreads, 60, ref, pb)
    # 16 schedulers through one context: the group commit batches them
    out["bind_16thr_1ctx"] = _bind_threads(ctx, 16, 60, ref, pb, shared=True)
    out["resident"] = ("Value0 = A ⊔ B resident (laspj_var); per bind: the %d-byte image of B "
                       "in, decode + `=:=` + merge on the device, the status out" % len(pb))
    for v in vs:
        v.close()
    var.close()
    return out


def _bind_threads(ctx, nthreads: int, per: int, ref: bytes, pb: bytes, shared: bool = False):
    """nthreads BEAM schedulers, each with a resident variable holding A ⊔ B, binding B
    `per` times at once (lasp_vnode.erl:213-237: concurrent callers) — each on a context
    of its own, or (shared) all on one context, whose group commit batches the binds
    queued while a pass runs into the next pass."""
    import ctypes as C
    import threading
    from lasp_amd._lib import check
    from lasp_amd import engine
    L = ctx.L
    loop = _bind_loop_lib()
    ready, errs, spans = threading.Barrier(nthreads + 1), [], []
    done = threading.Barrier(nthreads)

    def worker():
        try:
            c2 = ctx if shared else engine.Context(ctx.device)
            v2 = c2.var("orset")
            v2.write(ref)
            s2, d2 = C.c_int32(), C.c_int32()
            check(L.laspj_var_etf_bind(v2.h, pb, len(pb), C.byref(s2), C.byref(d2)), c2.h)
            ready.wait()
            t = time.perf_counter()
            # the loop in C (tests/c/bind_loop.c): the threads meet in the library, not on
            # the interpreter lock
            check(loop.bind_loop(v2.h, pb, len(pb), per, C.byref(s2), C.byref(d2)), c2.h)
            spans.append((t, time.perf_counter()))
            if (d2.value, s2.value) != (0, 1):
                errs.append("bad answer")
            # (teardown only once every scheduler is done: freeing device memory waits for
            # the device and would stall the others' binds inside the timed span)
            done.wait()
            v2.close()
            if not shared:
                c2.close()
        except Exception as e:       # noqa: BLE001 — reported below
            errs.append(repr(e))
            for b in (ready, done):
                try:
                    b.abort()
                except Exception:
                    pass

    ths = [threading.Thread(target=worker) for _ in range(nthreads)]
    for t in ths:
        t.start()
    try:
        ready.wait(timeout=120)
    except threading.BrokenBarrierError:
        pass
    st0 = ctx.nif_stats() if shared else None
    for t in ths:
        t.join(timeout=300)
    if errs or len(spans) != nthreads:
        raise RuntimeError(f"config1: {nthreads}-context binds failed: {errs[:3]}")
    wall = max(b for _a, b in spans) - min(a for a, _b in spans)
    extra = {}
    if shared:
        # binds per device pass (the group commit's batches) and where a pass's host time
        # goes (µs per pass)
        st1 = ctx.nif_stats()
        passes = max(1, st1["device_passes"] - st0["device_passes"])
        extra["binds_per_pass"] = nthreads * per / passes
        extra["pass_stages_us"] = {k: round((st1[k] - st0[k]) / passes / 1e3, 1) for k in
                                   ("ns_stage_enqueue", "ns_stage_copy", "ns_device_wait")}
    return {**extra, "contexts": 1 if shared else nthreads, "threads": nthreads,
            "binds": nthreads * per,
            "us_per_bind": wall * 1e6 / (nthreads * per),
            "binds_per_s": nthreads * per / wall,
            "merged_elements_per_s": nthreads * per * 10_000 / wall,
            "pcie_GBps": nthreads * per * len(pb) / wall / 1e9}


def _bind_loop_lib():
    """tests/c/bind_loop.c built against include/laspj.h and liblaspj.so (gcc, in /tmp)."""
    import ctypes as C
    import subprocess
    import tempfile
    from lasp_amd import _lib
    libdir = os.path.dirname(_lib.LIB_PATH)
    out = os.path.join(tempfile.gettempdir(), f"laspj_bind_loop_{os.getpid()}.so")
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", out,
                    os.path.join(ROOT, "tests", "c", "bind_loop.c"), "-L", libdir, "-llaspj",
                    f"-Wl,-rpath,{libdir}"], check=True)
    lib = C.CDLL(out)
    lib.bind_loop.restype = C.c_int
    lib.bind_loop.argtypes = [C.c_void_p, C.c_char_p, C.c_uint64, C.c_int,
                              C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    return lib


def steady_leg(ctx, nvars: int = 32, steps: int = 200):
    """The drop-in's steady state (lasp_core.erl:283-312, lasp_update_fsm.erl:174-216): two
    nodes, each a context holding `nvars` resident variables (a vnode's store), one replica
    of every variable on each.  Each step picks a variable and a node: update/4 {add, E}
    there (a token minted), the updated state read out (what gossip ships), bound into the
    other node's replica (a token that node has not seen), then a threshold read there.
    Every 10th step also removes an element (update {remove, E}).  Config 1's shape: 10k
    elements, 1-2 tokens each.  Reported per op and per step, with the fallback / reset
    counts and the bytes that crossed PCIe."""
    import ctypes as C
    import numpy as np
    from lasp_amd._lib import check
    from lasp_amd import engine, etf
    from lasp_amd import etf as oetf            # op images, built untimed
    from lasp_amd.terms import Atom
    L = ctx.L
    n = 10_000
    nodes = [ctx, engine.Context(ctx.device)]
    base = [(e, [(b"S" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    img0 = etf.term_to_binary(base)
    vs = [[c.var("orset") for _ in range(nvars)] for c in nodes]
    for row in vs:
        for v in row:
            if v.write(img0) != 0:
                raise RuntimeError("steady: write fell back")
    rng = np.random.default_rng(11)
    plan = [(int(rng.integers(nvars)), int(rng.integers(2)), int(rng.integers(n)), k % 10 == 9)
            for k in range(steps)]
    ops = {}
    for _i, _nd, e, rm in plan:
        ops[(e, rm)] = oetf.term_to_binary((Atom("remove" if rm else "add"), e))
    th = etf.term_to_binary(base[:50])
    res, vd, nm = C.c_int32(), C.c_int32(), C.c_uint32()
    ei, el, mi = C.c_void_p(), C.c_uint64(), C.c_void_p()
    rp, rl = C.c_void_p(), C.c_uint64()
    st = C.c_int32()
    t_upd = t_read = t_bind = t_th = 0.0
    shipped = 0
    s0 = [c.nif_stats() for c in nodes]
    t_all = time.perf_counter()
    for i, nd, e, rm in plan:
        src, dst = vs[nd][i], vs[1 - nd][i]
        op = ops[(e, rm)]
        t0 = time.perf_counter()
        check(L.laspj_var_etf_update(src.h, op, len(op), C.byref(res), C.byref(ei), C.byref(el),
                                     C.byref(mi), C.byref(nm), C.byref(vd)), nodes[nd].h)
        t1 = time.perf_counter()
        if vd.value != 0:
            raise RuntimeError("steady: update fell back")
        check(L.laspj_var_etf_read(src.h, C.byref(rp), C.byref(rl), C.byref(vd)), nodes[nd].h)
        img = C.string_at(rp, rl.value)          # (the gossip message: copied out)
        t2 = time.perf_counter()
        check(L.laspj_var_etf_bind(dst.h, img, len(img), C.byref(st), C.byref(vd)),
              nodes[1 - nd].h)
        t3 = time.perf_counter()
        if vd.value != 0:
            raise RuntimeError("steady: bind fell back")
        check(L.laspj_var_etf_threshold(dst.h, th, len(th), 0, C.byref(res), C.byref(vd)),
              nodes[1 - nd].h)
        t4 = time.perf_counter()
        if vd.value != 0 or res.value != 1:
            raise RuntimeError("steady: threshold answered wrongly")
        t_upd += t1 - t0
        t_read += t2 - t1
        t_bind += t3 - t2
        t_th += t4 - t3
        shipped += 2 * len(img) + len(op) + len(th)
    wall = time.perf_counter() - t_all
    s1 = [c.nif_stats() for c in nodes]
    d = {k: sum(s1[j][k] - s0[j][k] for j in range(2))
         for k in ("device_passes", "registrations", "dict_resets", "fallbacks", "vars_spilled",
                   "image_rebuilds", "image_patches")}
    # the replicas converge: every variable's two replicas read alike after a final exchange
    for i in range(nvars):
        _v, a = vs[0][i].read()
        vs[1][i].bind(a)
        _v, b = vs[1][i].read()
        vs[0][i].bind(b)
        if vs[0][i].read() != vs[1][i].read():
            raise RuntimeError(f"steady: variable {i} did not converge")
    for row in vs:
        for v in row:
            v.close()
    nodes[1].close()
    return {"workload": (f"2 nodes x {nvars} resident variables (10k elements each, config 1's "
                         f"shape); {steps} steps of update/4 (a minted token; 1 in 10 a "
                         f"remove) -> read (gossip) -> bind on the other node -> threshold"),
            "us_per_step": wall * 1e6 / steps, "us_update": t_upd * 1e6 / steps,
            "us_read": t_read * 1e6 / steps, "us_bind": t_bind * 1e6 / steps,
            "us_threshold": t_th * 1e6 / steps,
            "device_passes_per_step": d["device_passes"] / steps,
            "pcie_GBps": shipped / wall / 1e9, "counts": d}


def wide_leg(ctx, args):
    """The join when elements carry more than 64 tokens (LASPJ_KIND_ORSET_WIDE, T = 128:
    two {p, r} pairs per cell; add_elem mints a token per add, lasp_orset.erl:222-241,
    261-262): the same k_or16 over twice the words, timed with HIP events."""
    R, E, k = args.wide_replicas, args.elements, 2
    a, b, c = (ctx.orset_wide_batch(R, E, k) for _ in range(3))
    a.fill_synthetic(2)
    b.fill_synthetic(3)
    for _ in range(2):
        c.join(a, b)
    ev0, ev1 = ctx.event(), ctx.event()
    ctx.synchronize()
    steps = 10
    ev0.record()
    for _ in range(steps):
        c.join(a, b)
    ev1.record()
    ctx.synchronize()
    ms = ev0.elapsed_ms(ev1) / steps
    per_elem = BYTES_PER_JOIN * k
    achieved = per_elem * R * E / (ms / 1e3) / 1e9
    del a, b, c
    ctx.synchronize()
    # HBM bytes per launch from the committed PMC passes of this join (tools/gpu_pmc_join.sh)
    traffic = None
    try:
        with open(os.path.join(ROOT, "profiles", "r06_pmc_join_t128.json")) as f:
            pm = json.load(f)
        if pm.get("replicas") == R and pm.get("elements") == E and pm.get("pairs") == k:
            traffic = pm.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return {"workload": "batched OR-Set join with 128 token slots per element "
                        "(LASPJ_KIND_ORSET_WIDE, k = 2 {p, r} pairs per cell)",
            "replicas": R, "elements": E, "token_slots": 64 * k, "kernel_ms": ms,
            "merged_elements_per_s": R * E / (ms / 1e3),
            "algorithmic_bytes_per_element": per_elem,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic}}


def list_leg(ctx):
    """lasp_core:bind/3 of config 5's 50k-entry intersection output into the previous one
    (laspj_list_bind: keys ascending -> the rank-indexed bind; reversed -> the chunked
    walk) and the Store end to end (update R -> intersection re-run -> re-bind), as
    tools/list_bench.py measures them."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from list_bench import cells, identity_order, intersection_list
    from lasp_amd import _lib, core, engine
    from lasp_amd.terms import Atom
    rng = np.random.default_rng(5)
    N, D = 100_000, 150_000
    order, _keep = identity_order(ctx, D)
    common = np.arange(D - N, N)
    pl, rl = cells(rng, len(common))
    pr, rr = cells(rng, len(common))
    old = intersection_list(common, pl, rl, pr, rr)
    pr2, rr2 = pr.copy(), rr.copy()
    pr2[rng.random(len(common)) < 0.10] |= np.uint64(8)
    rm = rng.random(len(common)) < 0.05
    rr2[rm] = pr2[rm]
    new = intersection_list(common, pl, rl, pr2, rr2)

    def rev(lst):
        runs = [lst[2][lst[1][i]:lst[1][i + 1]] for i in range(len(lst[0]))][::-1]
        return (lst[0][::-1].copy(), np.concatenate([[0], np.cumsum([len(x) for x in runs])]).astype(np.uint32),
                np.concatenate(runs))

    out = {"workload": "config 5's intersection output (50k entries {X, Cx ++ Cy}) re-bound "
                       "after R changed; the Store: update R -> intersection -> re-bind"}
    for name, (o, n) in (("us_rebind_50k", (old, new)), ("us_rebind_50k_reversed", (rev(old), rev(new)))):
        a = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*o)
        b = engine.ListBatch(ctx, _lib.KIND_ORSET_LIST).upload(*n)
        for _ in range(3):
            a.bind(b, order)
        t0 = time.perf_counter()
        for _ in range(30):
            a.bind(b, order)
        out[name] = (time.perf_counter() - t0) * 1e6 / 30
    st = core.Store(capacity=1 << 18, ctx=ctx)
    lv, rv, xv = (st.declare("lasp_orset")[1] for _ in range(3))
    tk = lambda c, e: bytes([c]) + int(e).to_bytes(19, "big")   # noqa: E731
    st.bind(lv, [(e, [(tk(1, e), False)]) for e in range(N)])
    st.bind(rv, [(e, [(tk(2, e), False)]) for e in range(D - N, D)])
    st.intersection(lv, rv, xv)
    st.update(rv, ("add_by_token", tk(3, 999), D - N + 1), Atom("a"))
    t0 = time.perf_counter()
    for i in range(10):
        st.update(rv, ("add_by_token", tk(3, i), D - N + 17 * i), Atom("a"))
    out["ms_store_update_rerun_rebind_50k"] = (time.perf_counter() - t0) / 10 * 1e3
    return out


def load_traffic(path: str, replicas: int, elements: int):
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("replicas") != replicas or d.get("elements") != elements:
        return None
    return d.get("hbm_bytes_per_launch")


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: run N rank processes under
    torch.distributed.run as a CHILD (nothing here has touched the GPU yet, and no
    process is replaced) and exit with its status."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def main():
    args = parse()
    if args.gpus < 1:
        print("bench: --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        sys.stdout.write(f"bench dry-run rank {os.environ.get('RANK', '0')} of {world}\n")
        sys.stdout.flush()
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    ae_on = args.antientropy == "on" or (args.antientropy == "auto" and world > 1)
    if world > 1 or ae_on:
        # torch first: its bundled HIP runtime is then the one liblaspj binds to
        import torch
        import torch.distributed as dist
        # one GPU per local rank; more ranks than GPUs (a rehearsal on a smaller box)
        # share them round-robin
        ndev = torch.cuda.device_count()
        local = local % ndev if ndev else local
        torch.cuda.set_device(local)
        if world == 1:                   # a one-rank group (the anti-entropy rehearsal)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)

    from lasp_amd import engine
    from lasp_amd._lib import TUNE_STREAM_GRID, TUNE_STREAM_NT, TUNE_STREAM_UNROLL

    R, E = args.replicas, args.elements
    ctx = engine.Context(local)
    if args.grid:
        ctx.set_tuning(TUNE_STREAM_GRID, args.grid)
    if args.unroll:
        ctx.set_tuning(TUNE_STREAM_UNROLL, args.unroll)
    if args.nt >= 0:
        ctx.set_tuning(TUNE_STREAM_NT, args.nt)
    a, b, c = ctx.orset_batch(R, E), ctx.orset_batch(R, E), ctx.orset_batch(R, E)
    a.fill_synthetic(2, replica_base=rank * R)
    b.fill_synthetic(3, replica_base=rank * R)
    ctx.synchronize()

    for _ in range(args.warmup):
        c.join(a, b)
    ctx.synchronize()

    def barrier():
        if dist is not None:
            dist.barrier()

    ev0, ev1 = ctx.event(), ctx.event()
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        c.join(a, b)
    ev1.record()
    ctx.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_ms(ev1) / args.steps

    if dist is not None:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())

    # the per-call legs run at N = 1 only: with more ranks, rank 0's host-side legs would
    # outlast the other ranks' anti-entropy guard (--ae-timeout) while they wait for it
    cfg1 = config1_gpu(ctx) if rank == 0 and world == 1 else None
    if cfg1 is not None:
        cfg1["steady"] = steady_leg(ctx)
    del a, b, c                          # free the 192 GiB of join operands first
    ctx.synchronize()
    wide = wide_leg(ctx, args) if rank == 0 and world == 1 and args.wide_replicas else None
    lists = list_leg(ctx) if rank == 0 and world == 1 and args.list_leg else None

    out = None
    if rank == 0:
        cells = R * E
        achieved = BYTES_PER_JOIN * cells / (kern_ms / 1000.0) / 1e9
        out = {
            "metric": METRIC,
            "value": cells * world / (wall / args.steps),
            "unit": "merged elements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall * 1000.0 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (seeded splitmix64 replicas, DESIGN.md §5)",
            "config": {
                "workload": "batched OR-Set join lasp_orset:merge/2 (BASELINE configs[1])",
                "replicas_per_gpu": R, "elements": E, "token_slots": 64,
                "global_replicas": R * world, "parallelism": f"replica shards x{world}",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": load_traffic(args.pmc, R, E),
                "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": BYTES_PER_JOIN * cells,
            },
            "cpu_baseline": None,
        }
        if cfg1 is not None:
            out["config1_gpu"] = cfg1
        if wide is not None:
            out["join_t128"] = wide
        if lists is not None:
            out["config5_list_bind"] = lists

    if ae_on:
        def abandon():
            # a collective that never completes must not cost the headline line: rank 0
            # prints it with the leg marked failed; every rank then exits with status 3
            if out is not None:
                out["antientropy"] = {"error": f"timed out after {args.ae_timeout:.0f} s"}
                print(json.dumps(out), flush=True)
            sys.stdout.flush()
            os._exit(3)

        guard = threading.Timer(args.ae_timeout, abandon)
        guard.daemon = True
        guard.start()
        try:
            ae = antientropy_leg(ctx, args, rank, world, barrier)
        except Exception as e:           # reported with the headline line, then rc 3
            ae = {"error": f"{type(e).__name__}: {e}"}
        guard.cancel()
        if out is not None:
            out["antientropy"] = ae
    else:
        ae = {}
    ae_failed = "error" in ae or not ae.get("converged", True) or \
        not ae.get("gcounter", {}).get("converged", True)

    if rank != 0:
        if ae_failed:                    # a peer may be gone: no final barrier
            os._exit(3)
        _final_barrier(dist)
        return

    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(E, args.cpu_budget)
        steady = out.get("config1_gpu", {}).get("steady")
        if isinstance(steady, dict):
            # the same step on the reference's algorithm, one core (C restatement): bind/3
            # is merge + is_inflation, read/6's threshold_met is is_inflation; update/3 and
            # the read's term copy are left out (a lower bound)
            c1 = out["cpu_baseline"]["config1"]
            steady["cpu_reference_us_per_step_lower_bound"] = c1["us_bind"] + c1["us_inflation"]
    print(json.dumps(out), flush=True)
    if ae_failed:
        print("bench: anti-entropy leg failed (see antientropy.error)", file=sys.stderr)
        sys.stdout.flush()
        os._exit(3)
    if dist is not None:
        _final_barrier(dist)


def _final_barrier(dist):
    try:
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:               # the line is printed; a lost peer is not fatal
        print(f"final barrier: {type(e).__name__}: {e}", file=sys.stderr)


if __name__ == "__main__":
    main()
