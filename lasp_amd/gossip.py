"""Gossip anti-entropy across GPUs (BASELINE config 3).

The reference's fan-out -> N-way fold-merge -> read-repair (lasp_update_fsm.erl:174-216,
lasp_bind_fsm.erl:170-212) is an all-reduce whose operator is the lattice join.  Each
rank holds one replica of every object; after one round every rank holds the join of
all ranks' replicas.  RCCL has no bitwise-OR reduction (rccl.h: sum/prod/max/min/avg),
and `max` on packed masks is not a join, so a round is

  1. all_to_all_single  — rank j receives every rank's copy of object chunk j
                          (the reduce-scatter layout), (n-1)/n * S bytes per GPU;
  2. reduce_chunks      — one HIP kernel joins the n copies in HBM (laspj_batch_reduce_chunks;
                          the kind's join: OR for set bitmaps, per-actor max for G-Counters);
  3. all_gather         — the joined chunks are redistributed, (n-1)/n * S bytes per GPU.

Per-GPU xGMI traffic 2(n-1)/n * S, the same as a ring all-reduce, but the all-to-all
phase drives all n-1 peer links at once instead of one ring neighbour.

`anti_entropy_round` is the whole orchestration; it runs over torch.distributed with
the nccl (= RCCL) backend on GPUs, and over gloo on CPU tensors in the tests, where the
caller supplies the reduce.

G-Counters are the one lattice here whose join IS a numeric max: riak_dt_gcounter
merges per actor with max (the counter behind the ad counter's threshold reads,
lasp_lattice.erl:87-90), so their anti-entropy is a single RCCL all_reduce(MAX) over
the count words (`gcounter_anti_entropy_round`), with no custom reduce.
"""

from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def anti_entropy_round(state: torch.Tensor, recv: torch.Tensor, chunk: torch.Tensor,
                       reduce_fn: Callable[[], None], group=None,
                       sync: Optional[Callable[[], None]] = None) -> None:
    """One anti-entropy round over flat int64 tensors: `state` (S bytes, objects laid
    out chunk-major: rank j owns chunk j), `recv` (S bytes) and `chunk` (S/n bytes).
    `reduce_fn()` must leave chunk[i] = ⊔_j recv[j*|chunk| + i] (the kind's join)."""
    world = dist.get_world_size(group)
    if state.numel() % world or chunk.numel() * world != state.numel() or \
            recv.numel() != state.numel():
        raise ValueError("state must split into world equal chunks")
    dist.all_to_all_single(recv, state, group=group)
    if sync:
        sync()
    reduce_fn()
    dist.all_gather_into_tensor(state, chunk, group=group)
    if sync:
        sync()


class DeviceAntiEntropy:
    """Device-resident anti-entropy over `objects` OR-Set objects of E element slots:
    this rank's replicas live in `state`; the reduce is the HIP kernel (OR-Sets only:
    G-Counters go through DeviceGCounterAntiEntropy)."""

    def __init__(self, ctx, objects: int, elements: int, group=None):
        from . import engine
        self.ctx = ctx
        self.group = group
        self.world = dist.get_world_size(group)
        if objects % self.world:
            raise ValueError("objects must be a multiple of the world size")
        self.objects, self.elements = objects, elements
        words = objects * 2 * elements
        dev = torch.device("cuda", ctx.device)
        self.state = torch.empty(words, dtype=torch.int64, device=dev)
        self.recv = torch.empty_like(self.state)
        self.chunk = torch.empty(words // self.world, dtype=torch.int64, device=dev)
        self.state_b = engine.WrappedORSetBatch(ctx, self.state, objects, elements)
        self.recv_b = engine.WrappedORSetBatch(ctx, self.recv, objects, elements)
        self.chunk_b = engine.WrappedORSetBatch(ctx, self.chunk, objects // self.world, elements)
        self.bytes = words * 8

    def fill(self, seed: int, replica_base: int = 0):
        self.state_b.fill_synthetic(seed, replica_base)
        self.ctx.synchronize()

    def _sync(self):
        torch.cuda.current_stream(self.state.device).synchronize()

    def _reduce(self):
        self.chunk_b.reduce_chunks(self.recv_b, self.world)
        self.ctx.synchronize()

    def round(self):
        anti_entropy_round(self.state, self.recv, self.chunk, self._reduce, self.group,
                           self._sync)


_SIGN = -(1 << 63)


def gcounter_anti_entropy_round(counts: torch.Tensor, group=None) -> None:
    """One G-Counter anti-entropy round: counts (int64 words holding uint64 counts,
    objects x actors, this rank's replica of every object) become the per-actor max
    over all ranks = the riak_dt_gcounter join.  torch.distributed's MAX on int64 is a
    signed max; flipping the sign bit before and after makes it the unsigned max the
    device join and reduces use (u ≤ v  ⇔  (u ^ 2^63) ≤ (v ^ 2^63) as signed), so
    counts at or above 2^63 join the same way on both paths."""
    counts.bitwise_xor_(_SIGN)
    dist.all_reduce(counts, op=dist.ReduceOp.MAX, group=group)
    counts.bitwise_xor_(_SIGN)


class DeviceGCounterAntiEntropy:
    """Device-resident G-Counter anti-entropy over `objects` counters of `actors` actor
    slots; `batch` exposes the state to the engine (values, threshold reads)."""

    def __init__(self, ctx, objects: int, actors: int, group=None):
        from . import engine
        self.ctx, self.group = ctx, group
        self.objects, self.actors = objects, actors
        dev = torch.device("cuda", ctx.device)
        self.state = torch.empty(objects * actors, dtype=torch.int64, device=dev)
        self.batch = engine.WrappedGCounterBatch(ctx, self.state, objects, actors)
        self.bytes = objects * actors * 8

    def fill(self, rank: int, world: int):
        """Synthetic replicas: rank r has counted its own actors (a % world == r) up to
        their current totals and holds stale views (up to 3 behind) of the others."""
        o = torch.arange(self.objects, device=self.state.device, dtype=torch.int64)
        a = torch.arange(self.actors, device=self.state.device, dtype=torch.int64)
        total = (o[:, None] * 7919 + a[None, :] * 104729) % 100003 + 8
        lag = (o[:, None] * 31 + a[None, :] * 17 + rank * 13) % 4
        own = (a[None, :] % world) == rank
        self.state.view(self.objects, self.actors).copy_(torch.where(own, total, total - 1 - lag))
        torch.cuda.current_stream(self.state.device).synchronize()

    def round(self):
        gcounter_anti_entropy_round(self.state, self.group)
