"""World-size-2 CPU coverage of the multi-GPU paths (gloo): the anti-entropy
orchestration (lasp_amd.gossip.anti_entropy_round) and the bench's shard layout."""

import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, %(root)r)
    import numpy as np
    import torch, torch.distributed as dist
    from lasp_amd.gossip import anti_entropy_round
    from oracle import columnar as orc

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    objects, E = 6, 33            # chunk = 3 objects per rank; odd E
    # this rank's replica of every object: synthetic stream 100 + rank
    mine = np.stack([orc.synth_orset(100 + rank, o, E) for o in range(objects)])
    state = torch.from_numpy(mine.reshape(-1).view(np.int64).copy())
    recv = torch.empty_like(state)
    chunk = torch.empty(state.numel() // world, dtype=torch.int64)

    def reduce_fn():     # CPU stand-in for laspj_batch_reduce_chunks (tested on GPU)
        r = recv.numpy().view(np.uint64).reshape(world, -1)
        chunk.numpy().view(np.uint64)[:] = np.bitwise_or.reduce(r, axis=0)

    anti_entropy_round(state, recv, chunk, reduce_fn)
    got = state.numpy().view(np.uint64).reshape(objects, E, 2)
    want = np.zeros_like(mine)
    for r in range(world):
        want |= np.stack([orc.synth_orset(100 + r, o, E) for o in range(objects)])
    assert np.array_equal(got, want), "anti-entropy did not converge to the join"
    # a second round is idempotent (the join is already everywhere)
    anti_entropy_round(state, recv, chunk, reduce_fn)
    assert np.array_equal(state.numpy().view(np.uint64).reshape(objects, E, 2), want)
    # bench shard layout: rank r's join shard is synthetic replicas [r*R, (r+1)*R)
    R = 4
    bases = [None] * world
    dist.all_gather_object(bases, rank * R)
    assert bases == [r * R for r in range(world)]
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)        # bench takes the max wall time
    assert t.item() == float(world)
    # G-Counter anti-entropy: one all_reduce(MAX) = riak_dt_gcounter's per-actor max
    from lasp_amd.gossip import gcounter_anti_entropy_round
    objs, actors = 5, 7
    rng = [np.random.default_rng(40 + r) for r in range(world)]
    views = [g.integers(0, 1 << 40, (objs, actors)).astype(np.int64) for g in rng]
    counts = torch.from_numpy(views[rank].copy())
    gcounter_anti_entropy_round(counts)
    want = np.maximum.reduce(views)
    assert np.array_equal(counts.numpy(), want)
    gcounter_anti_entropy_round(counts)             # idempotent
    assert np.array_equal(counts.numpy(), want)
    # counts at and above 2^63 (uint64 in int64 words): the join is the UNSIGNED max,
    # as the device join / reduces compute it
    big = [g.integers(0, 1 << 64, (objs, actors), dtype=np.uint64) for g in
           [np.random.default_rng(70 + r) for r in range(world)]]
    big[0][0, 0], big[1][0, 0] = np.uint64(1 << 63), np.uint64(5)
    counts = torch.from_numpy(big[rank].view(np.int64).copy())
    gcounter_anti_entropy_round(counts)
    assert np.array_equal(counts.numpy().view(np.uint64), np.maximum.reduce(big))
    print("ok", rank)
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_anti_entropy_gloo_world2(tmp_path):
    from oracle import columnar
    columnar.lib()
    script = tmp_path / "worker.py"
    script.write_text(WORKER % {"root": ROOT})
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(script)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    assert res.stdout.count("ok") == 2


def test_bench_self_launches_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (torch.distributed.run
    as a child process) and each sees WORLD_SIZE=2; a launcher world that disagrees
    with --gpus is refused with a non-zero status."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--dry-run"], capture_output=True, text=True, timeout=120, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    import re
    assert sorted(re.findall(r"bench dry-run rank \d+ of \d+", res.stdout)) == \
        ["bench dry-run rank 0 of 2", "bench dry-run rank 1 of 2"], res.stdout
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--dry-run"], capture_output=True, text=True, timeout=60,
                         env=dict(env, WORLD_SIZE="1", RANK="0"))
    assert bad.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in bad.stderr
