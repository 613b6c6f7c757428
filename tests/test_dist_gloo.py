"""CPU coverage of the multi-GPU paths (gloo, world sizes 2, 4 and 8).

The anti-entropy round bench.py runs at N > 1 is `laspj_antientropy` (laspj_comm.hip),
which executes the steps of `laspj_antientropy_plan` on RCCL.  Here every rank asks the
same library for the same plan and executes exactly those steps with gloo point-to-point
calls over host buffers: SEND / RECV steps of one group posted together (an RCCL group),
REDUCE as the kind's join over the received copies, ALLREDUCE_MAX as an unsigned max.
Small piece sizes force many pieces per chunk, as 1 GiB pieces do at BASELINE config 3
(64 GiB per GPU).  After one round every rank must hold the join of every rank's
replica of every object (the reference's fan-out -> foldl(merge) -> repair,
lasp_update_fsm.erl:174-216), checked against numpy and, on sampled objects, against the
C restatement's orddict merge fold.
"""

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
    from lasp_amd import _lib
    from lasp_amd.engine import antientropy_plan
    from oracle import columnar as orc

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    SIGN = np.uint64(1 << 63)

    def run_round(kind, state, recv, piece):
        '''Execute this rank's plan: state / recv are uint64 numpy arrays.'''
        plan = antientropy_plan(kind, rank, world, state.size, piece)
        ts = torch.from_numpy(state.view(np.int64))
        tr = torch.from_numpy(recv.view(np.int64)) if recv is not None else None
        groups = {}
        for s in plan:
            groups.setdefault(s["group"], []).append(s)
        assert sorted(groups) == list(range(len(groups)))
        for g in range(len(groups)):
            reqs = []
            for s in groups[g]:
                o, w = s["offset"], s["words"]
                if s["op"] in (_lib.AE_SEND, _lib.AE_RECV):
                    buf = ts if s["buf"] == _lib.AE_BUF_STATE else tr
                    view = buf[o:o + w]
                    if s["op"] == _lib.AE_SEND:
                        reqs.append(dist.isend(view, s["peer"], tag=s["tag"]))
                    else:
                        reqs.append(dist.irecv(view, s["peer"], tag=s["tag"]))
                elif s["op"] == _lib.AE_REDUCE:
                    assert len(groups[g]) == 1
                    runs = [recv[s["src"] + j * w:s["src"] + (j + 1) * w] for j in range(s["nsrc"])]
                    state[o:o + w] = np.bitwise_or.reduce([state[o:o + w]] + runs)
                elif s["op"] == _lib.AE_ALLREDUCE_MAX:
                    # riak_dt_gcounter's join is the per-actor max of uint64 counts: the
                    # sign flip makes gloo's signed max the unsigned one
                    state[o:o + w] ^= SIGN
                    dist.all_reduce(ts[o:o + w], op=dist.ReduceOp.MAX)
                    state[o:o + w] ^= SIGN
                else:
                    raise AssertionError(s)
            for r in reqs:
                r.wait()
        return plan

    # ---- OR-Set: objects x E cells {p, r}; this rank's replica = synthetic stream 100 + rank
    objects, E = 4 * world, 33
    mine = np.stack([orc.synth_orset(100 + rank, o, E) for o in range(objects)])
    state = mine.reshape(-1).copy()
    recv = np.full(state.size // world * (world - 1), 0xDEAD, np.uint64)
    want = np.zeros_like(mine)
    for r in range(world):
        want |= np.stack([orc.synth_orset(100 + r, o, E) for o in range(objects)])
    for piece in (0, 7, 66):
        state[:] = mine.reshape(-1)
        plan = run_round(_lib.KIND_ORSET, state, recv, piece)
        assert np.array_equal(state.reshape(mine.shape), want), ("not the join", piece)
    assert any(s["op"] == _lib.AE_REDUCE for s in plan)
    tokens = orc.synth_tokens(E)
    for o in (0, objects - 1):
        acc = orc.ORDict.from_cells(orc.synth_orset(100, o, E), tokens)
        for r in range(1, world):
            acc = acc.merge(orc.ORDict.from_cells(orc.synth_orset(100 + r, o, E), tokens))
        assert orc.ORDict.from_cells(state.reshape(mine.shape)[o], tokens).equal(acc), o
    # a second round is idempotent (the join is already everywhere)
    run_round(_lib.KIND_ORSET, state, recv, 7)
    assert np.array_equal(state.reshape(mine.shape), want)

    # ---- G-Set: objects x ceil(E/64) words
    gw = 3
    gmine = np.stack([np.random.default_rng(300 + rank).integers(0, 1 << 63, (gw,), dtype=np.uint64)
                      for _ in range(2 * world)])
    gstate = gmine.reshape(-1).copy()
    grecv = np.zeros(gstate.size // world * (world - 1), np.uint64)
    gwant = np.bitwise_or.reduce([np.stack([np.random.default_rng(300 + r).integers(
        0, 1 << 63, (gw,), dtype=np.uint64) for _ in range(2 * world)]) for r in range(world)])
    run_round(_lib.KIND_GSET, gstate, grecv, 4)
    assert np.array_equal(gstate.reshape(gmine.shape), gwant)

    # ---- G-Counter: all-reduce(max) in pieces, counts at and above 2^63 included
    objs, actors = 5, 7
    big = [np.random.default_rng(70 + r).integers(0, 1 << 64, (objs, actors), dtype=np.uint64)
           for r in range(world)]
    big[0][0, 0], big[-1][0, 0] = np.uint64(1 << 63), np.uint64(5)
    counts = big[rank].reshape(-1).copy()
    run_round(_lib.KIND_GCOUNTER, counts, None, 6)
    assert np.array_equal(counts.reshape(objs, actors), np.maximum.reduce(big))

    # ---- bench shard layout: rank r's join shard is synthetic replicas [r*R, (r+1)*R)
    R = 4
    bases = [None] * world
    dist.all_gather_object(bases, rank * R)
    assert bases == [r * R for r in range(world)]
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)        # bench takes the max wall time
    assert t.item() == float(world)
    print("ok", rank, flush=True)
    # every rank done before any closes its pairs (a peer's early exit aborted gloo's
    # pair threads in another rank under load)
    dist.barrier()
    dist.destroy_process_group()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4, 8])
def test_antientropy_plan_over_gloo(tmp_path, world):
    from lasp_amd import build
    from oracle import columnar
    build.build()
    columnar.lib()
    script = tmp_path / "worker.py"
    script.write_text(WORKER % {"root": ROOT})
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", str(script)]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-4000:]
    assert res.stdout.count("ok") == world


def test_antientropy_plan_shape():
    """Host-only properties of the plan for every world size 1..8: every SEND is matched
    by one RECV on its peer (same group, tag and length), groups hold at most 2(n-1)
    point-to-point steps, every word of recv is written exactly once before the REDUCE,
    and every non-owned chunk of state is overwritten exactly once by the all-gather."""
    from lasp_amd import _lib, build
    from lasp_amd.engine import antientropy_plan
    build.build()
    for n in range(1, 9):
        cw, piece = 2 * 37, 10
        plans = [antientropy_plan(_lib.KIND_ORSET, r, n, n * cw, piece) for r in range(n)]
        if n == 1:
            assert plans == [[]]
            continue
        for r, plan in enumerate(plans):
            per_group = {}
            for s in plan:
                per_group.setdefault(s["group"], []).append(s)
            red = [s for s in plan if s["op"] == _lib.AE_REDUCE]
            assert len(red) == 1 and red[0]["offset"] == r * cw and red[0]["nsrc"] == n - 1
            for g, steps in per_group.items():
                p2p = [s for s in steps if s["op"] in (_lib.AE_SEND, _lib.AE_RECV)]
                assert len(p2p) <= 2 * (n - 1)
                assert all(s["words"] <= piece for s in p2p)
            seen_recv = [0] * ((n - 1) * cw)
            seen_state = [0] * (n * cw)
            for s in plan:
                if s["op"] == _lib.AE_SEND:
                    match = [t for t in plans[s["peer"]] if t["op"] == _lib.AE_RECV and
                             t["peer"] == r and t["group"] == s["group"] and t["tag"] == s["tag"]]
                    assert len(match) == 1 and match[0]["words"] == s["words"]
                if s["op"] == _lib.AE_RECV:
                    tgt = seen_recv if s["buf"] == _lib.AE_BUF_RECV else seen_state
                    for w in range(s["offset"], s["offset"] + s["words"]):
                        tgt[w] += 1
                    if s["buf"] == _lib.AE_BUF_RECV:
                        assert s["group"] < red[0]["group"]
                    else:
                        assert s["group"] > red[0]["group"]
            assert seen_recv == [1] * ((n - 1) * cw)
            assert seen_state == [0 if w // cw == r else 1 for w in range(n * cw)]
    L = _lib.load()
    import ctypes as C
    cnt = C.c_uint64()
    assert L.laspj_antientropy_plan(_lib.KIND_ORSET, 0, 3, 10, 0, None, 0, C.byref(cnt)) == \
        _lib.E_INVAL                                    # 10 words do not split 3 ways
    arr = (_lib.AEStep * 1)()
    assert L.laspj_antientropy_plan(_lib.KIND_ORSET, 0, 2, 8, 1, arr, 1, C.byref(cnt)) == \
        _lib.E_RANGE and cnt.value > 1
    assert C.sizeof(_lib.AEStep) == 48


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
