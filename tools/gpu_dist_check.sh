#!/bin/bash
# torch-first runtime check + single-rank rehearsal of the multi-process bench path
# (gloo barrier, nccl anti-entropy leg) on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/torch_first_check.py > gpurun_out/tf.log 2>&1
rc=$?; echo "torch-first rc=$rc"; tail -4 gpurun_out/tf.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --steps 5 --warmup 1 --no-cpu \
    --antientropy on > gpurun_out/bench_dist1.log 2>&1
rc=$?; echo "bench-dist1 rc=$rc"; tail -3 gpurun_out/bench_dist1.log
exit $rc
