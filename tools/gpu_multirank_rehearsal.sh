#!/bin/bash
# The bench's N > 1 join path rehearsed on one GPU: 2 and 4 ranks (torchrun, gloo
# barriers, max-over-ranks) sharing the card with smaller shards; the anti-entropy leg
# needs one GPU per rank (RCCL) and is off here.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 5 \
      --warmup 1 --replicas $((524288 / n)) --antientropy off > gpurun_out/bench_rehearse$n.log 2>&1
  rc=$?; echo "n=$n rc=$rc"; grep -o '"value": [0-9.e+]*, "unit": "[^"]*", "n_gpus": [0-9]*' gpurun_out/bench_rehearse$n.log
  [ $rc -eq 0 ] || exit $rc
done
