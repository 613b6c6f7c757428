#!/bin/bash
# A/B: the same join sweep point with /opt/rocm's HIP runtime vs torch's bundled one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS="--grids 16384 --unrolls 2 --nts 1 --steps 10"
for i in 1 2; do
  timeout -k 10 120 python -u tools/sweep_join.py $ARGS > gpurun_out/ab_plain_$i.log 2>&1 || exit $?
  timeout -k 10 120 python -u -c "import torch; torch.zeros(1, device='cuda'); import runpy, sys; sys.argv=['sweep_join.py'] + '$ARGS'.split(); runpy.run_path('tools/sweep_join.py', run_name='__main__')" > gpurun_out/ab_torch_$i.log 2>&1 || exit $?
done
grep -h GBps gpurun_out/ab_*.log
