#!/bin/bash
# rocprofv3 evidence for the kernels below 0.74 of HBM (bench_suite.py --only weak):
# kernel-trace stats, FETCH_SIZE, WRITE_SIZE and two SQ passes, each its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 tools/bench_suite.py --only weak --steps ${STEPS:-3}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/weak_stats -o run -- \
    $CMD > gpurun_out/weak_stats.log 2>&1 || exit $?
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/weak_pmc$i -o run -- \
      $CMD > gpurun_out/weak_pmc$i.log 2>&1 || exit $?
done
python3 tools/pmc_bind_table.py gpurun_out weak_pmc > gpurun_out/weak_table.txt
cat gpurun_out/weak_table.txt
