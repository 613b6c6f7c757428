#!/bin/bash
# rocprofv3 evidence for the to_binary payload kernels (tools/bench_suite.py --only etf):
# kernel-trace stats, then PMC passes, each in its own run (one counter group per pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 tools/bench_suite.py --only etf --steps 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/etf_stats -o run -- \
    $CMD > gpurun_out/etf_stats.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "WRITE_SIZE" "FETCH_SIZE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/etf_pmc$i -o run -- \
      $CMD > gpurun_out/etf_pmc$i.log 2>&1 || exit $?
done
echo etf profile ok
