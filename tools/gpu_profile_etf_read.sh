#!/bin/bash
# Counters of the from_binary kernels (tools/etf_read_probe.py): kernel-trace stats,
# then one PMC pass per counter group, each in its own run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KNOB=${KNOB:-0}
CMD="python3 tools/etf_read_probe.py --reps 1 --knob $KNOB"
timeout -k 10 120 $CMD > gpurun_out/rd_probe.log 2>&1 || exit $?
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rd_stats -o run -- \
    $CMD > gpurun_out/rd_stats.log 2>&1 || exit $?
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/rd_pmc$i -o run -- \
      $CMD > gpurun_out/rd_pmc$i.log 2>&1 || exit $?
done
python3 tools/pmc_dispatch.py etf_read gpurun_out/rd_pmc1 gpurun_out/rd_pmc2 > gpurun_out/rd_pmc_table.txt 2>&1
echo rd profile ok
