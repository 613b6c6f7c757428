#!/bin/bash
# PMC passes over the from_binary probe for ONE workload (ONLY=t64 / t3): instruction
# mix, activity and waits of the decode kernel, one counter group per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ONLY=${ONLY:-t64}
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SENDMSG"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/${OP:-read}_${ONLY}_pmc$i -o run -- \
      python3 tools/etf_read_probe.py --only $ONLY --op ${OP:-read} --reps 1 > gpurun_out/${OP:-read}_${ONLY}_pmc$i.log 2>&1 || exit $?
done
echo read profile ok
