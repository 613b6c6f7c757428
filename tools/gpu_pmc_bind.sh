#!/bin/bash
# rocprofv3 counter passes over the resident bind (tools/bind_probe.py): FETCH_SIZE,
# WRITE_SIZE and two SQ passes, each its own run (summarised by tools/pmc_bind_table.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export BIND_ITERS=${BIND_ITERS:-50}
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/bind_pmc$i -o run -- \
      python3 tools/bind_probe.py > gpurun_out/bind_pmc$i.log 2>&1 || exit $?
done
