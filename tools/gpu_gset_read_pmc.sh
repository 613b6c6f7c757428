#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05gsp
export TMPDIR=/tmp
export KNOBS=0 STEPS=3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r05gsp/p1 -o run -- python3 tools/gset_read_probe.py > gpurun_out/r05gsp/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d gpurun_out/r05gsp/p2 -o run -- python3 tools/gset_read_probe.py > gpurun_out/r05gsp/p2.log 2>&1 || exit $?
