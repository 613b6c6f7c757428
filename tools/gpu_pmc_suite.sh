#!/bin/bash
# HBM traffic of every kernel in the suite: one rocprofv3 PMC pass for FETCH_SIZE and
# one for WRITE_SIZE (never combined with tracing), then a per-kernel table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CMD="python3 tools/bench_suite.py --steps 1 ${SUITE_ARGS:-}"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
    $CMD > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
    $CMD > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_table.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_table.txt
cat gpurun_out/pmc_table.txt
