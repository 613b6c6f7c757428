#!/bin/bash
# One GPU call = a few steps, each under its own time limit, stopping at the first
# failure.  Usage: tools/gpu_step.sh "<pytest -k expr or file list>" [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
    timeout -k 10 ${TLIMIT:-400} python -u -m pytest $TESTS ${KEXPR:+-k "$KEXPR"} -m gpu -x -v \
        --timeout 150 --timeout-method thread > gpurun_out/tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3
    [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${TOOL:-}" ]; then
    timeout -k 10 ${TOOL_LIMIT:-300} python -u $TOOL > gpurun_out/tool.log 2>&1
    rc=$?; echo "tool rc=$rc"; tail -3 gpurun_out/tool.log
    [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH:-}" ]; then
    timeout -k 10 ${BENCH_LIMIT:-300} python -u bench.py $BENCH > gpurun_out/bench.log 2>&1
    rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
    exit $rc
fi
