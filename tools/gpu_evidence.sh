#!/bin/bash
# Round evidence in one GPU session: parity tests, the per-kernel suite, the CPU
# restatement timed beside the core kernels, and the rocprofv3 kernel stats of the
# suite.  Stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
ok $rc || exit $rc
timeout -k 10 300 python -u tools/bench_suite.py --steps 5 > gpurun_out/suite.log 2>&1 || exit $?
echo suite ok
timeout -k 10 200 python -u tools/cpu_beside.py > gpurun_out/cpu_beside.log 2>&1 || exit $?
echo cpu_beside ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/suite_prof -o run -- \
    python3 tools/bench_suite.py --steps 3 > gpurun_out/suite_prof.log 2>&1 || exit $?
find gpurun_out/suite_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/suite_kernel_stats.csv \;
echo profile ok
