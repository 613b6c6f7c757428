#!/bin/bash
# Everything the round's profiles/ cite, in one GPU session (stops at the first
# failure): parity tests, the headline bench, rocprofv3 kernel stats of the bench,
# the per-kernel suite and its kernel stats, PMC traffic of the suite, the CPU
# restatement beside the core kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
echo "bench ok"; tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_prof -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_prof.log 2>&1 || exit $?
find gpurun_out/bench_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/bench_kernel_stats.csv \;
echo "bench profile ok"
timeout -k 10 300 python -u tools/bench_suite.py --steps 5 > gpurun_out/suite.log 2>&1 || exit $?
echo "suite ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/suite_prof -o run -- \
    python3 tools/bench_suite.py --steps 3 > gpurun_out/suite_prof.log 2>&1 || exit $?
find gpurun_out/suite_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/suite_kernel_stats.csv \;
echo "suite profile ok"
bash tools/gpu_pmc_suite.sh > gpurun_out/pmc_run.log 2>&1 || exit $?
echo "pmc ok"
timeout -k 10 200 python -u tools/cpu_beside.py > gpurun_out/cpu_beside.log 2>&1 || exit $?
echo "cpu_beside ok"
