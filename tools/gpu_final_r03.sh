#!/bin/bash
# Round-3 closing evidence in one GPU session (stops at the first failure): the GPU
# parity tests, smoke(), the headline bench, rocprofv3 kernel stats + FETCH / WRITE
# passes of the bench (tools/gpu_profile.sh), the per-kernel suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/final_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/final_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
echo "bench ok"; tail -1 gpurun_out/final_bench.log | cut -c1-400
TAG=r03z bash tools/gpu_profile.sh > gpurun_out/final_prof.log 2>&1 || exit $?
echo "profile ok"
timeout -k 10 300 python -u tools/bench_suite.py --steps 5 > gpurun_out/final_suite.log 2>&1 || exit $?
echo "suite ok"
