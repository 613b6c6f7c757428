#!/bin/bash
# Round-3 evidence pass 2: weak-kernel rocprofv3 stats + PMC, stream ceilings by size,
# list re-bind rows.  Each step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_keyed.py tests/test_gpu_configs.py -k "config4 or keyed" -m gpu -x -q \
    --timeout 150 --timeout-method thread > gpurun_out/tests_c4.log 2>&1
rc=$?; echo "tests c4 rc=$rc"; tail -3 gpurun_out/tests_c4.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_suite.py --only gather_ab --steps 5 > gpurun_out/gather_ab.log 2>&1
rc=$?; echo "gather_ab rc=$rc"; cut -c1-140 gpurun_out/gather_ab.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_pmc_weak.sh > gpurun_out/pmc_weak.out 2>&1
rc=$?; echo "pmc_weak rc=$rc"; tail -20 gpurun_out/pmc_weak.out
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_suite.py --only ceilings --steps 5 > gpurun_out/ceilings.log 2>&1
rc=$?; echo "ceilings rc=$rc"; cut -c1-160 gpurun_out/ceilings.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/list_bench.py > gpurun_out/list_bench.log 2>&1
rc=$?; echo "list_bench rc=$rc"; tail -c 3000 gpurun_out/list_bench.log
exit $rc
