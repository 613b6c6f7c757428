#!/bin/bash
# Round 3 pass 4: ETF tests, config-1 end to end under a rocprofv3 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_etf.py tests/test_gpu_configs.py -m gpu -x -q \
    --timeout 150 --timeout-method thread > gpurun_out/tests_etf.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests_etf.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c1_prof -o run -- \
    python3 tools/config1_e2e.py > gpurun_out/c1.log 2>&1
rc=$?; echo "c1 rc=$rc"; tail -c 1200 gpurun_out/c1.log
exit $rc
