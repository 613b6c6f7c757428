#!/bin/bash
# from_binary decode: its GPU tests, then the codec suite entries (tools/bench_suite.py --only etf).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_etf.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/etf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/etf_tests.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_suite.py --only etf > gpurun_out/etf_suite.log 2>&1 || exit $?
cut -c1-200 gpurun_out/etf_suite.log
