#!/bin/bash
# GPU tests, then the per-kernel suite; stop at the first fault/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/bench_suite.py ${SUITE_ARGS:-} > gpurun_out/suite.log 2>&1
rc2=$?; echo "suite rc=$rc2"; cat gpurun_out/suite.log | cut -c1-220
exit $(( rc > rc2 ? rc : rc2 ))
