#!/bin/bash
# GPU parity tests only (optionally a subset: TESTS="tests/test_x.py ..."), one process,
# per-test timeout; stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TLIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu ${PYARGS:--x} -v \
    --timeout 150 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests.log | tail -3
exit $rc
