#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace.  Stops at the first
# fault / abort / timeout (exit codes other than 0 = pass and 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests.log
ok $rc || exit $rc

timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc

if [ "${PROFILE:-0}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name '*stats*' | head
fi
