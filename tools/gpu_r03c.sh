#!/bin/bash
# Round 3 pass 3: the list / store GPU tests after the incremental rank tables, then the
# list re-bind rows (incl. the Store end to end), each step under its own limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
PROFILE_STORE=1 timeout -k 10 300 python -u tools/list_bench.py > gpurun_out/list_bench.log 2> gpurun_out/list_bench_prof.txt
rc=$?; echo "list_bench rc=$rc"; tail -c 1500 gpurun_out/list_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/bench.log
exit $rc
