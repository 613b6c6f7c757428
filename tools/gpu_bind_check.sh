#!/bin/bash
# list-value bind path: the list / store GPU tests, then tools/list_bench.py (re-binds and
# the Store end to end)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_lists_sorted.py tests/test_gpu_core.py tests/test_gpu_random.py tests/test_gpu_many.py tests/test_list_space.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/bind_tests.log 2>&1
rc=$?; tail -3 gpurun_out/bind_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/list_bench.py > gpurun_out/list_bench.log 2>&1 || exit $?
tail -c 600 gpurun_out/list_bench.log
