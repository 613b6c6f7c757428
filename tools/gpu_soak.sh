#!/bin/bash
# Device soak of the list / store / codec tests (hypothesis examples x LASPJ_SOAK),
# output to a file that grows as tests pass (-v) so the run shows progress.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LASPJ_SOAK=${SOAK:-10} timeout -k 10 ${LIMIT:-600} python -u -m pytest \
    tests/test_gpu_lists.py tests/test_gpu_lists_sorted.py tests/test_gpu_core.py \
    tests/test_gpu_random.py tests/test_etf.py -m gpu -x -v -p no:cacheprovider \
    --timeout 400 --timeout-method thread > gpurun_out/soak.log 2>&1
rc=$?; echo "soak rc=$rc"; grep -E "passed|failed|error" gpurun_out/soak.log | tail -3
exit $rc
