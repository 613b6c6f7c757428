#!/bin/bash
# rocprofv3 kernel-trace stats over the per-kernel suite (all kernels of the path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_suite -o run -- \
    python3 tools/bench_suite.py --steps 3 > gpurun_out/prof_suite.log 2>&1 || exit $?
find gpurun_out/prof_suite -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_suite_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/${TAG}_suite_kernel_stats.csv | cut -c1-160
