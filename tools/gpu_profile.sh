#!/bin/bash
# rocprofv3 evidence for the join kernel: kernel-trace stats, then one PMC pass per
# counter (FETCH_SIZE, WRITE_SIZE), each in its own run; summary into gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS="--steps 5 --warmup 1 --no-cpu --wide-replicas 0 --list-leg 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stats -o run -- \
    python3 bench.py $ARGS > gpurun_out/prof_stats.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o run -- \
    python3 bench.py $ARGS > gpurun_out/prof_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o run -- \
    python3 bench.py $ARGS > gpurun_out/prof_write.log 2>&1 || exit $?
python3 tools/pmc_summary.py --stats-dir gpurun_out/prof_stats --fetch-dir gpurun_out/prof_fetch \
    --write-dir gpurun_out/prof_write --out gpurun_out/${TAG}_pmc_join.json
find gpurun_out/prof_stats -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
tail -2 gpurun_out/prof_stats.log
