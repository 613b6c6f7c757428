#!/bin/bash
# Every GPU test in one process (time-limited), then the list bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05full}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python -u tools/list_bench.py > "$OUT/list_bench.log" 2>&1
