#!/bin/bash
# List bind/3 (laspj_list_bind) on one GPU: the list bench (config 5 re-binds, the Store
# update), then a kernel trace of the 50k intersection re-bind.  Every GPU step has its
# own time limit.  $2 = 1 also runs the list GPU tests first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05l}
mkdir -p "$OUT"
if [ "${2:-0}" = 1 ]; then
    timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
        tests/test_gpu_lists.py tests/test_gpu_lists_sorted.py tests/test_gpu_lists_walk.py \
        tests/test_gpu_core.py > "$OUT/tests.log" 2>&1
fi
timeout -k 10 300 python -u tools/list_bench.py > "$OUT/list_bench.log" 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o lb -- python3 tools/list_bind_probe.py > "$OUT/prof.log" 2>&1
if [ "${3:-0}" = 1 ]; then
    timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
        tests/test_gpu_nif.py tests/test_gpu_nif_vars.py > "$OUT/nif_tests.log" 2>&1
    timeout -k 10 120 python -u tools/nif_probe.py > "$OUT/nif_probe.log" 2>&1
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/nprof" -o nif -- python3 tools/nif_probe.py > "$OUT/nprof.log" 2>&1
fi
