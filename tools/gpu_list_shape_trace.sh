#!/bin/bash
# Kernel traces of one list bind per shape (tools/list_bind_probe.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05st}
mkdir -p "$OUT"
for shape in ${SHAPES:-shuffled_each}; do
    SHAPE=$shape ITERS=5 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$shape" -o t -- python3 tools/list_bind_probe.py > "$OUT/$shape.log" 2>&1
done
