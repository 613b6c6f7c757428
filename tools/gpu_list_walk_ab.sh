#!/bin/bash
# The chunked list walk (k_merge_spec) at chunk sizes, per shape, then a kernel trace of
# the shuffled-each bind.  Every GPU step has its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05w}
mkdir -p "$OUT"
for shape in shuffled_each reversed shuffled_same; do
    for chunk in 0 256 1024 4096 16384; do
        SHAPE=$shape CHUNK=$chunk ITERS=10 timeout -k 10 60 python -u tools/list_bind_probe.py >> "$OUT/walk_ab.jsonl"
    done
done
SHAPE=shuffled_each ITERS=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o lw -- python3 tools/list_bind_probe.py > "$OUT/prof.log" 2>&1
