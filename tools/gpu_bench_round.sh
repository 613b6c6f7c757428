#!/bin/bash
# The round's closing measurements: bench.py (N=1, defaults), then rocprofv3 kernel stats of
# a short bench run.  Every GPU step has its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05b}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/prof_bench.log" 2>&1
