#!/bin/bash
# Resident bind (laspj_var_etf_bind) A/B on one GPU: the NIF tests, then the config-1
# bind and merge probes at from_binary segment sizes (0 = the launch's own sizing), then
# a kernel trace of the default bind.  Every GPU step has its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r05d}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_nif_vars.py tests/test_gpu_nif.py > "$OUT/tests.log" 2>&1
for seg in 0 1024 512 256; do
    BIND_SEG=$seg timeout -k 10 60 python -u tools/bind_probe.py >> "$OUT/bind_seg.jsonl"
    BIND_SEG=$seg BIND_MANY=32 BIND_ITERS=40 timeout -k 10 60 python -u tools/bind_probe.py >> "$OUT/bind_many_seg.jsonl"
    NIF_SEG=$seg timeout -k 10 60 python -u tools/nif_probe.py >> "$OUT/merge_seg.jsonl"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bind -- python3 tools/bind_probe.py > "$OUT/prof.log" 2>&1
