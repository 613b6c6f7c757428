#!/bin/bash
# from_binary per-element vs per-record cost (tools/decoder_probe.py): timing, then one
# SQ counter pass per dispatch
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/decoder_probe.py > gpurun_out/decoder_probe.log 2>&1 || exit $?
cat gpurun_out/decoder_probe.log
STEPS=2 KS=${PMC_KS:-4,32,64} timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  --output-format csv -d gpurun_out/dec_pmc -o run -- python3 tools/decoder_probe.py > gpurun_out/decoder_probe_pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = sorted(glob.glob("gpurun_out/dec_pmc/**/*counter_collection.csv", recursive=True))
rows = list(csv.DictReader(open(f[0])))
by = collections.OrderedDict()
for r in rows:
    if "etf_read" not in r["Kernel_Name"]:
        continue
    key = (int(r["Dispatch_Id"]), r["Kernel_Name"][:60])
    by.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
with open("gpurun_out/decoder_probe_pmc.txt", "w") as o:
    for (i, n), c in by.items():
        print(i, n, {k: f"{v:.4g}" for k, v in sorted(c.items())}, file=o)
print(open("gpurun_out/decoder_probe_pmc.txt").read())
PY
