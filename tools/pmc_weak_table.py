#!/usr/bin/env python3
"""One row per kernel of `bench_suite.py --only weak` under tools/gpu_pmc_weak.sh:
average duration (kernel-trace stats), HBM bytes per dispatch (2 x FETCH_SIZE +
WRITE_SIZE, KiB, MI355X_MICROARCH.md §HBM) against the algorithmic bytes the suite
prints, and per-dispatch SQ counters (VALU / VMEM / LDS instructions per wave, the share
of wave cycles parked in s_waitcnt / barriers).  usage: pmc_weak_table.py <gpurun_out>"""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

D = sys.argv[1]


def kname(k):
    k = k.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", k).replace("void ", "").replace("laspj::", "")


def counters(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                per[(kname(r["Kernel_Name"]), int(r["Dispatch_Id"]))][r["Counter_Name"]] += \
                    float(r["Counter_Value"])
    return per


algo = {}
for f in ("weak_stats.log", "weak_pmc1.log"):
    p = os.path.join(D, f)
    if os.path.exists(p):
        for line in open(p):
            if line.startswith("{"):
                d = json.loads(line)
                algo.setdefault(d["kernel"], d)
stats = {}
for f in glob.glob(os.path.join(D, "weak_stats", "**", "*kernel_stats.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            stats[kname(r["Name"])] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
merged = collections.defaultdict(lambda: collections.defaultdict(list))
for i in range(1, 5):
    for (k, _disp), cs in counters(os.path.join(D, f"weak_pmc{i}")).items():
        for c, v in cs.items():
            merged[k][c].append(v)
order = ["config4_dataflow_fused", "config5_intersection", "config5_product_diag",
         "orset_reduce_chunks_n8", "ae_reduce_in_place_n8", "gset_join_16x"]
print("# suite rows (HIP events)")
for n in order:
    if n in algo:
        a = algo[n]
        print(f"{n:26s} {a['ms']:9.3f} ms  {a['algorithmic_bytes'] / 1e9:8.2f} GB alg  "
              f"frac {a['frac_hbm']:.3f}")
print("# kernels (rocprofv3): avg ms, calls, HBM GB per dispatch, VALU/VMEM/LDS per wave, "
      "wait share")
for k, cs in sorted(merged.items()):
    if k.startswith(("__amd", "rocprim", "k_fill")):
        continue
    med = {c: statistics.median(v) for c, v in cs.items()}
    hbm = (2 * med.get("FETCH_SIZE", 0) + med.get("WRITE_SIZE", 0)) * 1024 / 1e9
    waves = med.get("SQ_WAVES", 0) or 1
    wc = med.get("SQ_WAVE_CYCLES", 0) or 1
    ms, calls = stats.get(k, (float("nan"), 0))
    print(f"{k[:48]:48s} {ms:8.3f} {calls:3d}  HBM {hbm:8.3f} GB  "
          f"read {2 * med.get('FETCH_SIZE', 0) * 1024 / 1e9:7.3f} write {med.get('WRITE_SIZE', 0) * 1024 / 1e9:7.3f}  "
          f"VALU/w {med.get('SQ_INSTS_VALU', 0) / waves:8.1f} VMEM/w "
          f"{(med.get('SQ_INSTS_VMEM_RD', 0) + med.get('SQ_INSTS_VMEM_WR', 0)) / waves:7.1f} "
          f"LDS/w {med.get('SQ_INSTS_LDS', 0) / waves:6.1f}  "
          f"wait {med.get('SQ_WAIT_ANY', 0) / wc:5.2f} instwait {med.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
          f"active {med.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}")
