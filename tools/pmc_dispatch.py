#!/usr/bin/env python3
"""Per-dispatch PMC counter table from rocprofv3 --pmc CSV directories.
usage: pmc_dispatch.py <kernel-substring> <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

key = sys.argv[1]
for d in sys.argv[2:]:
    rows = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    print(d)
    for i in sorted(rows):
        print("  ", i, " ".join(f"{c}={v:.4g}" for c, v in sorted(rows[i].items())))
