#!/usr/bin/env python3
"""Host HIP API calls and device kernels of a rocprofv3 csv run (--hip-trace
--kernel-trace --output-format csv), merged on one clock: the last N events with start
times relative to the first of them (microseconds) — where one call's host time goes."""
import csv
import sys


def short(name):
    n = str(name).replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].replace("laspj::", "")[:48]


def main(prefix, last):
    ev = []
    for r in csv.DictReader(open(prefix + "_hip_api_trace.csv")):
        fn = r.get("Function") or r.get("Operation") or ""
        if fn.startswith("__hip") or fn == "hipGetLastError":
            continue
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "host " + fn))
    for r in csv.DictReader(open(prefix + "_kernel_trace.csv")):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "  gpu " + short(r["Kernel_Name"])))
    ev.sort()
    ev = ev[-last:]
    t0 = ev[0][0]
    for s, e, n in ev:
        print("%9.1f %8.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, n))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
