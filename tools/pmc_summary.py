#!/usr/bin/env python3
"""Summarise rocprofv3 outputs for the join kernel into profiles/.

  kernel stats : <dir>/**/*kernel_stats.csv (rocprofv3 --kernel-trace --stats)
  PMC passes   : <fetch_dir>/**/*counter_collection.csv with FETCH_SIZE, and
                 <write_dir>/**/*counter_collection.csv with WRITE_SIZE.
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports exactly half of a 16-B-per-lane streaming read, so
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
"""
import argparse
import csv
import glob
import json
import os
import statistics


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def counter(dirpath, name, kernel_sub):
    vals = {}
    for r in rows(os.path.join(dirpath, "**", "*counter_collection.csv")):
        if r.get("Counter_Name") != name or kernel_sub not in r.get("Kernel_Name", ""):
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats-dir", required=True)
    ap.add_argument("--fetch-dir", required=True)
    ap.add_argument("--write-dir", required=True)
    ap.add_argument("--kernel", default="k_or16<2")
    ap.add_argument("--replicas", type=int, default=1 << 20)
    ap.add_argument("--elements", type=int, default=4096)
    ap.add_argument("--pairs", type=int, default=1,
                    help="{p, r} pairs per cell (2: the T = 128 wide join)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    stats = [r for r in rows(os.path.join(a.stats_dir, "**", "*kernel_stats.csv"))
             if a.kernel in r.get("Name", "")]
    fetch = counter(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write = counter(a.write_dir, "WRITE_SIZE", a.kernel)
    algo = 48 * a.pairs * a.replicas * a.elements
    f_kib = statistics.median(fetch) if fetch else None
    w_kib = statistics.median(write) if write else None
    hbm = (2 * f_kib + w_kib) * 1024 if fetch and write else None
    out = {
        "kernel": a.kernel, "replicas": a.replicas, "elements": a.elements, "pairs": a.pairs,
        "algorithmic_bytes_per_launch": algo,
        "fetch_size_kib_per_launch": f_kib, "write_size_kib_per_launch": w_kib,
        "fetch_launches": len(fetch), "write_launches": len(write),
        "hbm_bytes_per_launch": hbm,
        "traffic_over_algorithmic": (hbm / algo) if hbm else None,
        "kernel_stats": stats,
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halves 16-B streaming reads)",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernel_stats"}))


if __name__ == "__main__":
    main()
