#!/usr/bin/env python3
"""Kernel statistics (name, calls, total / average microseconds (the top_kernels view), %) from a rocprofv3 SQLite
result (`rocprofv3 --kernel-trace --stats` without --output-format csv) as CSV."""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage "
                     "from top_kernels").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
        for r in rows:
            w.writerow(r)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
