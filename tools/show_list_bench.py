#!/usr/bin/env python3
"""Print the last line of a tools/list_bench.py log compactly (the us_* timings)."""
import json
import sys

with open(sys.argv[1]) as f:
    lines = [ln for ln in f if ln.startswith("{")]
d = json.loads(lines[-1])
for k, v in d.items():
    if isinstance(v, dict):
        v = {x: round(y, 1) for x, y in v.items() if x.startswith("us_")}
    print(k, v)
