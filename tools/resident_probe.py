"""bench.py's resident-variable leg (config1_resident) alone, with the NIF counters after it:
for finding a regression in the update / new-token bind legs without the whole bench."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from lasp_amd import engine, etf  # noqa: E402
from oracle import orset as oorset  # noqa: E402


def main():
    n = 10_000
    ctx = engine.Context(0)
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    pa, pb = etf.term_to_binary(ta), etf.term_to_binary(tb)
    ref = etf.term_to_binary(oorset.merge(ta, tb))
    out = bench.config1_resident(ctx, pa, pb, ref)
    keep = {k: v for k, v in out.items() if k.startswith("us_") or k.endswith("stages")
            or k.endswith("samples_us") or k.startswith("bind_")}
    print(json.dumps(keep))
    print(json.dumps(ctx.nif_stats()))


if __name__ == "__main__":
    main()
