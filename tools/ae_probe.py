"""Probe: one-rank laspj_antientropy rounds at growing sizes, each checked against the
synthetic stream (where does a large round stop reproducing the state?)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from lasp_amd.engine import Comm, Context  # noqa: E402

ctx = Context(0)
comm = Comm(ctx, 1, Comm.unique_id(), 0)
E = 4096
for lg in [int(x) for x in sys.argv[1:]] or [14, 16, 18, 19, 20]:
    O = 1 << lg
    st, rv = ctx.orset_batch(O, E), ctx.orset_batch(O, E)
    st.fill_synthetic(10)
    ctx.synchronize()
    t0 = time.perf_counter()
    comm.antientropy(st, rv)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    bad = []
    ref = ctx.orset_batch(1, E)
    for o in sorted({int(x) for x in np.linspace(0, O - 1, 9)}):
        ref.fill_synthetic(10, replica_base=o)
        for name, b in (("state", st),):
            if not np.array_equal(b.download(o, 1), ref.download()):
                bad.append((name, o))
    print(f"O=2^{lg} ({O * E * 16 / 2**30:.0f} GiB): {dt * 1e3:.1f} ms, mismatches {bad[:12]}",
          flush=True)
    del st, rv
