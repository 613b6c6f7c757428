#!/usr/bin/env python3
"""OR-Set from_binary cost split into per-element and per-record parts: the t64 decode
(4096 payloads x 1024 elements, 20-byte tokens, 64 token slots) with exactly k tokens
per element for several k, every element present, half the tokens removed.  Time per
launch vs k gives the per-record slope and the per-element intercept; under rocprofv3
--pmc the per-dispatch SQ counters split the same way (dispatches come in k order,
STEPS + 3 per k)."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import _lib, engine  # noqa: E402
from lasp_amd.codec import Domain  # noqa: E402

R, E, T = 4096, 1024, 64
# k tokens in every element; 0: random masks (~32 of 64, the suite's t64 row)
KS = [int(k) for k in os.environ.get("KS", "4,16,32,48,64").split(",")]
STEPS = int(os.environ.get("STEPS", "10"))
SEGS = [int(x) for x in os.environ.get("SEGS", "0").split(",")]   # LASPJ_TUNE_ETF_SEG values
# LASPJ_TUNE_ETF_READ values to A/B (0: the item decoder at this shape, 8: the wave decoder)
READS = [int(x) for x in os.environ.get("READS", "0").split(",")]

ctx = engine.Context(0)
L = ctx.L
dom = Domain()
for e in range(E):
    es = dom.element_slot(e * 1000)
    for k in range(T):
        dom.token_slot(es, hashlib.blake2b(b"%d:%d" % (e, k), digest_size=20).digest())
d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
for k in KS:
    h = np.zeros((R, E, 2), np.uint64)
    if k == 0:
        rng = np.random.default_rng(7)
        h[:, :, 0] = rng.integers(1, 1 << 63, (R, E), dtype=np.uint64) | np.uint64(1)
        h[:, :, 1] = h[:, :, 0] & rng.integers(0, 1 << 63, (R, E), dtype=np.uint64)
    else:
        p = np.uint64((1 << k) - 1) if k < 64 else ~np.uint64(0)
        h[:, :, 0] = p
        h[:, :, 1] = p & np.uint64(0x5555555555555555)
    b = ctx.orset_batch(R, E)
    b.upload(h)
    offs = ctx.buffer(8 * (R + 1))
    total = _lib.C.c_uint64()
    _lib.check(L.laspj_orset_etf_size(ctx.h, b.h, d.h, 76, offs.h, _lib.C.byref(total)), ctx.h)
    out = ctx.buffer(total.value)
    _lib.check(L.laspj_orset_etf_write(ctx.h, b.h, d.h, 76, 1, offs.h, out.h), ctx.h)
    back = ctx.orset_batch(R, E)
    stb = ctx.buffer(4 * R)

    def run():
        _lib.check(L.laspj_orset_etf_read(ctx.h, back.h, d.h, 76, 1, out.h, offs.h, stb.h),
                   ctx.h)
    for seg, rd in [(s_, r_) for s_ in SEGS for r_ in READS]:
        ctx.set_tuning(_lib.TUNE_ETF_SEG, seg)
        ctx.set_tuning(_lib.TUNE_ETF_READ, rd)
        back.clear()
        for _ in range(3):
            run()
        ctx.synchronize()
        e0, e1 = ctx.event(), ctx.event()
        e0.record()
        for _ in range(STEPS):
            run()
        e1.record()
        ms = e0.elapsed_ms(e1) / STEPS
        ok = bool(np.array_equal(back.download(), h))
        print(json.dumps({"k": k, "seg": seg, "read": rd, "ms": round(ms, 4), "payload_bytes": total.value,
                          "ns_per_element_wave": round(ms * 1e6 / (E), 2), "exact": ok}),
              flush=True)
    ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)
    ctx.set_tuning(_lib.TUNE_ETF_READ, 0)
    del back, stb, out, offs, b
