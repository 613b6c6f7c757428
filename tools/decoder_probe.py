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
KS = [int(k) for k in os.environ.get("KS", "4,16,32,48,64").split(",")]
STEPS = int(os.environ.get("STEPS", "10"))
SEGS = [int(x) for x in os.environ.get("SEGS", "0").split(",")]   # LASPJ_TUNE_ETF_SEG values

ctx = engine.Context(0)
L = ctx.L
dom = Domain()
for e in range(E):
    es = dom.element_slot(e * 1000)
    for k in range(T):
        dom.token_slot(es, hashlib.blake2b(b"%d:%d" % (e, k), digest_size=20).digest())
d = engine.ETFDict(ctx, E, *dom.etf_arrays(E))
for k in KS:
    p = np.uint64((1 << k) - 1) if k < 64 else ~np.uint64(0)
    h = np.zeros((R, E, 2), np.uint64)
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
    for seg in SEGS:
        ctx.set_tuning(_lib.TUNE_ETF_SEG, seg)
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
        print(json.dumps({"k": k, "seg": seg, "ms": round(ms, 4), "payload_bytes": total.value,
                          "ns_per_element_wave": round(ms * 1e6 / (E), 2), "exact": ok}),
              flush=True)
    ctx.set_tuning(_lib.TUNE_ETF_SEG, 0)
    del back, stb, out, offs, b
