#!/usr/bin/env python3
"""G-Set from_binary at the suite's shape (tools/bench_suite.py: 65536 replicas x 1024
integer elements, ~50 % present, SMALL_INTEGER_EXT / INTEGER_EXT images): the wave
decoder's forms (LASPJ_TUNE_ETF_READ 0 = default, 11 = round 4's, 12 = 11 with the
payload's tail taken from the window, 13 = 4 elements per lane, 14 = 512-element chunks),
interleaved, each checked against the batch it was encoded from."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import _lib, engine  # noqa: E402
from lasp_amd.codec import Domain  # noqa: E402

R = int(os.environ.get("GS_R", "65536"))
E = int(os.environ.get("GS_E", "1024"))
STEPS = int(os.environ.get("STEPS", "10"))
KNOBS = [int(k) for k in os.environ.get("KNOBS", "0,11,12,13,14").split(",")]

ctx = engine.Context(0)
L = ctx.L
g = ctx.gset_batch(R, E)
g.fill_synthetic(12)
dom = Domain()
for e in range(E):
    dom.element_slot(e)
d = engine.ETFDict(ctx, E, *dom.etf_arrays(E, tokens=False))
offs = ctx.buffer(8 * (R + 1))
total = _lib.C.c_uint64()
_lib.check(L.laspj_gset_etf_size(ctx.h, g.h, d.h, 82, offs.h, _lib.C.byref(total)), ctx.h)
out = ctx.buffer(total.value)
_lib.check(L.laspj_gset_etf_write(ctx.h, g.h, d.h, 82, 1, offs.h, out.h), ctx.h)
want = g.download()
back = ctx.gset_batch(R, E)
stb = ctx.buffer(4 * R)


def run():
    _lib.check(L.laspj_gset_etf_read(ctx.h, back.h, d.h, 82, 1, out.h, offs.h, stb.h), ctx.h)


for rep in range(2):
    for knob in KNOBS:
        ctx.set_tuning(_lib.TUNE_ETF_READ, knob)
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
        ok = bool(np.array_equal(back.download(), want)) and \
            not stb.download(np.int32, count=R).any()
        print(json.dumps({"knob": knob, "rep": rep, "ms": round(ms, 4),
                          "payload_bytes": total.value,
                          "elements_per_s": round(R * E / (ms / 1e3), 1),
                          "payload_GBps": round(total.value / (ms / 1e3) / 1e9, 1),
                          "exact": ok}), flush=True)
ctx.set_tuning(_lib.TUNE_ETF_READ, 0)
# the writer side: laspj_gset_etf_size + laspj_gset_etf_write of the same batch
if os.environ.get("WRITE", "1") == "1":
    def enc():
        _lib.check(L.laspj_gset_etf_size(ctx.h, g.h, d.h, 82, offs.h, _lib.C.byref(total)), ctx.h)
        _lib.check(L.laspj_gset_etf_write(ctx.h, g.h, d.h, 82, 1, offs.h, out.h), ctx.h)
    for _ in range(3):
        enc()
    ctx.synchronize()
    e0, e1 = ctx.event(), ctx.event()
    e0.record()
    for _ in range(STEPS):
        enc()
    e1.record()
    print(json.dumps({"write_ms": round(e0.elapsed_ms(e1) / STEPS, 4),
                      "payload_bytes": total.value}), flush=True)
