#!/usr/bin/env python3
"""Where one Store.update of the list_bench scenario spends its host time: the same
update (R gains a token -> the intersection re-runs -> its 50k-entry output is re-bound)
with every device entry point timed from the host (each call as the caller sees it)."""
import collections
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import _lib, core  # noqa: E402
from lasp_amd.terms import Atom  # noqa: E402

st = core.Store(capacity=1 << 18)
L = st.ctx.L
acc = collections.defaultdict(lambda: [0, 0.0])


class Timed:
    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if not name.startswith("laspj_"):
            return f

        def call(*a):
            t0 = time.perf_counter()
            r = f(*a)
            acc[name][0] += 1
            acc[name][1] += time.perf_counter() - t0
            return r
        return call


N, D = 100_000, 150_000
l, r, x = (st.declare("lasp_orset")[1] for _ in range(3))
tk = lambda c, e: bytes([c]) + int(e).to_bytes(19, "big")   # noqa: E731
st.bind(l, [(e, [(tk(1, e), False)]) for e in range(N)])
st.bind(r, [(e, [(tk(2, e), False)]) for e in range(D - N, D)])
st.intersection(l, r, x)
st.update(r, ("add_by_token", tk(3, 999), D - N + 1), Atom("a"))       # warm
st.ctx.L = Timed(L)
import lasp_amd.engine as E  # noqa: E402
k = 10
t0 = time.perf_counter()
for i in range(k):
    st.update(r, ("add_by_token", tk(3, i), D - N + 17 * i), Atom("a"))
wall = (time.perf_counter() - t0) / k * 1e3
st.ctx.L = L
# the same join, alone, back to back
v = st.vars[r]
dst = st._new_batch(v.type)
core._or_into(st.ctx, dst, v.val, v.val)
st.ctx.synchronize() if hasattr(st.ctx, "synchronize") else None
t0 = time.perf_counter()
for _ in range(100):
    core._or_into(st.ctx, dst, v.val, v.val)
join_alone_us = (time.perf_counter() - t0) / 100 * 1e6
rows = sorted(((n, c / k, s / k * 1e3) for n, (c, s) in acc.items()), key=lambda x: -x[2])
print(json.dumps({"ms_per_update": wall, "join_alone_host_us": join_alone_us, "entry_points_ms_per_update":
                  {n: [round(c, 1), round(ms, 3)] for n, c, ms in rows}}, indent=1))
