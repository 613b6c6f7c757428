#!/usr/bin/env python3
"""Latency of the drop-in's host paths (not the batched headline):
  * config 1 end to end: lasp_orset:merge/2 of two 10k-element orddicts through the
    mirror (lasp_amd.orset.merge: dictionary + encode, upload, k_or16, download, decode)
    next to the kernel on resident inputs;
  * the same merge on the NIF's native path: payload bytes -> laspj_dict_encode ->
    upload -> k_or16 -> device to_binary -> download;
  * the Store's bind path: 1000 OR-Set variables each bound to a new value, one bind/3
    at a time vs Store.bind_many (one laspj_batch_bind_many launch);
  * a list-value re-bind (an intersection output re-run after an input change)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lasp_amd import core, orset  # noqa: E402
from lasp_amd.terms import Atom  # noqa: E402


def cfg1_terms(n=10_000):
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    return ta, tb


def main():
    out = {}
    a, b = cfg1_terms()
    orset.merge(a, b)
    t0 = time.perf_counter()
    it = 5
    for _ in range(it):
        m = orset.merge(a, b)
    out["config1_mirror_merge_us"] = (time.perf_counter() - t0) / it * 1e6
    assert len(m) == 10_000
    ctx = orset.context()
    A, B, C = ctx.orset_batch(1, 20_000), ctx.orset_batch(1, 20_000), ctx.orset_batch(1, 20_000)
    A.fill_synthetic(2)
    B.fill_synthetic(3)
    C.join(A, B)
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        C.join(A, B)
    ctx.synchronize()
    out["config1_kernel_merge_us"] = (time.perf_counter() - t0) / 200 * 1e6

    # the NIF's native path for the same call: payloads (what term_to_binary/1 hands the
    # NIF; made here untimed) -> native dictionary encode -> upload -> k_or16 -> device
    # to_binary -> download of the merged payload
    from lasp_amd import _lib, etf
    from lasp_amd.engine import ETFDict
    from lasp_amd.hostdict import NativeDict
    pa, pb = etf.term_to_binary(a), etf.term_to_binary(b)
    nd = NativeDict()
    t0 = time.perf_counter()
    nd.add(_lib.KIND_ORSET, [pa, pb])
    out["config1_native_dict_register_us"] = (time.perf_counter() - t0) * 1e6
    E = nd.info()[0]
    d = ETFDict(ctx, E, *nd.export(E))
    NA, NB, NC = ctx.orset_batch(1, E), ctx.orset_batch(1, E), ctx.orset_batch(1, E)
    host = np.zeros((2, 2 * E), np.uint64)

    def native_merge():
        cells, stt = nd.encode(_lib.KIND_ORSET, [pa, pb], E, out=host)
        assert not stt.any()
        NA.upload(cells[0])
        NB.upload(cells[1])
        NC.join(NA, NB)
        return NC.to_binaries(d)[0]
    got = native_merge()
    assert got == etf.term_to_binary(m), "native path disagrees with the mirror"
    t0 = time.perf_counter()
    for _ in range(it):
        native_merge()
    out["config1_native_e2e_merge_us"] = (time.perf_counter() - t0) / it * 1e6
    t0 = time.perf_counter()
    for _ in range(it):
        nd.encode(_lib.KIND_ORSET, [pa, pb], E, out=host)
    out["config1_native_encode_2x10k_us"] = (time.perf_counter() - t0) / it * 1e6
    # where the rest goes: upload, kernel, device to_binary (size pass, write pass), download
    stages = {"upload": 0.0, "join": 0.0, "etf_size_write": 0.0, "download": 0.0}
    for _ in range(it):
        t0 = time.perf_counter()
        NA.upload(host[0])
        NB.upload(host[1])
        t1 = time.perf_counter()
        NC.join(NA, NB)
        ctx.synchronize()
        t2 = time.perf_counter()
        offs, buf, total = NC.etf_encode(d)
        ctx.synchronize()
        t3 = time.perf_counter()
        o = offs.download(np.uint64)
        buf.download(np.uint8, count=total)
        t4 = time.perf_counter()
        for k, v in zip(stages, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            stages[k] += v
    for k, v in stages.items():
        out["config1_native_%s_us" % k] = v / it * 1e6
    out["config1_native_payload_bytes"] = int(total)
    # from_binary/1 of the merged payload on the device (laspj_orset_etf_read), one replica
    pay = ctx.buffer(len(got))
    pay.upload(np.frombuffer(got, np.uint8))
    po = ctx.buffer(16)
    po.upload(np.array([0, len(got)], np.uint64))
    st_ = NA.etf_decode(d, pay, po)
    assert st_[0] == 0 and np.array_equal(NA.download_words(), NC.download_words())
    t0 = time.perf_counter()
    for _ in range(it):
        NA.etf_decode(d, pay, po)
    out["config1_device_from_binary_us"] = (time.perf_counter() - t0) / it * 1e6

    n = 1000
    st = core.Store(capacity=256)
    ids = [st.declare("lasp_orset")[1] for _ in range(n)]
    for k, i in enumerate(ids):
        st.update(i, ("add_by_token", b"x" * 19 + bytes([k % 251]), k % 200), Atom("a"))
    vals = [[(k % 200, [(b"y" * 19 + bytes([k % 251]), False)])] for k in range(n)]
    t0 = time.perf_counter()
    for i, v in zip(ids, vals):
        st.bind(i, v)
    out["store_bind_sequential_us"] = (time.perf_counter() - t0) / n * 1e6
    vals2 = [[(k % 200, [(b"z" * 19 + bytes([k % 251]), False)])] for k in range(n)]
    t0 = time.perf_counter()
    st.bind_many(list(zip(ids, vals2)))
    out["store_bind_many_us_per_bind"] = (time.perf_counter() - t0) / n * 1e6
    out["pool_hits"] = ctx.pool_hits

    s2 = core.Store(capacity=256)
    l, r, x = (s2.declare("lasp_orset")[1] for _ in range(3))
    s2.intersection(l, r, x)
    for e in range(100):
        s2.update(l, ("add_by_token", b"l" + e.to_bytes(19, "big"), e), Atom("a"))
        s2.update(r, ("add_by_token", b"r" + e.to_bytes(19, "big"), e), Atom("a"))
    t0 = time.perf_counter()
    k = 20
    for e in range(k):
        s2.update(l, ("add_by_token", b"m" + e.to_bytes(19, "big"), e), Atom("a"))
    out["list_rebind_update_plus_rerun_ms"] = (time.perf_counter() - t0) / k * 1e3
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
