"""The update -> read -> replica bind -> far bind interleaving of bench.py's new-token leg,
then the same far variable's warm re-binds, with per-phase NIF counters (host stages) —
under rocprofv3 --kernel-trace the two phases' kernels can be told apart by order."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lasp_amd import engine, etf  # noqa: E402
from lasp_amd._lib import check  # noqa: E402
from oracle import etf as oetf  # noqa: E402
from oracle import orset as oorset  # noqa: E402
from oracle.terms import Atom  # noqa: E402


def main():
    n = 10_000
    ctx = engine.Context(0)
    L = ctx.L
    ta = [(e, [(b"A" + e.to_bytes(19, "big"), False)]) for e in range(n)]
    tb = [(e, [(b"B" + e.to_bytes(19, "big"), e % 10 == 0)]) for e in range(n)]
    ref = etf.term_to_binary(oorset.merge(ta, tb))
    uv = ctx.var("orset")
    uv.write(ref)
    rep, far = uv.replica(), ctx.var("orset")
    rep.write(ref)
    far.write(ref)
    st, vd = C.c_int32(), C.c_int32()
    res, vd2, nm = C.c_int32(), C.c_int32(), C.c_uint32()
    ei, el, mi = C.c_void_p(), C.c_uint64(), C.c_void_p()
    keys = ("ns_stage_enqueue", "ns_stage_copy", "ns_device_wait", "ns_answers", "ns_register",
            "ns_rebuild", "device_passes")

    def upd(e):
        op = oetf.term_to_binary((Atom("add"), e))
        check(L.laspj_var_etf_update(uv.h, op, len(op), C.byref(res), C.byref(ei), C.byref(el),
                                     C.byref(mi), C.byref(nm), C.byref(vd2)), ctx.h)

    def bind(v, img):
        t = time.perf_counter()
        check(L.laspj_var_etf_bind(v.h, img, len(img), C.byref(st), C.byref(vd)), ctx.h)
        return (time.perf_counter() - t) * 1e6

    out = {}
    tr, tf = [], []
    s0 = ctx.nif_stats()
    for k in range(30):
        upd(97 * k + 1)
        _, img = uv.read()
        tr.append(bind(rep, img))
        tf.append(bind(far, img))
    s1 = ctx.nif_stats()
    out["interleaved"] = {"replica_us": sorted(tr)[15], "far_us": sorted(tf)[15],
                          "per_iter": {x: (s1[x] - s0[x]) / 30 for x in keys}}
    tw = [bind(far, img) for _ in range(30)]
    s2 = ctx.nif_stats()
    out["warm"] = {"far_us": sorted(tw)[15], "per_bind": {x: (s2[x] - s1[x]) / 30 for x in keys}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
