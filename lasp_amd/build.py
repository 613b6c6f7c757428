"""Build liblaspj.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

Each translation unit is compiled to its own object in parallel (lasp_amd/build/, git-
ignored) and only when it or a header changed; the objects are then linked."""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "build")
OUT = os.path.join(HERE, "liblaspj.so")
SOURCES = ["laspj_runtime.hip", "laspj_kernels.hip", "laspj_combinators.hip",
           "laspj_codec.hip", "laspj_lists.hip", "laspj_comm.hip",
           "laspj_many.hip", "laspj_wide.hip", "laspj_nif.hip", "laspj_host.cpp", "laspj_list_etf.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         "-Wall", "-Wno-unused-value", "-Wno-unused-result"]


def _jobs() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(n, 8, len(SOURCES)))


def build(force: bool = False) -> str:
    headers = [os.path.join(CSRC, "laspj_internal.h"),
               os.path.join(os.path.dirname(HERE), "include", "laspj.h")]
    hdr_t = max(os.path.getmtime(h) for h in headers)
    os.makedirs(OBJ, exist_ok=True)
    objs, todo = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(OBJ, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or \
                os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            todo.append((src, obj))
    if not todo and os.path.exists(OUT) and \
            os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs):
        return OUT

    def compile_one(job):
        src, obj = job
        subprocess.run([HIPCC, *FLAGS, "-c", "-o", obj + ".tmp", src], check=True)
        os.replace(obj + ".tmp", obj)

    with ThreadPoolExecutor(_jobs()) as pool:
        list(pool.map(compile_one, todo))
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp",
                    *objs, "-lamdhip64", "-ldl"], check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
