"""Build liblaspj.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""

from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "liblaspj.so")
SOURCES = ["laspj_runtime.hip", "laspj_kernels.hip", "laspj_combinators.hip",
           "laspj_codec.hip", "laspj_lists.hip", "laspj_comm.hip",
           "laspj_many.hip", "laspj_host.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-value", "-Wno-unused-result"]


def build(force: bool = False) -> str:
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, "laspj_internal.h"),
                   os.path.join(os.path.dirname(HERE), "include", "laspj.h")]
    if not force and os.path.exists(OUT) and \
            os.path.getmtime(OUT) >= max(os.path.getmtime(d) for d in deps):
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", *srcs, "-lamdhip64", "-ldl"]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
