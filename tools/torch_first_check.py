"""Run the engine GPU tests with torch (and its bundled HIP runtime) loaded first, as
the multi-process bench does, and report which libamdhip64 the process mapped."""
import sys

import torch

torch.zeros(1, device="cuda")
import pytest  # noqa: E402

rc = pytest.main(["tests/test_gpu_engine.py", "-m", "gpu", "-q", "-x", "-p", "no:cacheprovider"])
maps = open("/proc/self/maps").read()
libs = sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "laspj" in l})
print("mapped:", libs)
sys.exit(rc)
