#!/usr/bin/env python3
"""BASELINE configs[0] on the device alone (bench.py's config1_gpu leg): per-call
latencies and the NIF-shaped merge end to end, for a rocprofv3 kernel trace of where the
end-to-end time goes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from lasp_amd import engine  # noqa: E402

ctx = engine.Context(0)
print(json.dumps(bench.config1_gpu(ctx)), flush=True)
