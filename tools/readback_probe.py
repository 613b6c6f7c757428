#!/usr/bin/env python3
"""Cost of the small device->host readbacks the entry points make (a status word, a
size): hipMemcpyAsync of 4 / 64 / 4096 bytes into pageable vs pinned (hipHostMalloc)
host memory, then hipStreamSynchronize; microseconds per round trip."""
import ctypes as C
import json
import time

hip = C.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
stream = C.c_void_p()
hip.hipStreamCreate(C.byref(stream))
dev = C.c_void_p()
hip.hipMalloc(C.byref(dev), C.c_size_t(1 << 16))
pin = C.c_void_p()
hip.hipHostMalloc(C.byref(pin), C.c_size_t(1 << 16), 0)
page = (C.c_char * (1 << 16))()
D2H = 2
res = {}
for n in (4, 64, 4096):
    for name, dst in (("pageable", C.cast(page, C.c_void_p)), ("pinned", pin)):
        for _ in range(50):
            hip.hipMemcpyAsync(dst, dev, C.c_size_t(n), D2H, stream)
            hip.hipStreamSynchronize(stream)
        t0 = time.perf_counter()
        for _ in range(2000):
            hip.hipMemcpyAsync(dst, dev, C.c_size_t(n), D2H, stream)
            hip.hipStreamSynchronize(stream)
        res[f"{name}_{n}B_us"] = (time.perf_counter() - t0) / 2000 * 1e6
t0 = time.perf_counter()
for _ in range(2000):
    hip.hipStreamSynchronize(stream)
res["sync_idle_us"] = (time.perf_counter() - t0) / 2000 * 1e6
print(json.dumps(res))
