#!/usr/bin/env python3
"""Probe: cost of pinning pageable memory on the fly (hipHostRegister + hipHostUnregister) per
call, against the staged path, for segment sizes of the reference ring.  Prints JSON."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from hydra_amd import _lib  # noqa: E402
from hydra_amd.reduce import HostContext  # noqa: E402

L = _lib.lib()
ctx = HostContext(0)
out = []
for n in (16384, 65536, 262144, 1 << 20, 4 << 20):
    a = np.ones(n, np.float32)
    b = np.ones(n, np.float32)
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(L.hydra_host_register(a.ctypes.data, a.nbytes))
        _lib.check(L.hydra_host_register(b.ctypes.data, b.nbytes))
        L.hydra_host_unregister(a.ctypes.data)
        L.hydra_host_unregister(b.ctypes.data)
    reg = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
    staged = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(L.hydra_host_register(a.ctypes.data, a.nbytes))
        _lib.check(L.hydra_host_register(b.ctypes.data, b.nbytes))
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        L.hydra_host_unregister(a.ctypes.data)
        L.hydra_host_unregister(b.ctypes.data)
    onfly = (time.perf_counter() - t0) / reps
    out.append({"elements": n, "register_unregister_2_buffers_us": round(reg * 1e6, 1),
                "staged_us": round(staged * 1e6, 1), "pin_on_the_fly_zero_copy_us": round(onfly * 1e6, 1)})
ctx.close()
print(json.dumps(out))
