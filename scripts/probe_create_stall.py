#!/usr/bin/env python3
"""Which creation step of a host context stalls while another thread keeps the resident reducer
busy (scripts/soak_resident.py saw context creation take up to 224 ms, destruction <= 1 ms)?
Times each HIP-object creation hydra_ctx_create makes -- stream, event, 12 MiB pinned block,
and a device block for comparison -- fresh (after hydra_cache_trim), with and without a thread
calling hydra_reduce_host in a loop.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

from hydra_amd import _lib, synth  # noqa: E402
from hydra_amd.reduce import HostContext  # noqa: E402

L = _lib.lib()


def steps(reps):
    out = {}

    def t(name, f):
        t0 = time.perf_counter()
        f()
        out.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)

    for _ in range(reps):
        _lib.check(L.hydra_cache_trim())
        s, e, p, d = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        t("stream_create", lambda: _lib.check(L.hydra_stream_create(0, ctypes.byref(s))))
        t("event_create", lambda: _lib.check(L.hydra_event_create_on(0, ctypes.byref(e))))
        t("malloc_host_12MiB", lambda: _lib.check(L.hydra_malloc_host(12 << 20, ctypes.byref(p))))
        t("malloc_dev_12MiB", lambda: _lib.check(L.hydra_malloc(0, 12 << 20, ctypes.byref(d))))
        t("ctx_create", lambda: out.setdefault("_c", []).append(HostContext(0)))
        for c in out.pop("_c"):
            c.close()
        _lib.check(L.hydra_stream_destroy(s))
        _lib.check(L.hydra_event_destroy(e))
        _lib.check(L.hydra_free_host(p))
        _lib.check(L.hydra_free(d))
        time.sleep(0.01)
    return {k: {"median": round(float(np.median(v)), 3), "max": round(max(v), 3)}
            for k, v in out.items()}


def main():
    res = {"idle": steps(10)}
    stop = threading.Event()

    def loop():
        c = HostContext(0)
        a, b = synth.stress_f32(2, 0, 40000), synth.stress_f32(2, 1, 40000)
        while not stop.is_set():
            _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                           b.ctypes.data, 40000))
        c.close()

    th = threading.Thread(target=loop)
    th.start()
    time.sleep(0.1)
    try:
        res["busy"] = steps(10)
    finally:
        stop.set()
        th.join()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
