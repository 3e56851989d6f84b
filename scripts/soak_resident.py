#!/usr/bin/env python3
"""Soak of the resident reducer (hydra_amd/csrc/resident.{h,hip}, resident_host.cpp): several
threads, one host context each, keep calling hydra_reduce_host with random sizes (solo calls of
<= 4 tiles, published jobs, multi-round staged calls), random operand memory (pageable,
registered from a long-lived pool, pinned blocks), random gaps (none, sub-idle, past the idle
limit so the instance leaves and is relaunched), while one more thread issues the library's
device-wide drains (freeing pinned blocks, trimming the caches, hydra_device_check, context
create / destroy).  Every result is checked bit for bit against the oracle.  Run with a short
idle limit and grace (HYDRA_RESIDENT_IDLE_US / HYDRA_RESIDENT_GRACE_US) to exercise the
relaunch, heartbeat and stop paths many times.

usage: soak_resident.py [seconds] [threads]; prints one JSON line; exit 1 on any mismatch/error."""
import ctypes
import json
import os
import random
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (bind the library to torch's HIP runtime)

from hydra_amd import _lib, synth  # noqa: E402
from hydra_amd.reduce import HostContext  # noqa: E402
from oracle import oracle as O  # noqa: E402

L = _lib.lib()
# the script's HYDRA_RESIDENT_IDLE_US / HYDRA_RESIDENT_GRACE_US -> the library's options
for _k, _e in ((_lib.OPT_RESIDENT_IDLE_US, "HYDRA_RESIDENT_IDLE_US"),
               (_lib.OPT_RESIDENT_GRACE_US, "HYDRA_RESIDENT_GRACE_US")):
    if os.environ.get(_e):
        _lib.set_option(_k, int(os.environ[_e]))
POOL_ELEMS = 3 << 20  # registered pool per worker (lives for the process)


def worker(k, seconds, out, stop):
    rng = random.Random(1000 + k)
    ctx = HostContext(0)
    pool = np.empty(POOL_ELEMS + 2048, np.float32)
    _lib.check(L.hydra_host_register(pool.ctypes.data, pool.nbytes))
    pinned = ctypes.c_void_p()
    _lib.check(L.hydra_malloc_host((POOL_ELEMS + 2048) * 4, ctypes.byref(pinned)))
    pin = np.frombuffer((ctypes.c_char * ((POOL_ELEMS + 2048) * 4)).from_address(pinned.value),
                        np.float32)
    calls, bad = 0, []
    t0 = time.perf_counter()
    try:
        while time.perf_counter() - t0 < seconds and not stop.is_set():
            r = rng.random()
            n = (rng.randint(1, 4096) if r < 0.45 else rng.randint(4097, 300000) if r < 0.9
                 else rng.randint(1 << 20, 3 << 20))
            kind = rng.choice(("pageable", "registered", "pinned"))
            a = synth.stress_f32(2, 0, n, seed=calls + 7 * k)
            b = synth.stress_f32(2, 1, n, seed=calls + 7 * k)
            exp = O.op(a, b, "sum", 6)
            off = rng.randint(0, 1000)
            if kind == "pageable":
                c = a
            else:
                base = pool if kind == "registered" else pin
                c = base[off:off + n]
                c[:] = a
            rc = L.hydra_reduce_host(ctx.handle, 0, 6, c.ctypes.data, c.ctypes.data,
                                     b.ctypes.data, n)
            if rc or not np.array_equal(c.view(np.uint32), exp.view(np.uint32)):
                bad.append({"call": calls, "n": n, "kind": kind, "rc": rc,
                            "err": L.hydra_last_error().decode(errors="replace")})
                break
            calls += 1
            g = rng.random()
            if g < 0.05:
                time.sleep(0.004)  # past the idle limit: the instance leaves
            elif g < 0.2:
                time.sleep(0.0003)
        st = ctx.stats()
    finally:
        _lib.check(L.hydra_host_unregister(pool.ctypes.data))
        del pin
        _lib.check(L.hydra_free_host(pinned))
        ctx.close()
    out[k] = {"calls": calls, "bad": bad, "resident_calls": st["resident_calls"],
              "launches": st["resident_launches"]}


def drainer(out, stop):
    ops, worst, n = {}, {}, 0
    rng = random.Random(7)
    while not stop.is_set():
        what = rng.choice(("free_pinned", "device_check", "ctx", "trim"))
        times = {}
        t0 = time.perf_counter()
        if what == "free_pinned":
            p = ctypes.c_void_p()
            _lib.check(L.hydra_malloc_host(1 << 20, ctypes.byref(p)))
            times["malloc_pinned"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            _lib.check(L.hydra_free_host(p))
            times["free_pinned"] = time.perf_counter() - t0
        elif what == "device_check":
            _lib.check(L.hydra_device_check(0))
            times[what] = time.perf_counter() - t0
        elif what == "ctx":
            c = HostContext(0)
            times["ctx_create"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            c.close()
            times["ctx_destroy"] = time.perf_counter() - t0
        else:
            _lib.check(L.hydra_cache_trim())
            times[what] = time.perf_counter() - t0
        for name, dt in times.items():
            ops[name] = ops.get(name, 0) + 1
            worst[name] = max(worst.get(name, 0.0), dt)
        n += 1
        time.sleep(0.02)
    out["drainer"] = {"ops": ops, "worst_ms": {k: round(v * 1e3, 2) for k, v in worst.items()}}


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    # HYDRA_SOAK_GEN_STRIDE=65536: every instance gets the same 16-bit generation tag (the test
    # switch of include/hydra_hip.h), so only the per-launch zeroing of the device record keeps an
    # old job word from a new instance's workers
    stride = int(os.environ.get("HYDRA_SOAK_GEN_STRIDE", "0"))
    if stride:
        _lib.test_set(_lib.TEST_RESIDENT_GEN_STRIDE, stride)
    out, stop = {}, threading.Event()
    ws = [threading.Thread(target=worker, args=(k, seconds, out, stop)) for k in range(threads)]
    d = threading.Thread(target=drainer, args=(out, stop))
    for t in ws:
        t.start()
    d.start()
    for t in ws:
        t.join()
    stop.set()
    d.join()
    _lib.check(L.hydra_device_check(0))
    bad = [b for k in range(threads) for b in out[k]["bad"]]
    res = {"seconds": seconds, "threads": threads,
           "idle_us": os.environ.get("HYDRA_RESIDENT_IDLE_US", "2000"),
           "grace_us": os.environ.get("HYDRA_RESIDENT_GRACE_US", "10000000"),
           "calls": sum(out[k]["calls"] for k in range(threads)),
           "resident_calls": sum(out[k]["resident_calls"] for k in range(threads)),
           "launches": max(out[k]["launches"] for k in range(threads)),
           "gen_stride": stride or 1,
           "done_regressions": _lib.test_get(_lib.TEST_RESIDENT_REGRESSIONS),
           "errors": bad[:5], "drainer": out.get("drainer")}
    print(json.dumps(res), flush=True)
    return 1 if bad or res["done_regressions"] else 0


if __name__ == "__main__":
    sys.exit(main())
