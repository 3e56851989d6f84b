#!/usr/bin/env python3
"""Per-call cost of the synchronous host-buffer Func (hydra_reduce_host: what the reference ring
calls once per arriving segment, allreduce.cc:301-305) at small and reference-sized segments.

Modes (operands c == a, b, as the ring passes them):
  registered        a and b inside host ranges registered once with hydra_host_register
                    (the bucket a maintainer registers; hydra's registry, no HIP lookups)
  pinned            a and b in hydra_malloc_host blocks (Context::setScratchAllocator(pinnedAlloc))
  caller_pinned     a and b in torch pinned tensors (the caller's own mapping: one HIP lookup)
  pageable          plain numpy buffers: copied by the CPU through the context's pinned staging
                    (hydra never pins pageable memory for a call)
  registered_staged the registered operands with everything forced through staging (1000)
and, for reference, the device-resident launch + synchronise floor (hydra_reduce on device
buffers followed by hydra_stream_synchronize) and one Zen core's gloo::sum<float>.
Median and p10 of individually timed calls.  Prints one JSON document.  Run it with
HYDRA_RESIDENT=0 as well: the same calls as one batched launch each (no resident reducer).
Usage (GPU box): python scripts/host_floor.py > out.json
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from hydra_amd import _lib  # noqa: E402
from hydra_amd.reduce import HostContext  # noqa: E402

L = _lib.lib()
# HYDRA_RESIDENT=0 in this script's environment: the library option HYDRA_OPT_RESIDENT = 0
_lib.set_option(_lib.OPT_RESIDENT, 0 if os.environ.get("HYDRA_RESIDENT") == "0" else 1)
SIZES = [int(x) for x in os.environ.get("FLOOR_SIZES", "64,1024,16384,262144").split(",")]


def timed(call, n):
    k = max(50, min(3000, int(3e8 / (12 * n + 1))))
    for _ in range(20):
        call()
    ts = np.empty(k)
    for i in range(k):
        t0 = time.perf_counter()
        call()
        ts[i] = time.perf_counter() - t0
    return {"us_median": round(float(np.median(ts)) * 1e6, 2),
            "us_p10": round(float(np.percentile(ts, 10)) * 1e6, 2), "calls": k}


def main():
    ctx = HostContext(0)
    rows = []
    big = 16 << 20
    import mmap  # (registered memory that never returns to the allocator)

    ra = np.frombuffer(mmap.mmap(-1, 4 * big), np.float32)
    rb = np.frombuffer(mmap.mmap(-1, 4 * big), np.float32)
    _lib.check(L.hydra_host_register(ra.ctypes.data, ra.nbytes))
    _lib.check(L.hydra_host_register(rb.ctypes.data, rb.nbytes))
    pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(L.hydra_malloc_host(4 * big, ctypes.byref(pa)))
    _lib.check(L.hydra_malloc_host(4 * big, ctypes.byref(pb)))
    ta = torch.empty(big, dtype=torch.float32).pin_memory()
    tb = torch.empty(big, dtype=torch.float32).pin_memory()
    dev = torch.device("cuda", 0)
    da = torch.zeros(big, dtype=torch.float32, device=dev)
    db = torch.ones(big, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    try:
        for n in SIZES:
            off = 4096  # inside the registered interior (a whole page past the array start)
            ops = {
                "registered": (ra.ctypes.data + 4 * off, rb.ctypes.data + 4 * off),
                "pinned": (pa.value + 4 * off, pb.value + 4 * off),
                "caller_pinned": (ta.data_ptr() + 4 * off, tb.data_ptr() + 4 * off),
            }
            xa = np.empty(n + 7, np.float32)[3:3 + n]  # odd offsets: ragged edge pages
            xb = np.empty(n + 7, np.float32)[5:5 + n]
            ops["pageable"] = (xa.ctypes.data, xb.ctypes.data)
            ops["registered_staged"] = ops["registered"]
            for mode, (a, b) in ops.items():
                ctx.set_option(_lib.OPT_FORCE_STAGING, 1 if mode == "registered_staged" else 0)
                try:
                    r = timed(lambda: _lib.check(
                        L.hydra_reduce_host(ctx.handle, 0, 6, a, a, b, n)), n)
                finally:
                    ctx.set_option(_lib.OPT_FORCE_STAGING, 0)
                rows.append(dict(elements=n, mode=mode, **r))
                print(json.dumps(rows[-1]), file=sys.stderr, flush=True)

            def dev_call():
                _lib.check(L.hydra_reduce(0, 6, da.data_ptr(), da.data_ptr(), db.data_ptr(), n, s))
                _lib.check(L.hydra_stream_synchronize(s))

            rows.append(dict(elements=n, mode="device launch + synchronize", **timed(dev_call, n)))
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
            try:
                from oracle import oracle as O  # CPU reference only

                if O.ref_available():
                    h = np.ones(n, np.float32)
                    per = O.ref_time_sum(6, h, h, h, max(3, int(1e8 / (12 * n))), 3)
                    rows.append({"elements": n, "mode": "reference gloo::sum<float>, 1 core",
                                 "us_median": round(per * 1e6, 3)})
            except Exception as e:  # noqa: BLE001
                rows.append({"elements": n, "mode": "reference", "error": str(e)})
        ctx_stats = ctx.stats()
    finally:
        L.hydra_host_unregister(ra.ctypes.data)
        L.hydra_host_unregister(rb.ctypes.data)
        L.hydra_free_host(pa)
        L.hydra_free_host(pb)
        ctx.close()
    print(json.dumps({"probe": "scripts/host_floor.py",
                      "resident": os.environ.get("HYDRA_RESIDENT", "1") != "0",
                      "stats": ctx_stats, "rows": rows}))


if __name__ == "__main__":
    main()
