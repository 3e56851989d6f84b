#!/usr/bin/env python3
"""Interleaved A/B of the P-way fold kernel variants (DIRECT/A2A owner step) in one process.
Bytes per element of the owner block: (nsrc + 1) x esize (read every contribution, write dst)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydra_amd import _lib  # noqa: E402

L = _lib.measure_lib()  # the A/B variants live in the measurement build
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev)
res = {}
CASES = [(8, 8 << 20, 6, 0), (8, 32 << 20, 9, 1), (4, 16 << 20, 6, 0), (2, 32 << 20, 6, 0)]
if os.environ.get("BASELINE_ONLY"):  # the BASELINE owner blocks: config 4 and config 5
    CASES = CASES[:2]
for (P, n, code, flags) in CASES:
    es = _lib.ESIZE[code]
    # ROTATE=k: k independent source sets used in turn (k x (P+1) x block bytes cycled), so the
    # Infinity Cache holds none of a launch's operands -- the HBM-resident measurement
    rot = int(os.environ.get("ROTATE", "1"))
    sets = [[torch.randint(0, 1 << 14, (n * es // 2,), dtype=torch.int16, device=dev)
             for _ in range(P)] for _ in range(rot)]
    ptrs = [(ctypes.c_void_p * P)(*[t.data_ptr() for t in srcs]) for srcs in sets]
    key = f"P{P}/n{n}/{'bf16acc32' if flags else 'f32'}" + (f"/rot{rot}" if rot > 1 else "")
    for rnd in range(5):
        for v in [int(x) for x in os.environ.get("VARIANTS", "0,1,2,3,4,5,6,7").split(",")]:
            L.hydra_set_variant(v)
            reps = 15 * rot
            for k in range(rot):  # warm-up
                _lib.check(L.hydra_fold(0, code, flags, sets[k][0].data_ptr(), ptrs[k], P, n,
                                        s.cuda_stream))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(reps):  # event span over the region / launches
                _lib.check(L.hydra_fold(0, code, flags, sets[k % rot][0].data_ptr(),
                                        ptrs[k % rot], P, n, s.cuda_stream))
            e1.record(s)
            torch.cuda.synchronize()
            res.setdefault(key, {}).setdefault(v, []).append(e0.elapsed_time(e1) / reps)
    del sets
L.hydra_set_variant(0)
out = {}
for k, d in res.items():
    P = int(k.split("/")[0][1:])
    n = int(k.split("/")[1][1:])  # (keys: P<P>/n<n>/<type>[/rot<k>])
    es = 2 if "bf16" in k else 4
    out[k] = {v: {"us": round(float(np.median(t)) * 1e3, 2),
                  "GBps": round((P + 1) * n * es / (np.median(t) * 1e-3) / 1e9, 1)}
              for v, t in d.items()}
print(json.dumps(out))
