#!/usr/bin/env python3
"""Interleaved A/B of the chunk-sum kernel variants in ONE process (methodology rule 24).
Prints a JSON dict: variant -> median kernel us per (size, mode) over rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydra_amd import _lib  # noqa: E402

L = _lib.measure_lib()  # the A/B variants live in the measurement build
dev = torch.device("cuda", 0)
variants = [int(v) for v in os.environ.get("VARIANTS", ",".join(map(str, range(20)))).split(",")]
sizes = [int(s) for s in os.environ.get("SIZES", str(64 << 20)).split(",")]
rounds = int(os.environ.get("ROUNDS", "5"))
reps = int(os.environ.get("REPS", "20"))
res = {}
s = torch.cuda.current_stream(dev)
for n in sizes:
    a = torch.rand(n, device=dev)
    b = torch.rand(n + 4, device=dev)
    c = torch.empty(n, device=dev)
    flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB: evicts the 256 MiB MALL
    # "rotate": bench.py's HBM-resident headline -- in place on 4 buffer pairs in turn, the
    # event span over `reps` launches / reps (no per-launch events)
    rot = [(torch.rand(n, device=dev), torch.rand(n, device=dev)) for _ in range(4)] \
        if "rotate" in os.environ.get("MODES", "") else []
    for mode in os.environ.get("MODES", "inplace,outofplace").split(","):
        if mode == "rotate":
            for r in range(rounds):
                for v in variants:
                    L.hydra_set_variant(v)
                    for k in range(4):
                        x, y = rot[k]
                        _lib.check(L.hydra_chunk_sum(6, x.data_ptr(), x.data_ptr(), y.data_ptr(),
                                                     n, s.cuda_stream))
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(s)
                    for k in range(reps):
                        x, y = rot[k % 4]
                        _lib.check(L.hydra_chunk_sum(6, x.data_ptr(), x.data_ptr(), y.data_ptr(),
                                                     n, s.cuda_stream))
                    e1.record(s)
                    torch.cuda.synchronize()
                    res.setdefault(f"{n}/{mode}", {}).setdefault(v, []).append(
                        e0.elapsed_time(e1) / reps * 1e3)
            continue
        pc = c.data_ptr() if mode == "outofplace" else a.data_ptr()
        # misalign: in place, b one element past 16-B alignment (the ring's tmp slot 1 at
        # +segmentBytes, allreduce.cc:236, when segmentBytes is not a multiple of 16)
        pb = b.data_ptr() + (4 if mode == "misalign" else 0)
        for r in range(rounds):
            for v in variants:
                L.hydra_set_variant(v)
                for _ in range(3):
                    _lib.check(L.hydra_chunk_sum(6, pc, a.data_ptr(), pb, n, s.cuda_stream))
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(reps)]
                for e0, e1 in ev:
                    if mode == "cold":
                        flush.fill_(1.0)
                    e0.record(s)
                    _lib.check(L.hydra_chunk_sum(6, pc, a.data_ptr(), pb, n, s.cuda_stream))
                    e1.record(s)
                torch.cuda.synchronize()
                t = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev])) * 1e3
                res.setdefault(f"{n}/{mode}", {}).setdefault(v, []).append(t)
    del a, b, c, flush, rot
L.hydra_set_variant(0)
out = {}
for k, d in res.items():
    n = int(k.split("/")[0])
    out[k] = {v: {"us": round(float(np.median(t)), 2), "min_us": round(float(np.min(t)), 2),
                  "GBps": round(12 * n / (np.median(t) * 1e-6) / 1e9, 1)} for v, t in d.items()}
print(json.dumps(out))
