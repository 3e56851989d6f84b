#!/usr/bin/env python3
"""Does the relative placement of the chunk-sum's two read streams matter on this HBM?

The ring hands the sum `c = a = out + offset` and `b = tmp slot` -- two unrelated addresses.
bench.py's rotation allocates every operand separately (512 MiB each, so a and b start at large
power-of-two-aligned addresses and tile i of a and tile i of b may land on the same HBM channel
/ bank at the same moment).  This probe times the default chunk-sum, HBM-resident (4 operand
pairs in turn, the bench's headline rotation), with b placed at a chosen byte distance `delta`
past the end of a inside ONE allocation, for several deltas, interleaved over rounds in one
process.  Prints one JSON dict: delta -> median us / TB/s.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydra_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
n = int(os.environ.get("N", str(64 << 20)))
rounds = int(os.environ.get("ROUNDS", "5"))
reps = int(os.environ.get("REPS", "40"))
# byte gaps between the end of a and the start of b (all multiples of 16 B)
deltas = [int(d) for d in os.environ.get(
    "DELTAS", "0,4096,8192,65536,262144,2097152,2101248,33554432").split(",")]
s = torch.cuda.current_stream(dev)
F32 = 6
res = {}
bytes_a = 4 * n
for d in deltas:
    assert d % 16 == 0
    pools = [torch.empty((2 * bytes_a + d) // 4, dtype=torch.float32, device=dev)
             for _ in range(4)]
    for p in pools:
        p.uniform_()
    pairs = [(p.data_ptr(), p.data_ptr() + bytes_a + d) for p in pools]
    for pa, pb in pairs:  # warm the code path
        _lib.check(L.hydra_chunk_sum(F32, pa, pa, pb, n, s.cuda_stream))
    torch.cuda.synchronize()
    res[d] = {"pools": pools, "pairs": pairs, "t": []}
for r in range(rounds):
    for d in deltas:
        pairs = res[d]["pairs"]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for k in range(reps):
            pa, pb = pairs[k % 4]
            _lib.check(L.hydra_chunk_sum(F32, pa, pa, pb, n, s.cuda_stream))
        e1.record(s)
        torch.cuda.synchronize()
        res[d]["t"].append(e0.elapsed_time(e1) / reps * 1e3)
out = {"n": n, "rounds": rounds, "reps": reps, "rotation": 4,
       "note": "b = a's allocation + 4n + delta bytes; default chunk-sum in place; us per launch"}
for d in deltas:
    t = res[d]["t"]
    out[str(d)] = {"us": round(float(np.median(t)), 2), "min_us": round(float(np.min(t)), 2),
                   "TBps": round(12 * n / (np.median(t) * 1e-6) / 1e12, 3),
                   "a_mod_2MiB": res[d]["pairs"][0][0] % (2 << 20),
                   "b_mod_2MiB": res[d]["pairs"][0][1] % (2 << 20)}
print(json.dumps(out))
