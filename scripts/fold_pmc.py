#!/usr/bin/env python3
"""Drive the default P-way fold kernel (DIRECT/A2A owner step) at the BASELINE owner-block
sizes, for rocprofv3 kernel-trace and PMC passes (`scripts/gpu_session.sh TAG pyprof:fold_pmc`):
  config 4: P = 8, owner block of a 64 Mi fp32 bucket = 8 Mi fp32 -> 9 x 4 B per element;
  config 5: P = 8, owner block of a 256 Mi bf16 bucket = 32 Mi bf16, fp32 accumulation ->
            9 x 2 B per element.
Launch k folds source set k mod 3, so no launch finds its operands in the Infinity Cache."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydra_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev)
reps = int(os.environ.get("REPS", "20"))
ROT = 3  # source sets used in turn: HBM-resident launches, as the bench headline
for (P, n, code, flags) in [(8, 8 << 20, _lib.FLOAT32, 0), (8, 32 << 20, _lib.BFLOAT16, 1)]:
    es = _lib.ESIZE[code]
    sets = [[torch.randint(0, 1 << 14, (n * es // 2,), dtype=torch.int16, device=dev)
             for _ in range(P)] for _ in range(ROT)]
    ptrs = [(ctypes.c_void_p * P)(*[t.data_ptr() for t in srcs]) for srcs in sets]
    for k in range(reps):
        _lib.check(L.hydra_fold(0, code, flags, sets[k % ROT][0].data_ptr(), ptrs[k % ROT], P, n,
                                s.cuda_stream))
    torch.cuda.synchronize()
    del sets
print("fold_pmc done")
