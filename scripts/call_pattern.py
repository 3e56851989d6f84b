#!/usr/bin/env python3
"""The reference ring's reduce call pattern on the device: one
gloo::sum<float> per arriving 1 MiB segment, i.e. 262 144 fp32 elements per call
(allreduce.cc:301-305, kMaxSegmentSize allreduce.h:78), c == a == out + recvOffset and
b == tmp + {0, segmentBytes}.  A 64 Mi-element bucket is 256 such segments.  Measured:

  single      one hydra_reduce per segment, back to back on one stream (async enqueue)
  sync        one hydra_reduce per segment + hipStreamSynchronize: the reference's synchronous
              Func contract, what a caller that sends the segment right after sees
  graph       32 single launches captured in a hipGraph, replayed
  batch_K     hydra_reduce_batch with K consecutive segments per call (K = 2 .. 32)

Prints one JSON document: microseconds per segment for each mode."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hydra_amd import _lib  # noqa: E402

L = _lib.lib()
dev = torch.device("cuda", 0)
SEG = 262144
NSEG = 256
reps = int(os.environ.get("REPS", "5"))
out = torch.rand(SEG * NSEG, device=dev)
tmp = torch.rand(2 * SEG, device=dev)
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
po, pt = out.data_ptr(), tmp.data_ptr()


def seg_ptrs(k):
    c = po + 4 * SEG * k
    return c, c, pt + 4 * SEG * (k & 1)


def single(k):
    c, a, b = seg_ptrs(k)
    _lib.check(L.hydra_chunk_sum(6, c, a, b, SEG, sp))


def timed(fn, count):
    """(wall us per segment, device-event us per segment) over `count` segments, median of reps"""
    walls, evs = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(s)
        fn()
        e1.record(s)
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) / count * 1e6)
        evs.append(e0.elapsed_time(e1) / count * 1e3)
    return round(float(np.median(walls)), 3), round(float(np.median(evs)), 3)


res = {"segment_elements": SEG, "segments": NSEG, "bytes_per_segment": 12 * SEG}
for k in range(NSEG):  # warm-up: code objects loaded, buffers touched
    single(k)
torch.cuda.synchronize()


def run_single():
    for k in range(NSEG):
        single(k)


def run_sync():
    for k in range(NSEG):
        single(k)
        s.synchronize()


w, e = timed(run_single, NSEG)
res["single"] = {"wall_us_per_segment": w, "event_us_per_segment": e}
w, e = timed(run_sync, NSEG)
res["sync"] = {"wall_us_per_segment": w, "event_us_per_segment": e}

g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cs = torch.cuda.current_stream(dev).cuda_stream  # the capture stream, not `sp`
    for k in range(32):
        c, a, b = seg_ptrs(k)
        _lib.check(L.hydra_chunk_sum(6, c, a, b, SEG, cs))
torch.cuda.synchronize()


def run_graph():
    for _ in range(NSEG // 32):
        g.replay()


w, e = timed(run_graph, NSEG)
res["graph32"] = {"wall_us_per_segment": w, "event_us_per_segment": e}

for K in (2, 4, 8, 16, 32):
    tables = []
    for b0 in range(0, NSEG, K):
        arr = (_lib.Segment * K)(*[_lib.Segment(*seg_ptrs(k), SEG) for k in range(b0, b0 + K)])
        tables.append(arr)

    def run_batch(tables=tables, K=K):
        for arr in tables:
            _lib.check(L.hydra_reduce_batch(0, 6, ctypes.cast(arr, ctypes.c_void_p), K, sp))

    run_batch()
    w, e = timed(run_batch, NSEG)
    res[f"batch_{K}"] = {"wall_us_per_segment": w, "event_us_per_segment": e,
                         "GBps_event": round(12 * SEG / (e * 1e-6) / 1e9, 1)}

# correctness of the batched form at this pattern: same bits as single calls
ref = out.clone()
x = out.clone()
for k in range(NSEG):
    c = x.data_ptr() + 4 * SEG * k
    _lib.check(L.hydra_chunk_sum(6, c, c, pt + 4 * SEG * (k & 1), SEG, sp))
y = ref.clone()
arr = (_lib.Segment * NSEG)(*[_lib.Segment(y.data_ptr() + 4 * SEG * k, y.data_ptr() + 4 * SEG * k,
                                           pt + 4 * SEG * (k & 1), SEG) for k in range(NSEG)])
_lib.check(L.hydra_reduce_batch(0, 6, ctypes.cast(arr, ctypes.c_void_p), NSEG, sp))
torch.cuda.synchronize()
res["batch_equals_single_calls"] = bool(torch.equal(x, y))
print(json.dumps(res))
