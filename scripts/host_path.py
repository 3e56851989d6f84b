#!/usr/bin/env python3
"""Host-resident path measurements: what the reduction costs when the segment
lives in host memory, as it does in the reference's TCP ring.

  1. isolated: hydra_reduce_host on 262 144 / 4 Mi / 16 Mi fp32 elements (ISO_SIZES=...), pageable vs
     hipHostRegister'ed buffers, vs the reference's gloo::sum<float> on the same host core
  2. config 1: new_allreduce_ring, 2 ranks, loopback TCP, the whole 4 .. 64 Mi doubling sweep
     -- the reference itself (oracle/_ref, CPU sum) timed beside the hydra C++ host runtime with
     the GPU reducer (staged and zero-copy), in the same run
  3. config 3: bew_allreduce_a, 2 ranks x 2 loopback rails -- hydra host runtime with the
     reference's gloo::sum<float> as reducer vs the GPU reducer (H2D + sum + D2H per segment)
Configs 1 and 3 run every size REPS times (default 3) with the implementations interleaved, and
report per implementation the median over repetitions of rank 0's p50 / p99 / avg and GiB/s
(and every repetition); the process is pinned to PIN_CORES (default 8) CPUs of the GPU's NUMA
node, never CPU 0 (PIN=0 leaves the affinity alone), as scripts/dropin_sweep.py.
Prints one JSON document.
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# pinned before this process touches HIP (its threads and the host runtime's inherit it); the
# GPU's NUMA node comes from a child process
pinned = None
if os.environ.get("PIN", "1") != "0" and hasattr(os, "sched_setaffinity"):
    import bench  # (no torch import at module level)

    q = subprocess.run([sys.executable, "-c", "import bench; print(bench.gpu_numa_node())"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    try:
        gnode = int(q.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        gnode = None
    cores, node, note = bench.baseline_cores(int(os.environ.get("PIN_CORES", "8")), node=gnode)
    os.sched_setaffinity(0, set(cores))
    pinned = {"cpus": cores, "numa_node": node, "placement": note}
import torch  # noqa: E402,F401

from hydra_amd import _lib, host  # noqa: E402
from hydra_amd.reduce import HostContext  # noqa: E402
from oracle import oracle as O  # noqa: E402  (CPU baseline only)

L = _lib.lib()
out = {"host": {"cpus": os.cpu_count()}, "pinned": pinned}
try:
    out["host"]["model"] = [ln.split(":")[1].strip() for ln in open("/proc/cpuinfo")
                            if ln.startswith("model name")][0]
except Exception:
    pass

# 1. isolated
iso = []
ctx = HostContext(0)
iso_sizes = ([int(x) for x in os.environ["ISO_SIZES"].split(",")] if os.environ.get("ISO_SIZES")
             else [1 << 18, 1 << 22, 1 << 24])
for n in iso_sizes:
    import mmap  # registered memory never returns to the allocator

    a = np.frombuffer(mmap.mmap(-1, 4 * n), np.float32)
    b = np.frombuffer(mmap.mmap(-1, 4 * n), np.float32)
    a[:] = np.arange(n, dtype=np.float32)
    b[:] = 1
    for mode in ("pageable", "registered_staged", "registered_zero_copy",
                 "bucket_registered_b_pageable"):
        # "pageable": copied by the CPU through the context's pinned staging (hydra never pins
        # pageable memory for a call); "registered_staged": registered, but forced through the
        # staging (HYDRA_OPT_FORCE_STAGING); "_zero_copy": the kernel reads and writes the registered host
        # ranges over PCIe directly (hydra_reduce_host's default whenever all three ranges are
        # pinned/registered); "bucket_registered_b_pageable": only c == a registered (a bucket
        # registered once), b pageable like the reference ring's scratch
        ctx.set_option(_lib.OPT_FORCE_STAGING, 1 if mode == "registered_staged" else 0)
        bb = b if mode != "bucket_registered_b_pageable" else np.ones(n, np.float32)
        if mode != "pageable":
            _lib.check(L.hydra_host_register(a.ctypes.data, a.nbytes))
        if mode in ("registered_staged", "registered_zero_copy"):
            _lib.check(L.hydra_host_register(b.ctypes.data, b.nbytes))
        reps = max(3, int(2e8 / (12 * n)))
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       bb.ctypes.data, n))
        t0 = time.perf_counter()
        for _ in range(reps):
            _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                           bb.ctypes.data, n))
        dt = (time.perf_counter() - t0) / reps
        ctx.set_option(_lib.OPT_FORCE_STAGING, 0)
        if mode != "pageable":
            L.hydra_host_unregister(a.ctypes.data)
        if mode in ("registered_staged", "registered_zero_copy"):
            L.hydra_host_unregister(b.ctypes.data)
        iso.append({"elements": n, "mode": mode, "us": round(dt * 1e6, 1),
                    "GBps_12B": round(12 * n / dt / 1e9, 2)})
    cpu = O.ref_time_sum(6, a, a, b, max(3, int(1e8 / (12 * n))), 3) if O.ref_available() else None
    if cpu:
        iso.append({"elements": n, "mode": "reference gloo::sum<float>, 1 core",
                    "us": round(cpu * 1e6, 1), "GBps_12B": round(12 * n / cpu / 1e9, 2)})
ctx.close()
out["isolated"] = iso


def dist(s, n):
    s = np.sort(s)
    return {"elements": n, "min_us": round(s[0] / 1e3, 1),
            "p50_us": round(float(np.percentile(s, 50)) / 1e3, 1),
            "p99_us": round(float(np.percentile(s, 99)) / 1e3, 1),
            "avg_us": round(float(s.mean()) / 1e3, 1),
            "GiBps": round(4 * n * len(s) / (s.sum() * 1e-9) / 2**30, 3)}  # runner.cc:631-635


ref_fn = ctypes.cast(O.ref().ref_sum_f32, ctypes.c_void_p).value if O.ref_available() else None
# BASELINE configs 1 and 3: the benchmark's whole doubling sweep, 4 .. 67 108 864 elements
# (runner.cc:338-362); SIZES=... overrides (comma-separated)
sizes = ([int(x) for x in os.environ["SIZES"].split(",")] if os.environ.get("SIZES")
         else [4 << k for k in range(25)])
if os.environ.get("SKIP_CONFIGS") == "1":  # the isolated measurements only
    sizes = []
c1, c3 = [], []
raw = {}  # impl -> [(elements, samples_ns)], for the reference-format tables (TABLE=path)


def keep(impl, n, samples):
    raw.setdefault(impl, []).append((n, samples))
    return samples


REPS = int(os.environ.get("REPS", "3"))
# (config, implementation, per-iteration ns of rank 0 for (n, iters)); interleaved per size
impls = []
if O.ref_available():
    impls.append(("c1", "reference (gloo, CPU sum)", lambda n, it: O.ref_bench_ring(2, n, 3, it)))
impls += [("c1", "hydra host runtime, GPU sum", lambda n, it: host.bench(1, 2, n, 3, it)),
          ("c1", "hydra host runtime, GPU sum zero-copy (pinned slots, registered out)",
           lambda n, it: host.bench(1, 2, n, 3, it, pinned=True))]
if ref_fn:  # the same runtime with the reference's CPU sum: transport vs reducer
    impls.append(("c1", "hydra host runtime + reference gloo::sum (CPU)",
                  lambda n, it: host.bench(1, 2, n, 3, it, reducer_fn=ref_fn)))
if ref_fn:  # one GPU per rank, approximated: only rank 0's reduces use the box's one GPU
    impls.append(("c1", "hydra host runtime, GPU sum zero-copy on rank 0 only "
                        "(rank 1: reference gloo::sum)",
                  lambda n, it: host.bench(1, 2, n, 3, it, reducer_fn=ref_fn,
                                           gpu_rank0_only=True)))
    impls.append(("c3", "hydra split + reference gloo::sum (CPU)",
                  lambda n, it: host.bench(3, 2, n, 3, it, reducer_fn=ref_fn)))
impls += [("c3", "hydra split, GPU sum (H2D+sum+D2H)", lambda n, it: host.bench(3, 2, n, 3, it)),
          ("c3", "hydra split, GPU sum zero-copy (pinned slots, registered out)",
           lambda n, it: host.bench(3, 2, n, 3, it, pinned=True))]
if ref_fn:
    impls.append(("c3", "hydra split, GPU sum zero-copy on rank 0 only "
                        "(rank 1: reference gloo::sum)",
                  lambda n, it: host.bench(3, 2, n, 3, it, reducer_fn=ref_fn,
                                           gpu_rank0_only=True)))
table_key = {"reference (gloo, CPU sum)": "c1 reference",
             "hydra host runtime, GPU sum": "c1 hydra GPU sum",
             "hydra host runtime, GPU sum zero-copy (pinned slots, registered out)":
                 "c1 hydra GPU sum zero-copy",
             "hydra split + reference gloo::sum (CPU)": "c3 hydra split + reference sum",
             "hydra split, GPU sum (H2D+sum+D2H)": "c3 hydra GPU sum"}

for n in sizes:
    iters = max(5, min(50, (1 << 27) // max(n, 1)))
    sys.stderr.write(f"[host_path] n={n} iters={iters} reps={REPS}\n")
    sys.stderr.flush()
    runs = {(tag, label): [] for tag, label, _ in impls}
    for rep in range(REPS):
        for tag, label, fn in impls:
            samples = fn(n, iters)
            if rep == 0 and label in table_key:
                keep(table_key[label], n, samples)
            runs[(tag, label)].append(dist(samples, n))
    for (tag, label), ds in runs.items():
        med = {k: round(statistics.median(d[k] for d in ds), 3 if k == "GiBps" else 1)
               for k in ("p50_us", "p99_us", "avg_us", "GiBps")}
        (c1 if tag == "c1" else c3).append(
            {"impl": label, "elements": n, "min_us": min(d["min_us"] for d in ds), **med,
             "reps": [{k: d[k] for k in ("p50_us", "avg_us", "GiBps")} for d in ds]})
out["config1_new_allreduce_ring_P2"] = c1
out["config3_bew_allreduce_a_P2"] = c3
out["reps"] = REPS
if os.environ.get("TABLE"):  # the reference benchmark's own table per implementation
    from benchkit import report

    algo = {"c1": "new_allreduce_ring", "c3": "bew_allreduce_a"}
    with open(os.environ["TABLE"], "w") as f:
        for impl, rows in raw.items():
            f.write(f"# {impl}\n" + report.table(algo[impl[:2]], 2, rows) + "\n\n")
print(json.dumps(out))
