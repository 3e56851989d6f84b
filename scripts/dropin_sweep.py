#!/usr/bin/env python3
"""BASELINE config 1 inside the reference itself: tests/cpp/dropin_gloo runs the reference's own
gloo::allreduce ring (2 thread-ranks, loopback TCP) with gloo::sum<float> and, on identical
inputs, with the hydra gfx950 Func plugged into setReduceFunction, over the benchmark's doubling
sweep 4 .. 67 108 864 elements (runner.cc:338-362).  Per size: bit-equality of every rank's
output, rank 0's per-iteration p50 / avg (runner.cc:631-635) for gloo::sum, for the hydra Func,
and for the hydra Func with the bucket registered once (HYDRA_DROPIN_REGISTER=1).

The loopback ring on a shared host is noisy from process to process, so every size runs REPS
times (default 3) with the two hydra settings interleaved (unregistered, registered,
unregistered, ...), each process timing gloo::sum beside it; the row reports the median over
repetitions of each setting's p50, and every repetition.  TRACE=1 adds the per-call trace of the
hydra Func (hydra_host_trace: zero-copy vs staged bytes per operand, rounds, resident, and the
call's time split into CPU copies in / GPU wait / CPU copies out).
Prints one JSON document (progress on stderr)."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "dropin_gloo")
sizes = ([int(x) for x in os.environ["SIZES"].split(",")] if os.environ.get("SIZES")
         else [4 << k for k in range(25)])
REPS = int(os.environ.get("REPS", "3"))
# (name, HYDRA_DROPIN_REGISTER, extra environment): the hydra Func alone, with the bucket
# registered once (the library's default path choice: results staged while the registration is
# at most HYDRA_OPT_STAGE_RESULT_REG_MAX, 8 MiB), and (STAGE_RESULT_AB=1) the two fixed choices:
# every result written in place over PCIe, every result staged (library options passed to the
# harness as HYDRA_DROPIN_OPT="key=value,...": keys 4 = STAGE_RESULT_MAX, 5 = _REG_MAX)
MODES = [("hydra", "0", {}), ("hydra_registered", "1", {})]
if os.environ.get("STAGE_RESULT_AB") == "1":
    MODES.append(("hydra_registered_zero_copy_result", "1", {"HYDRA_DROPIN_OPT": "5=0"}))
    MODES.append(("hydra_registered_staged_result", "1",
                  {"HYDRA_DROPIN_OPT": f"5=0,4={1 << 30}"}))
# every process of the sweep on the same CPUs: the GPU's NUMA node, never CPU 0 (bench.py's
# placement for the CPU baselines); PIN=0 leaves the affinity alone
sys.path.insert(0, ROOT)
pinned = None
if os.environ.get("PIN", "1") != "0" and hasattr(os, "sched_setaffinity"):
    import bench  # (no torch import at module level)

    # the GPU's NUMA node from a child process: this one never initialises HIP (it only starts
    # the harness processes)
    q = subprocess.run([sys.executable, "-c", "import bench; print(bench.gpu_numa_node())"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    try:
        gnode = int(q.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        gnode = None
    cores, node, note = bench.baseline_cores(int(os.environ.get("PIN_CORES", "8")), node=gnode)
    os.sched_setaffinity(0, set(cores))
    pinned = {"cpus": cores, "numa_node": node, "placement": note}
rows = []
for n in sizes:
    iters = max(5, min(50, (1 << 27) // n))
    sys.stderr.write(f"[dropin_sweep] n={n} iters={iters} reps={REPS}\n")
    sys.stderr.flush()
    row = {"n": n, "iters": iters, "reps": []}
    for rep in range(REPS):
        for mode, reg, env in MODES:
            r = subprocess.run([EXE, "new_ring", "2", str(n), "f32", str(iters)],
                               capture_output=True, text=True, timeout=600,
                               env=dict(os.environ, HYDRA_DROPIN_REGISTER=reg,
                                        HYDRA_DROPIN_TRACE=os.environ.get("TRACE", "0"), **env))
            if r.returncode:
                row["error"] = (r.stdout + r.stderr)[-500:]
                break
            j = json.loads(r.stdout.strip().splitlines()[-1])
            row["reps"].append({"mode": mode, "mismatched_bytes": j["mismatched_bytes"],
                                "ref_ms": j["ref_ms"], "hydra_ms": j["hydra_ms"],
                                "hydra_trace": j.get("hydra_trace")})
        if "error" in row:
            break
    if "error" not in row:
        row["p50_median_ms"] = {"gloo_sum": statistics.median(x["ref_ms"]["p50"]
                                                              for x in row["reps"])}
        row["mismatched_bytes"] = sum(x["mismatched_bytes"] for x in row["reps"])
        for mode, _, _ in MODES:
            mine = [x for x in row["reps"] if x["mode"] == mode]
            row["p50_median_ms"][mode] = statistics.median(x["hydra_ms"]["p50"] for x in mine)
            tr = [x["hydra_trace"] for x in mine if x["hydra_trace"]]
            if tr:
                row[f"{mode}_call_us_p50_median"] = statistics.median(t["total_us_p50"]
                                                                      for t in tr)
    rows.append(row)
    if "error" in row:
        break
# gloo::sum<float> per call at the Func's call sizes (the reference's own, oracle/_ref), on one
# of the same CPUs, in place on warm buffers as the ring calls it: the per-call crossover
per_call = {}
try:
    import numpy as np

    from oracle import oracle as O

    if O.ref_available():
        os.sched_setaffinity(0, {pinned["cpus"][0]} if pinned else os.sched_getaffinity(0))
        for m in sorted({int(x["hydra_trace"]["elements_avg"]) for r in rows
                         for x in r.get("reps", []) if x.get("hydra_trace")}):
            a = np.arange(m, dtype=np.float32)
            b = np.ones(m, dtype=np.float32)
            per = O.ref_time_sum(6, a, a, b, max(20, (1 << 26) // max(m, 1)), 5)
            per_call[m] = round(per * 1e6, 2)
except Exception as e:  # context only
    per_call = {"error": str(e)}
print(json.dumps({"pinned": pinned, "gloo_sum_call_us_by_elements": per_call,
                  "harness": "tests/cpp/dropin_gloo new_ring P=2 f32 (reference ring, "
                             "gloo::sum<float> vs hydra Func; hydra_registered: the bucket "
                             "hydra_host_register'ed once, HYDRA_DROPIN_REGISTER=1); REPS "
                             "interleaved processes per size, medians of the per-process p50",
                  "reps": REPS, "rows": rows}))
