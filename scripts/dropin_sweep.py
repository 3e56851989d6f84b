#!/usr/bin/env python3
"""BASELINE config 1 inside the reference itself: tests/cpp/dropin_gloo runs the reference's own
gloo::allreduce ring (2 thread-ranks, loopback TCP) with gloo::sum<float> and, on identical
inputs, with the hydra gfx950 Func plugged into setReduceFunction, over the benchmark's whole
doubling sweep 4 .. 67 108 864 elements (runner.cc:338-362).  Per size: bit-equality of every
rank's output, and rank 0's per-iteration p50/avg and GiB/s (runner.cc:631-635) for both.
Prints one JSON document (progress on stderr)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "dropin_gloo")
sizes = ([int(x) for x in os.environ["SIZES"].split(",")] if os.environ.get("SIZES")
         else [4 << k for k in range(25)])
rows = []
for n in sizes:
    iters = max(5, min(50, (1 << 27) // n))
    sys.stderr.write(f"[dropin_sweep] n={n} iters={iters}\n")
    sys.stderr.flush()
    row = {"n": n}
    for reg in ("0", "1"):  # the hydra Func alone; and with the bucket registered once
        r = subprocess.run([EXE, "new_ring", "2", str(n), "f32", str(iters)],
                           capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, HYDRA_DROPIN_REGISTER=reg,
                                    HYDRA_DROPIN_TRACE=os.environ.get("TRACE", "0")))
        if r.returncode:
            row["error"] = (r.stdout + r.stderr)[-500:]
            break
        j = json.loads(r.stdout.strip().splitlines()[-1])
        if reg == "0":
            row.update({k: j[k] for k in ("mismatched_bytes", "iters", "ref_ms", "hydra_ms")})
            if j.get("hydra_trace"):
                row["hydra_trace"] = j["hydra_trace"]
        else:
            row["mismatched_bytes_registered"] = j["mismatched_bytes"]
            row["hydra_registered_ms"] = j["hydra_ms"]
            if j.get("hydra_trace"):
                row["hydra_registered_trace"] = j["hydra_trace"]
    rows.append(row)
    if "error" in row:
        break
print(json.dumps({"harness": "tests/cpp/dropin_gloo new_ring P=2 f32 (reference ring, "
                             "gloo::sum<float> vs hydra Func; hydra_registered: the bucket "
                             "hydra_host_register'ed once, HYDRA_DROPIN_REGISTER=1)",
                  "rows": rows}))
