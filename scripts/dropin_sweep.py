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
    r = subprocess.run([EXE, "new_ring", "2", str(n), "f32", str(iters)], capture_output=True,
                       text=True, timeout=600)
    if r.returncode:
        rows.append({"n": n, "error": (r.stdout + r.stderr)[-500:]})
        break
    j = json.loads(r.stdout.strip().splitlines()[-1])
    rows.append({k: j[k] for k in ("n", "mismatched_bytes", "iters", "ref_ms", "hydra_ms")})
print(json.dumps({"harness": "tests/cpp/dropin_gloo new_ring P=2 f32 (reference ring, "
                             "gloo::sum<float> vs hydra Func)", "rows": rows}))
