#!/usr/bin/env python3
"""Why does bench.py's cpu_baseline (the reference's gloo::sum<float> over 64 Mi fp32, one pinned
core) read ~45 GB/s on some boxes and ~70 GB/s on others?  On one box, time it with the thread
pinned to a core of each NUMA node and the operands first-touched either by that core (local
pages) or by a core of the other node (remote pages).  Prints one JSON line.  CPU only (the
reference built into oracle/_ref); no GPU call."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402

N = int(os.environ.get("N", str(64 << 20)))
SECONDS = float(os.environ.get("SECONDS", "2"))


def nodes():
    out = []
    for d in sorted(os.listdir("/sys/devices/system/node")):
        if d.startswith("node") and d[4:].isdigit():
            out.append(int(d[4:]))
    return out


def core_of(node):
    """A core of `node` within this process's affinity (bench.py's choice), or None."""
    mine = set(bench._cpulist(bench._read(f"/sys/devices/system/node/node{node}/cpulist")))
    cores, _, _ = bench.baseline_cores(1, node=node)
    return cores[0] if cores and cores[0] in mine else None


def touch(core):
    os.sched_setaffinity(0, {core})
    a = np.arange(N, dtype=np.float32)
    b = np.ones(N, dtype=np.float32)
    return a, b


def timed(core, a, b):
    os.sched_setaffinity(0, {core})
    per = O.ref_time_sum(6, a, a, b, 1, 1)
    iters = max(1, int(SECONDS / max(per, 1e-6) / 3))
    return [round(12.0 * N / O.ref_time_sum(6, a, a, b, iters, 1) / 1e9, 2) for _ in range(3)]


def main():
    if not O.ref_available():
        print(json.dumps({"error": "oracle/_ref not built"}))
        return 1
    aff = os.sched_getaffinity(0)
    ns = nodes()
    cores = {n: core_of(n) for n in ns}
    rows = []
    try:
        for run_on in ns:
            for pages_on in ns:
                if cores[run_on] is None or cores[pages_on] is None:
                    continue
                a, b = touch(cores[pages_on])
                rows.append({"thread_node": run_on, "pages_node": pages_on,
                             "cpu": cores[run_on], "GBps": timed(cores[run_on], a, b)})
                del a, b
    finally:
        os.sched_setaffinity(0, aff)
    print(json.dumps({"elements": N, "affinity": sorted(aff), "nodes": ns,
                      "gpu_numa_node": bench.gpu_numa_node(), "rows": rows}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
