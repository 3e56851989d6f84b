"""The reference benchmark's result table (gloo/gloo/benchmark/runner.cc:563-649, Distribution in
benchmark/timer.h:68-102), so a host-path run of hydra reads like the reference's own output:

       elements   min (us)   p50 (us)   p99 (us)  p995 (us)   max (us)   avg (us)  avg (GB/s)    samples

Same column widths, the same integer microseconds (long / 1000), the same percentile index
(sorted[int(pct * size)]) and the same bandwidth (bytes x samples / summed ns, in GiB/s though
the label says GB/s: runner.cc:631-635).  Pure formatting: no timing happens here."""
from __future__ import annotations

import numpy as np


def header(algorithm: str, processes: int, device: str = "tcp (loopback)", inputs: int = 1,
           threads: int = 1) -> str:
    """runner.cc:563-613 (Runner::printHeader), single transport device, microseconds."""
    lines = [f"{'Device:':<13}{device}", f"{'Algorithm:':<13}{algorithm}",
             f"{'Options:':<13}processes={processes}, inputs={inputs}, threads={threads}", ""]
    cols = ["elements", "min (us)", "p50 (us)", "p99 (us)", "p995 (us)", "max (us)", "avg (us)"]
    lines.append("".join(f"{c:>11}" for c in cols) + f"{'avg (GB/s)':>13}" + f"{'samples':>11}")
    return "\n".join(lines)


def row(elements: int, element_size: int, samples_ns, threads: int = 1) -> str:
    """runner.cc:615-649 (Runner::printDistribution) for one size; samples in nanoseconds."""
    s = np.sort(np.asarray(samples_ns, dtype=np.int64))
    if s.size < 1:
        raise ValueError("No latency samples found")
    size = s.size

    def pct(p: float) -> int:
        return int(s[int(np.float32(p) * np.float32(size))])  # samples_[pct * size]

    total_bytes = elements * element_size * size
    total_nanos = int(s.sum()) // threads
    gib_s = float(np.float32(total_bytes * np.float32(1e9)) / np.float32(total_nanos)
                  / np.float32(1024 * 1024 * 1024)) if total_nanos else float("inf")
    avg = int(s.sum()) // size
    vals = [elements, int(s[0]) // 1000, pct(0.50) // 1000, pct(0.99) // 1000,
            pct(0.995) // 1000, int(s[-1]) // 1000, avg // 1000]
    return "".join(f"{v:>11}" for v in vals) + f"{gib_s:>13.3f}" + f"{size:>11}"


def table(algorithm: str, processes: int, rows, element_size: int = 4, **kw) -> str:
    """header + one row per (elements, samples_ns)."""
    return "\n".join([header(algorithm, processes, **kw)] +
                     [row(n, element_size, s) for n, s in rows])
