#!/usr/bin/env python3
"""Per-size kernel durations of the chunk-sum from a rocprofv3 --kernel-trace CSV
(e.g. of `bench.py --sweep`): groups k_reduce<float ...> dispatches by grid size
(one 256-thread workgroup per 256 16-B vectors, so elements = 1024 x workgroups).

Usage: python scripts/trace_sizes.py gpurun_out/<dir>/kt/run_kernel_trace.csv
"""
import collections
import csv
import statistics
import sys


def main(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if "k_reduce<float" in r["Kernel_Name"]:
            d[int(r["Grid_Size_X"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("elements  workgroups  launches  median_us  min_us  GB/s(median, 12 B/el)")
    for g in sorted(d):
        v = d[g]
        n = g // 256 * 1024
        med = statistics.median(v)
        print(f"{n:9d}  {g // 256:10d}  {len(v):8d}  {med:9.2f}  {min(v):6.2f}  "
              f"{12 * n / (med * 1e-6) / 1e9:9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
