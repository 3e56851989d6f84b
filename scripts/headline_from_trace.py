#!/usr/bin/env python3
"""The headline's HBM-resident launches, read back from a rocprofv3 --kernel-trace CSV of
`bench.py --steps S --warmup W --no-cpu-baseline` (what `scripts/gpu_session.sh TAG prof` profiles).

bench.py's N = 1 run launches the 64 Mi fp32 chunk-sum (k_reduce<float ...>, 65 536 workgroups)
in this order: W warmup, S headline (rotating over 4 buffer pairs), min(100, S) bracketed one by
one, 20 cold (each after a 1 GiB fill), then 2 + 20 on ONE pair (the MALL-assisted leg).  So the
headline is dispatches [W, W + S) of that kernel.  Prints per-dispatch durations and the
roofline fraction they imply (12 B/element against the 8 TB/s spec).

Usage: python scripts/headline_from_trace.py <run_kernel_trace.csv> W S [tag]"""
import csv
import json
import statistics
import sys

N = 1 << 26
PEAK = 8000.0


def main(path, warmup, steps, tag):
    durs = []
    for r in csv.DictReader(open(path)):
        # Grid_Size_X counts work-items: one per 16-B vector (4 fp32), 256 per workgroup
        if "k_reduce<float" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == N // 4:
            durs.append((int(r["Start_Timestamp"]),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    durs.sort()
    head = [d for _, d in durs[warmup:warmup + steps]]
    mean, med = statistics.fmean(head), statistics.median(head)
    gbs = lambda us: 12.0 * N / (us * 1e-6) / 1e9  # noqa: E731
    out = {"tag": tag, "source": "rocprofv3 --kernel-trace of bench.py --steps %d --warmup %d" % (
               steps, warmup),
           "dispatches_of_kernel": len(durs), "headline_dispatches": len(head),
           "mean_us": round(mean, 3), "median_us": round(med, 3),
           "achieved_GBps_mean": round(gbs(mean), 1), "frac_mean": round(gbs(mean) / PEAK, 4),
           "achieved_GBps_median": round(gbs(med), 1), "frac_median": round(gbs(med) / PEAK, 4),
           "target_frac": 0.85, "per_dispatch_us": [round(d, 3) for d in head]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] if len(sys.argv) > 4 else "")
