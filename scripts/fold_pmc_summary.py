#!/usr/bin/env python3
"""Summarise `scripts/gpu_session.sh TAG pyprof:fold_pmc` output into profiles/<tag>_pmc_fold.json: per-launch kernel
time (trace median) and HBM bytes (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, KiB x1024,
MI355X_MICROARCH.md §HBM) of the P-way fold at the BASELINE owner-block sizes, against the
algorithmic (P + 1) x E bytes per element."""
import csv
import json
import os
import statistics
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fold_pmc"  # gpurun_out/<TAG>
tag = sys.argv[2] if len(sys.argv) > 2 else "r02"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {  # kernel template marker -> (label, elements, algorithmic bytes per launch)
    "k_fold<float, 0, false, true, 1>": ("config 4 owner block: P=8, 8 Mi fp32", 8 << 20,
                                          9 * 4 * (8 << 20)),
    "k_fold<hydra::bf16_t, 0, true, true, 0>": ("config 5 owner block: P=8, 32 Mi bf16, fp32 "
                                                "accumulate", 32 << 20, 9 * 2 * (32 << 20)),
}


def rows(p):
    with open(os.path.join(src, p)) as f:
        return list(csv.DictReader(f))


out = {"source": "rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE and "
                 "--pmc WRITE_SIZE passes of scripts/fold_pmc.py (20 launches per case)",
       "cases": []}
kt = rows("fold_pmc_kt/run_kernel_trace.csv")
fetch = rows("fold_pmc_fetch/run_counter_collection.csv")
write = rows("fold_pmc_write/run_counter_collection.csv")
for marker, (label, n, algo) in CASES.items():
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt
         if marker in r["Kernel_Name"]]
    fs = [float(r["Counter_Value"]) for r in fetch if marker in r["Kernel_Name"]]
    ws = [float(r["Counter_Value"]) for r in write if marker in r["Kernel_Name"]]
    us = statistics.median(d)
    hbm = (2 * statistics.median(fs) + statistics.median(ws)) * 1024
    out["cases"].append({
        "case": label, "kernel": marker, "launches": len(d), "us_median": round(us, 2),
        "algorithmic_bytes": algo, "achieved_TBps": round(algo / (us * 1e-6) / 1e12, 3),
        "fraction_of_8TBps": round(algo / (us * 1e-6) / 8e12, 4),
        "fetch_size_kib_median": statistics.median(fs),
        "write_size_kib_median": statistics.median(ws),
        "hbm_bytes": hbm, "traffic_over_algorithmic": round(hbm / algo, 5)})
with open(os.path.join(root, "profiles", f"{tag}_pmc_fold.json"), "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out, indent=1))
