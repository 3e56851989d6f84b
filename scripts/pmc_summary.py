#!/usr/bin/env python3
"""Summarise one `gpu_session.sh TAG prof` session's rocprofv3 output into profiles/.

Usage: python scripts/pmc_summary.py gpurun_out/<tag> <round-tag>
Writes profiles/<round>_kernel_stats.csv (the --kernel-trace --stats summary),
profiles/<round>_pmc.csv (per-dispatch FETCH_SIZE / WRITE_SIZE of the hot kernel) and
profiles/pmc_chunk_sum.json (per-launch HBM bytes, read by bench.py as roofline.traffic).

HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: rocprofv3 reports KiB, and on gfx950 FETCH_SIZE
counts exactly half of a wide coalesced streaming read (MI355X_MICROARCH.md §HBM)."""
import csv
import hashlib
import json
import os
import shutil
import statistics
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.path.join(root, "profiles")
os.makedirs(prof, exist_ok=True)
HOT = "k_reduce<float, 0"
# the kernel sources the profiled run used: gpu_session.sh records their hash on the box (the same
# hash bench.py's kernel_src_hash() computes); fall back to the working tree
rec = os.path.join(src, "kernel_src.sha256")
if os.path.exists(rec):
    src_hash = open(rec).read().split()[0]
else:
    h = hashlib.sha256()
    for f in ("reduce_kernels.hip", "reduce_ops.h", "reduce_kernels.h"):
        h.update(open(os.path.join(root, "hydra_amd", "csrc", f), "rb").read())
    src_hash = h.hexdigest()

shutil.copy(os.path.join(src, "prof_kt", "run_kernel_stats.csv"),
            os.path.join(prof, f"{tag}_kernel_stats.csv"))
stats = list(csv.DictReader(open(os.path.join(src, "prof_kt", "run_kernel_stats.csv"))))
hot = [r for r in stats if HOT in r["Name"]]
avg_ns = float(hot[0]["AverageNs"]) if hot else None


def per_dispatch(path, name):
    rows = [r for r in csv.DictReader(open(path)) if HOT in r["Kernel_Name"]
            and r["Counter_Name"] == name]
    return [float(r["Counter_Value"]) for r in rows], rows


fetch, frows = per_dispatch(os.path.join(src, "prof_fetch", "run_counter_collection.csv"),
                            "FETCH_SIZE")
write, wrows = per_dispatch(os.path.join(src, "prof_write", "run_counter_collection.csv"),
                            "WRITE_SIZE")
with open(os.path.join(prof, f"{tag}_pmc.csv"), "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["dispatch", "kernel", "grid", "FETCH_SIZE_KiB", "WRITE_SIZE_KiB"])
    for i, (fr, wr) in enumerate(zip(frows, wrows)):
        w.writerow([i, fr["Kernel_Name"][:80], fr["Grid_Size"], fr["Counter_Value"],
                    wr["Counter_Value"]])
fm, wm = statistics.median(fetch), statistics.median(write)
hbm = (2 * fm + wm) * 1024
out = {"kernel": hot[0]["Name"] if hot else None, "round": tag,
       "elements": 64 << 20, "algorithmic_bytes_per_launch": 12 * (64 << 20),
       "fetch_size_kib_median": fm, "write_size_kib_median": wm,
       "hbm_bytes_per_launch": hbm, "traffic_over_algorithmic": hbm / (12 * (64 << 20)),
       "kernel_trace_avg_ns": avg_ns, "dispatches": len(fetch),
       "correction": "FETCH_SIZE x2 (gfx950 wide-stream read counting), KiB x1024",
       "mode": "bench.py N=1 default command: HBM-resident rotation over 4 buffer pairs",
       "kernel_src_sha256": src_hash}
json.dump(out, open(os.path.join(prof, "pmc_chunk_sum.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
