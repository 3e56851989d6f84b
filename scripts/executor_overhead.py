"""Host-side cost of the RCCL plan executor (hydra_amd/csrc/xgmi_allreduce.cpp run_plan_rccl) on
one GPU: rank 0's DIRECT plan for BASELINE config 4 (P = 8, 64 Mi fp32) at several pipelining
chunks, every peer remapped to rank 0 so a 1-rank communicator runs it (RCCL send/recv to
self).  Reports the plan's op count, the host time to enqueue one allreduce (the call returns
before the GPU finishes) and the wall time with synchronisation.  The device time here is
HBM-bound self copies, not xGMI; the enqueue time is what an 8-GPU run pays on the CPU per
allreduce.  (The test hook re-validates the plan on every call, which the library's cached
allreduce path does not, so the enqueue figures are an upper bound.)

Usage (GPU box): python scripts/executor_overhead.py > out.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from hydra_amd import ring

    dev = torch.device("cuda", 0)
    P, n = 8, 64 << 20
    comm = ring.XgmiComm(0, 1, 0, ring._rccl_unique_id())
    t = torch.zeros(n, dtype=torch.float32, device=dev)
    rows = []
    try:
        for ch_mib in (1, 4, 16, 64):
            ops, scr = ring.plan("direct", P, 0, n, 4, 0, ch_mib << 20)
            for o in ops:
                if o["kind"] in (1, 2):  # SEND, RECV (xgmi_plan.h)
                    o["peer"] = 0
            for _ in range(2):
                comm.run_plan_(ops, t, scr)
            torch.cuda.synchronize()
            k = 10
            enq = []
            t0 = time.perf_counter()
            for _ in range(k):
                a = time.perf_counter()
                comm.run_plan_(ops, t, scr)
                enq.append(time.perf_counter() - a)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k
            enq.sort()
            rows.append({"chunk_MiB": ch_mib, "plan_ops": len(ops),
                         "enqueue_us_median": round(enq[k // 2] * 1e6, 1),
                         "enqueue_us_per_op": round(enq[k // 2] * 1e6 / len(ops), 2),
                         "wall_ms_per_allreduce": round(wall * 1e3, 3)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    finally:
        comm.close()
    print(json.dumps({"plan": "DIRECT, P=8, 64 Mi fp32, rank 0, peers remapped to self",
                      "rows": rows}))


if __name__ == "__main__":
    main()
