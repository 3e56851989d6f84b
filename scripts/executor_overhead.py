"""Host-side cost of the RCCL plan executor (hydra_amd/csrc/xgmi_allreduce.cpp run_plan_rccl) on
one GPU: rank 0's DIRECT plan for BASELINE config 4 (P = 8, 64 Mi fp32) at several pipelining
chunks, every peer remapped to rank 0 so a 1-rank communicator runs it (RCCL send/recv to
self).  Reports the plan's op count, the host time to enqueue one allreduce (the call returns
before the GPU finishes) and the wall time with synchronisation.  The device time here is
HBM-bound self copies, not xGMI; the enqueue time is what an 8-GPU run pays on the CPU per
allreduce.  (The test hook re-validates the plan on every call, which the library's cached
allreduce path does not, so the enqueue figures are an upper bound; round 3 marshals the op
array once, outside the timed call -- round 2 timed the Python marshalling too.)

Usage (GPU box): python scripts/executor_overhead.py > out.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import ctypes

    import torch

    from hydra_amd import _lib, ring

    dev = torch.device("cuda", 0)
    P, n = 8, 64 << 20
    comm = ring.XgmiComm(0, 1, 0, ring._rccl_unique_id())
    t = torch.zeros(n, dtype=torch.float32, device=dev)
    L = _lib.lib()
    s = torch.cuda.current_stream(dev).cuda_stream
    rows = []
    try:
        # (algo, chunk): the explicit chunks, the library default (chunk 0 = 16 MiB since
        # round 3) and AUTO (A2A when the reference blocks are equal -- they are here)
        for algo, ch in (("direct", 1 << 20), ("direct", 4 << 20), ("direct", 16 << 20),
                         ("direct", 64 << 20), ("direct", 0), ("auto", 0)):
            ops, scr = ring.plan(algo, P, 0, n, 4, 0, ch)
            arr = (_lib.PlanOp * max(1, len(ops)))()  # marshalled once: the C call is timed
            for i, o in enumerate(ops):
                if o["kind"] in (1, 2):  # SEND, RECV (xgmi_plan.h): every peer is rank 0 here
                    o["peer"] = 0
                for f, _ in _lib.PlanOp._fields_:
                    setattr(arr[i], f, int(o[f]))

            def call():
                _lib.check(L.hydra_comm_run_plan(comm._h, arr, len(ops), 0, _lib.FLOAT32, 0,
                                                 t.data_ptr(), t.numel() * 4, scr, s))

            for _ in range(2):
                call()
            torch.cuda.synchronize()
            k = 10
            enq = []
            t0 = time.perf_counter()
            for _ in range(k):
                a = time.perf_counter()
                call()
                enq.append(time.perf_counter() - a)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / k
            enq.sort()
            rows.append({"algo": algo, "chunk_MiB": (ch >> 20) if ch else "default (16)",
                         "plan_ops": len(ops),
                         "enqueue_us_median": round(enq[k // 2] * 1e6, 1),
                         "enqueue_us_per_op": round(enq[k // 2] * 1e6 / len(ops), 2),
                         "wall_ms_per_allreduce": round(wall * 1e3, 3)})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    finally:
        comm.close()
    print(json.dumps({"plan": "config 4 (P=8, 64 Mi fp32), rank 0, peers remapped to self, "
                              "hydra_comm_run_plan on a marshalled op array (the executor's "
                              "enqueue; the test hook also re-validates the plan each call)",
                      "rows": rows}))


if __name__ == "__main__":
    main()
