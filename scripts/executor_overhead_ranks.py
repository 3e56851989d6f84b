#!/usr/bin/env python3
"""Host-side enqueue cost of the device allreduce with REAL peers: BASELINE config 4 (P = 8,
64 Mi fp32 per rank) on 8 RCCL ranks, all on the box's one GPU (per-rank NCCL_HOSTID, RCCL over
loopback sockets; tests/test_gpu_rccl_ranks.py).  Each rank times the library call itself --
hydra_allreduce through XgmiComm.allreduce_, cached plan, the product path -- which returns once
everything is enqueued; the collective then completes over the sockets (slow, untimed) before
the next timed call, so no call waits on a full RCCL queue.  scripts/executor_overhead.py
measured the same on a 1-rank self-loop (peers remapped to self); this confirms it with 7
distinct peers per rank.

    timeout -k 10 300 python scripts/executor_overhead_ranks.py > out.json
"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CASES = (("direct", 16 << 20, "DIRECT, 16 MiB chunk (the library default)"),
         ("direct", 4 << 20, "DIRECT, 4 MiB chunk"),
         ("auto", 0, "AUTO (= A2A: equal reference blocks)"))


def worker(rank, world, port, q):
    os.environ.update({"NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                       "NCCL_HOSTID": f"hydra-probe-rank-{rank}", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    import numpy as np
    import torch
    import torch.distributed as dist

    from hydra_amd import ring

    res = {}
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        comm = ring.XgmiComm(rank, world, 0, ring.exchange_unique_id(rank))
        n = 64 << 20
        t = torch.ones(n, dtype=torch.float32, device=dev)
        for algo, ch, _ in CASES:
            enq = []
            for it in range(6):  # 1 warm-up (plan, scratch, RCCL channels) + 5 timed
                torch.cuda.synchronize()
                dist.barrier()
                a = time.perf_counter()
                comm.allreduce_(t, algo=algo, chunk_bytes=ch)
                b = time.perf_counter()
                comm.wait(120000)
                if it:
                    enq.append(b - a)
            res[f"{algo}/{ch >> 20}"] = float(np.median(enq))
        res["ok"] = bool(torch.isfinite(t[:16]).all())
        comm.close()
    except Exception as e:  # report instead of hanging the parent
        import traceback

        res["error"] = repr(e) + traceback.format_exc()[-800:]
    q.put((rank, res))
    q.close()
    q.join_thread()
    os._exit(0)


def main():
    import torch.multiprocessing as mp

    world = 8
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    rows = []
    for algo, ch, what in CASES:
        k = f"{algo}/{ch >> 20}"
        vals = [res[r][k] * 1e6 for r in range(world) if k in res[r]]
        rows.append({"case": what, "enqueue_us_median_over_ranks": round(sorted(vals)[len(vals) // 2], 1)
                     if vals else None, "enqueue_us_max_over_ranks": round(max(vals), 1) if vals else None})
    errors = {r: v["error"] for r, v in res.items() if "error" in v}
    print(json.dumps({"plan": "config 4: P = 8 real RCCL ranks (one GPU, loopback sockets), "
                              "64 Mi fp32 per rank, hydra_allreduce enqueue (cached plan), "
                              "median of 5 per rank", "rows": rows, "errors": errors}))
    sys.exit(1 if errors else 0)


if __name__ == "__main__":
    main()
