#!/usr/bin/env python3
"""probe_graph_ranks.py -- does a multi-rank allreduce captured into a hipGraph replay?

World 2 on the box's one GPU (per-rank NCCL_HOSTID, RCCL over loopback sockets, as
tests/test_gpu_rccl_ranks.py).  For each schedule -- RCCL's own ncclAllReduce first (is capture
of a socket-linked communicator possible at all?), then A2A, DIRECT, RING -- every rank: one
warm-up call, capture, 3 replays on fresh inputs, each checked against the oracle's reference
ring.  Every step is logged with a timestamp to gpurun_out/<tag>/graph_rank<r>.log and flushed,
so a hang names its step; faulthandler dumps the stacks after `HANG_S`.

    timeout -k 10 150 python scripts/probe_graph_ranks.py TAG
"""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HANG_S = 40


def worker(rank, world, port, out):
    os.environ.update({"NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                       "NCCL_HOSTID": f"hydra-probe-rank-{rank}", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    log = open(os.path.join(out, f"graph_rank{rank}.log"), "w", buffering=1)
    faulthandler.enable(file=log)  # a native crash leaves the Python stack here
    faulthandler.dump_traceback_later(HANG_S, repeat=True, file=log)
    t0 = time.time()

    def say(msg):
        log.write(f"{time.time() - t0:8.3f} {msg}\n")

    import numpy as np
    import torch
    import torch.distributed as dist

    from hydra_amd import ring, synth
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = ring.XgmiComm(rank, world, 0, ring.exchange_unique_id(rank))
    say("comm up")
    n = 1 << 20
    for algo in os.environ.get("ALGOS", "rccl,a2a,direct,ring").split(","):
        xs = [[synth.stress_f32(world, r, n, seed=s) for r in range(world)] for s in (5, 6, 7)]
        t = torch.from_numpy(xs[0][rank].copy()).to(dev)
        comm.allreduce_(t, algo=algo)
        comm.wait(30000)
        say(f"{algo}: warm-up done")
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                comm.allreduce_(t, algo=algo)
        except Exception as e:  # capture refused: report and go on
            say(f"{algo}: capture failed: {e!r}")
            continue
        say(f"{algo}: captured")
        for rep in range(3):
            t.copy_(torch.from_numpy(xs[rep][rank]).to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            say(f"{algo}: replay {rep} enqueued")
            torch.cuda.synchronize()
            got = t.cpu().numpy()
            if algo == "rccl":
                st = np.stack(xs[rep]).astype(np.float64)
                ok = bool(np.all(np.abs(got - st.sum(0)) <= 2.0 ** -23 * np.abs(st).sum(0)))
            else:
                ok = bool(np.array_equal(got.view(np.uint32), O.ring_result(xs[rep]).view(np.uint32)))
            say(f"{algo}: replay {rep} done, {'ok' if ok else 'MISMATCH'}")
        del g
    comm.close()
    dist.destroy_process_group()
    say("done")
    faulthandler.cancel_dump_traceback_later()


def main():
    import torch.multiprocessing as mp

    tag = sys.argv[1] if len(sys.argv) > 1 else "graph_ranks"
    out = os.path.join(ROOT, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, 2, port, out)) for r in range(2)]
    for p in procs:
        p.start()
    deadline = time.time() + 120
    for p in procs:
        p.join(timeout=max(1, deadline - time.time()))
    rc = 0
    for p in procs:
        if p.is_alive():
            p.kill()
            rc = 3
        elif p.exitcode:
            rc = rc or 1
    for r in range(2):
        print(open(os.path.join(out, f"graph_rank{r}.log")).read()[-3000:])
    print("exit codes:", [p.exitcode for p in procs])
    sys.exit(rc)


if __name__ == "__main__":
    main()
