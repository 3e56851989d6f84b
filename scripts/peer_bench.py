#!/usr/bin/env python3
"""Peer-access allreduce on ONE GPU: P processes share cuda:0 and map each other's buckets by
hipIpc, so every "remote" read is a local HBM read.  This measures the kernel and its protocol
(barriers, flag waits, slab mapping) against the HBM roofline -- not xGMI, which needs the
8-GPU node (bench.py --gpus 8 times it there).

HBM bytes per allreduce, all ranks together (they share one HBM):
  two-shot: P x [ P reads + 1 write of n/P (phase 1) + (P-1)/P n read + write (phase 2) ] x E
          = (P + 1 + 2(P-1)) n E
  one-shot: P x [ P reads of n + 1 write of n (scratch) + n read + n write (copy back) ] x E
          = P (P + 3) n E
  push (peer2w): P x [ P reads + P writes of n/P ] x E = 2 P n E

Usage: python scripts/peer_bench.py [--P 2 --n 16777216 --iters 50]   (spawns the ranks)
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(a):
    import numpy as np
    import torch
    import torch.distributed as dist

    from hydra_amd import synth
    from hydra_amd.peer import PeerComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    dist.init_process_group("gloo", rank=a.rank, world_size=a.P)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from hydra_amd import _lib

    _lib.select_measure()  # the peer A/B variants (hydra_set_variant) live in libhydra_measure.so
    # every rank's grid must be resident at once on the one GPU (512 of the kernel's workgroups
    # fit): --blocks 0 = 512 / P per rank
    peer = PeerComm(a.rank, a.P, 0, blocks=a.blocks or max(1, 512 // a.P))
    out = {}
    try:
        for n in a.n:
            x0 = torch.from_numpy(synth.stress_f32(a.P, a.rank, n)).to(dev)
            x = x0.clone()
            peer.register(x)
            for algo in a.algos:
                ref = None
                for var in a.variants:  # hydra_set_variant: 0 = shipped, 2001.. = peer A/B
                    _lib.lib().hydra_set_variant(var)
                    x.copy_(x0)  # one checked call first: every variant must give the same bits
                    peer.allreduce_(x, algo=algo)
                    torch.cuda.synchronize(dev)
                    got = x.cpu().numpy()
                    same = True if ref is None else bool((got.view("u4") == ref.view("u4")).all())
                    ref = got if ref is None else ref
                    for _ in range(a.warmup):
                        peer.allreduce_(x, algo=algo)
                    torch.cuda.synchronize(dev)
                    dist.barrier()
                    s = torch.cuda.current_stream(dev)
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    t0 = time.perf_counter()
                    e0.record(s)
                    for _ in range(a.iters):
                        peer.allreduce_(x, algo=algo)
                    e1.record(s)
                    torch.cuda.synchronize(dev)
                    wall = time.perf_counter() - t0
                    key = f"{algo}/{n}" + (f"/v{var}" if len(a.variants) > 1 else "")
                    out[key] = {"event_ms": e0.elapsed_time(e1) / a.iters,
                                "wall_ms": wall * 1e3 / a.iters, "err": peer.error(),
                                "same_bits_as_first_variant": same}
                    dist.barrier()
                _lib.lib().hydra_set_variant(0)
            peer.unregister(x)
            del x, x0
    finally:
        peer.close()
    dist.barrier()
    print("RESULT " + json.dumps(out), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--n", type=int, nargs="+", default=[1 << 16, 1 << 20, 1 << 24])
    ap.add_argument("--algos", nargs="+", default=["peer2", "peer1"])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--variants", type=int, nargs="+", default=[0])
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    if a.rank >= 0:
        worker(a)
        return
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.P):
        cmd = [sys.executable, "-u", os.path.abspath(__file__), "--rank", str(r), "--port",
               str(port), "--P", str(a.P), "--iters", str(a.iters), "--warmup", str(a.warmup),
               "--blocks", str(a.blocks), "--n", *map(str, a.n), "--algos", *a.algos,
               "--variants", *map(str, a.variants)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    res = []
    for p in procs:
        o, _ = p.communicate(timeout=600)
        o = o.decode(errors="replace")
        if p.returncode != 0:
            print(o[-3000:], file=sys.stderr)
            raise SystemExit(p.returncode)
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("RESULT ")][-1][7:]))
    summary = {"P": a.P, "note": "all ranks on one GPU: remote reads are local HBM reads"}
    for key in res[0]:
        algo, n = key.split("/")[:2]
        n = int(n)
        ms = max(r[key]["wall_ms"] for r in res)
        ev = max(r[key]["event_ms"] for r in res)
        hbm = {"peer2": (a.P + 1 + 2 * (a.P - 1)) * n * 4, "peer2w": 2 * a.P * n * 4}.get(
            algo, a.P * (a.P + 3) * n * 4)
        summary[key] = {"ms": round(ms, 4), "event_ms": round(ev, 4),
                        "hbm_bytes": hbm, "hbm_GBps": round(hbm / (ev * 1e-3) / 1e9, 1),
                        "algbw_GBps": round(n * 4 / (ev * 1e-3) / 1e9, 1),
                        "err": max(r[key]["err"] for r in res),
                        "same_bits": all(r[key]["same_bits_as_first_variant"] for r in res)}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
