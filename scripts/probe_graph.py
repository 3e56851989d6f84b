#!/usr/bin/env python3
"""Diagnostic: which parts of the RCCL plan executor survive hipGraph capture on one GPU?
Each variant runs in its own child process (a crash in one does not hide the others).

Usage: python scripts/probe_graph.py            (parent: runs every variant, prints rc)
       python scripts/probe_graph.py VARIANT    (child)
"""
import faulthandler
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = ["fork_join_reduce", "rccl_allreduce", "p2p_self", "alltoall", "direct_plan",
            "fork_join_twice", "fold_wait", "reduce_then_rccl"]


def child(v):
    faulthandler.enable()
    import numpy as np
    import torch

    from hydra_amd import ring

    dev = torch.device("cuda", 0)
    n = 1 << 16
    comm = ring.XgmiComm(0, 1, 0, ring._rccl_unique_id())
    t = torch.arange(n, dtype=torch.float32, device=dev)
    B = n * 4
    if v == "fork_join_reduce":
        ops = [dict(kind=4, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1)]
        fn = lambda: comm.run_plan_(ops, t, B)  # noqa: E731
    elif v == "rccl_allreduce":
        fn = lambda: comm.allreduce_(t, algo="rccl")  # noqa: E731
    elif v == "p2p_self":
        ops = [dict(kind=1, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1),
               dict(kind=2, peer=0, buf=1, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1),
               dict(kind=3, peer=0, buf=0, nsrc=0, off=0, bytes=0, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1)]
        fn = lambda: comm.run_plan_(ops, t, B)  # noqa: E731
    elif v == "alltoall":
        ops = [dict(kind=6, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1)]
        fn = lambda: comm.run_plan_(ops, t, B)  # noqa: E731
    elif v == "fork_join_twice":
        ops = [dict(kind=4, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1)]

        def fn():
            comm.run_plan_(ops, t, B)
            comm.run_plan_(ops, t, B)
    elif v == "fold_wait":
        ops = [dict(kind=4, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1),
               dict(kind=5, peer=-1, buf=0, nsrc=2, off=0, bytes=B, src_off=B, slot_stride=B,
                    wait0=0, wait1=-1)]
        fn = lambda: comm.run_plan_(ops, t, 2 * B)  # noqa: E731
    elif v == "reduce_then_rccl":
        ops = [dict(kind=4, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                    wait0=-1, wait1=-1)]

        def fn():
            comm.run_plan_(ops, t, B)
            comm.allreduce_(t, algo="rccl")
    else:
        ops, scr = ring.plan("direct", 4, 0, n, 4, 0, 1 << 14)
        for o in ops:
            if o["kind"] in (1, 2):
                o["peer"] = 0
        fn = lambda: comm.run_plan_(ops, t, scr)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    print(f"{v}: eager ok", flush=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    print(f"{v}: captured", flush=True)
    g.replay()
    torch.cuda.synchronize()
    print(f"{v}: replayed", flush=True)
    del g
    comm.close()
    _ = np


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    for v in VARIANTS:
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), v],
                           capture_output=True, timeout=120)
        out = (r.stdout.decode() + r.stderr.decode()).strip().splitlines()
        tail = [ln for ln in out if ln.startswith(v) or "Error" in ln or "error" in ln][-4:]
        print(f"== {v}: rc={r.returncode}  " + " | ".join(tail), flush=True)


if __name__ == "__main__":
    main()
