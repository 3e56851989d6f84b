"""One rank of the peer-access allreduce test (tests/test_gpu_peer.py).

Launched by the test as a child process per rank, all ranks on cuda:0 of the one-GPU box (IPC
between processes on one device exercises the same handles, barriers and fences as xGMI peers).
Rendezvous over gloo on 127.0.0.1 (handle exchange only).  Runs the case list in order, writes
every rank's result bytes to <out>/rank<r>.npz; the parent compares them with the oracle.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def inputs(case, P, r):
    from hydra_amd import synth

    n, kind = case["n"], case["data"]
    if kind == "stress_f32":
        return synth.stress_f32(P, r, n)
    if kind == "int32":
        return synth.int32_bucket(P, r, n)
    if kind == "f16":
        rng = np.random.default_rng(1000 + r)
        v = rng.uniform(-4, 4, n).astype(np.float16)
        return v.view(np.uint16).copy()
    if kind == "bf16":
        return synth.bf16_bits(synth.uniform_f32(n, 100 + r) * 4)
    if kind == "typed":  # every other Gloo element type: full-range integers (the sums wrap),
        # fp64 at stress_f32's rank-dependent scales (fold-order-sensitive)
        rng = np.random.default_rng(7000 + 31 * r)
        dt = np.dtype(case["np"])
        if dt.kind in "iu":
            info = np.iinfo(dt)
            return rng.integers(info.min, info.max, n, dtype=dt, endpoint=True)
        return rng.uniform(-1, 1, n) * 2.0 ** ((3 * r) % 17)
    if kind == "bf16_native":  # bf16 arithmetic (each hop rounds to bf16; no ACC_F32)
        return synth.bf16_bits(synth.uniform_f32(n, 300 + r) * 8)
    if kind == "bf16_cancel":  # config 5's fold-order stress (the bf16 result shows the order)
        return synth.bf16_bits(synth.stress_cancel_at(P, r, np.arange(n, dtype=np.int64)))
    raise ValueError(kind)


def stress(peer, arena, c, rank, world, dev):
    """`iters` allreduces of integer-valued fp32 buckets that change every iteration (a stale
    read of the previous call's data cannot go unnoticed), each rank delayed by a random spin
    before every call (uneven arrival), every word of every result checked exactly.  Returns
    the number of wrong words (sums of small integers are exact in any order)."""
    import torch

    n, off = c["n"], c.get("offset_bytes", 0)
    view = arena[off:off + 4 * n].view(torch.float32)
    base = torch.arange(n, device=dev, dtype=torch.int64) % 1000
    g = np.random.default_rng(99 + rank)
    bad = 0
    spin = getattr(torch.cuda, "_sleep", None)
    for it in range(c["iters"]):
        view.copy_((base * (rank + 1) + it * (rank + 2)).to(torch.float32))
        if spin is not None:
            spin(int(g.integers(0, 200000)))
        peer.allreduce_(view, algo=c["algo"], dtype_code=c["dtype"])
        exp = base * (world * (world + 1) // 2) + it * (world * (world + 3) // 2)
        bad += int((view != exp.to(torch.float32)).sum().item())
    return bad


def alternating_streams(peer, arena, c, rank, world, dev):
    """`iters` allreduces issued alternately on two streams with no ordering between them, on
    two buckets at different offsets of the arena: the group's calls must still run one after
    another on the device (they share barrier epochs and scratch).  Small integer inputs, so
    every result is exact in fp32; every word checked.  Returns the number of wrong words."""
    import torch

    n = c["n"]
    views = [arena[0:4 * n].view(torch.float32), arena[8 * n:12 * n].view(torch.float32)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    base = torch.arange(n, device=dev, dtype=torch.int64) % 100
    for k, v in enumerate(views):
        v.copy_((base * (rank + 1) + k).to(torch.float32))
    torch.cuda.synchronize(dev)
    for it in range(c["iters"]):
        k = it % 2
        peer.allreduce_(views[k], algo=c["algo"], dtype_code=c["dtype"],
                        stream=streams[k].cuda_stream)
    torch.cuda.synchronize(dev)
    bad = 0
    for k, v in enumerate(views):
        calls = (c["iters"] + 1 - k) // 2
        # the first call sums the ranks' inputs; each later one sums `world` equal copies
        first = base * (world * (world + 1) // 2) + k * world
        exp = first.to(torch.float64) * float(world) ** (calls - 1)
        bad += int((v.to(torch.float64) != exp).sum().item())
    return bad


def reregister(peer, c, rank, world, dev):
    """`iters` rounds of: a FRESH allocation (the caching allocator emptied first), register,
    allreduce with inputs that change every round, every word checked, collective unregister,
    free.  Each round's mappings must be of that round's memory (round 1's symptom: a peer's
    mapping of a re-registered bucket read zeros or garbage).  Returns wrong words."""
    import torch

    n = c["n"]
    bad = 0
    base = torch.arange(n, device=dev, dtype=torch.int64) % 1000
    for it in range(c["iters"]):
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        t = ((base * (rank + 1)) + it * (rank + 2)).to(torch.float32)
        peer.register(t)
        peer.allreduce_(t, algo=c["algo"], dtype_code=c["dtype"])
        exp = base * (world * (world + 1) // 2) + it * (world * (world + 3) // 2)
        bad += int((t != exp.to(torch.float32)).sum().item())
        peer.unregister(t)  # collective: every rank closed its mappings before anyone frees
        del t
    return bad


def full_size(peer, arena, c, rank, world, dev):
    """BASELINE configs 4 / 5 at their full size: the bucket is generated on the GPU from the
    index-addressable order-sensitive generators (fp32 synth.stress_at; bf16 synth.stress_cancel_at
    for ACC_F32), allreduced once, and reported as the sha256 of the whole result (fp32) or its
    values at the parent's sample indices (bf16, checked against the reference fold there)."""
    import hashlib

    import torch

    from fold_expect import device_bucket
    from hydra_amd import synth

    n, off = c["n"], c.get("offset_bytes", 0)
    if c["data"] == "full_stress":
        view = arena[off:off + 4 * n].view(torch.float32)
        device_bucket(synth.stress_at, world, rank, n, dev, torch.float32, out=view)
    else:  # full_cancel_bf16
        view = arena[off:off + 2 * n].view(torch.bfloat16)
        device_bucket(synth.stress_cancel_at, world, rank, n, dev, torch.bfloat16, out=view)
    torch.cuda.synchronize(dev)
    peer.allreduce_(view, algo=c["algo"], dtype_code=c["dtype"], flags=c.get("flags", 0))
    torch.cuda.synchronize(dev)
    if c["data"] == "full_stress":
        return hashlib.sha256(view.cpu().numpy().tobytes()).hexdigest(), None
    idx = torch.from_numpy(np.load(c["idx_file"], allow_pickle=False)).to(dev)
    return None, view.view(torch.int16)[idx].cpu().numpy().view(np.uint16).copy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--blocks", type=int, default=64)
    ap.add_argument("--arena-bytes", type=int, default=64 << 20)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    from hydra_amd import _lib
    from hydra_amd.peer import PeerComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with open(a.cases) as f:
        cases = json.load(f)
    peer = PeerComm(a.rank, a.world, 0, timeout_ms=30000, blocks=a.blocks)
    results, status = {}, {}
    try:
        # one large registered arena; buckets are views at a per-case element offset (same on
        # every rank), so sub-allocation offsets and 16-B misalignment are exercised
        arena = torch.zeros(a.arena_bytes, dtype=torch.uint8, device=dev)
        peer.register(arena)
        for c in cases:
            name = c["name"]
            if c.get("skip_rank") == a.rank:  # timeout case: this rank never arrives
                dist.barrier()
                dist.barrier()
                continue
            if c["data"] == "stress":  # varying inputs, uneven arrival, every word checked
                status[name] = stress(peer, arena, c, a.rank, a.world, dev)
                continue
            if c["data"] == "reregister":  # fresh allocations, register/unregister loop
                status[name] = reregister(peer, c, a.rank, a.world, dev)
                continue
            if c["data"] == "streams":  # calls on two unordered streams
                status[name] = alternating_streams(peer, arena, c, a.rank, a.world, dev)
                continue
            if c["data"] == "set_blocks":  # the co-residency rule: refused at once, or accepted
                import time

                t0 = time.perf_counter()
                try:
                    peer.set_option(_lib.PEER_OPT_BLOCKS, c["blocks"])
                    status[name] = "accepted"
                except _lib.HydraError as e:
                    status[name] = f"refused in {time.perf_counter() - t0:.3f} s: {e}"
                peer.set_option(_lib.PEER_OPT_BLOCKS, 0)
                continue
            if c["data"] in ("full_stress", "full_cancel_bf16"):  # configs 4 / 5, full size
                digest, sample = full_size(peer, arena, c, a.rank, a.world, dev)
                status[name] = peer.error()
                if digest is not None:
                    status[name + "#sha256"] = digest
                if sample is not None:
                    results[name] = sample
                continue
            if c.get("timeout_ms"):
                peer.set_option(_lib.PEER_OPT_TIMEOUT_MS, c["timeout_ms"])
            x = inputs(c, a.world, a.rank)
            nbytes = x.nbytes
            off = c.get("offset_bytes", 0)
            view = arena[off:off + nbytes]
            own = None
            if c.get("rank_shift"):  # a bucket of its own, at a rank-dependent address mod 16
                own = torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev)
                view = own[a.rank * c["rank_shift"]:a.rank * c["rank_shift"] + nbytes]
                peer.register(view)
            view.copy_(torch.from_numpy(x.view(np.uint8)))
            code = c["dtype"]
            kw = dict(algo=c["algo"], op=c.get("op", "sum"), dtype_code=code,
                      flags=c.get("flags", 0), max_segment=c.get("ms", 0))
            for _ in range(c.get("repeat", 1)):
                view.copy_(torch.from_numpy(x.view(np.uint8)))
                peer.allreduce_(view, **kw)
            if c.get("graph"):  # capture once, replay: the kernel arguments never change
                xin = torch.from_numpy(x.view(np.uint8)).to(dev)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    peer.allreduce_(view, **kw)
                for _ in range(3):
                    view.copy_(xin)
                    g.replay()
                # and eager calls still line up with the replays' barriers afterwards
                view.copy_(xin)
                peer.allreduce_(view, **kw)
            torch.cuda.synchronize(dev)
            if c.get("skip_rank") is not None:
                status[name] = peer.error()
                try:
                    peer.allreduce_(view, algo=c["algo"], dtype_code=code)
                    status[name + "/next"] = "accepted"
                except _lib.HydraError as e:
                    status[name + "/next"] = str(e)
                dist.barrier()
                dist.barrier()
                continue
            results[name] = view.cpu().numpy().copy()
            status[name] = peer.error()
            if own is not None:
                peer.unregister(view)
                del view, own
        dist.barrier()
    finally:
        peer.close()
    np.savez(os.path.join(a.out, f"rank{a.rank}.npz"), **results)
    with open(os.path.join(a.out, f"status{a.rank}.json"), "w") as f:
        json.dump(status, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
