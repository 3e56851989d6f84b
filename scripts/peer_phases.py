#!/usr/bin/env python3
"""Where the peer-access allreduce's time goes: P rank processes share the
one GPU's cuda:0 (the one-GPU proxy of scripts/peer_bench.py: every "remote" read is a local
HBM read), each running the shipped two-shot kernel (--algo peer2: pull, peer2w: push) with its phase
clocks on
(hydra_measure_peer_stamps, libhydra_measure.so): per workgroup b of every rank, s_memrealtime
(100 MHz, one clock for the whole GPU, so ranks compare directly) at

  t0 entry | t1 after barrier 1 | t2 end of the fold | t3 after barrier 2 | t4 end of the copy |
  t5 after barrier 3

Per call, over all ranks: the fold phase's window (earliest t1 to latest t2) carries the fold's
HBM bytes, all ranks together (P x [P reads + 1 write] of n/P elements = (P+1) n E); the copy
phase's window (earliest t3 to latest t4) carries 2 (P-1) n E; the barrier waits are t1-t0,
t3-t2, t5-t4 per workgroup; skew = spread of the ranks' first t0.  The same call's bytes over
the kernel span give the proxy's overall fraction of HBM (peer_bench.py's 0.49 / 0.57).

Usage (parent: touches no GPU; every rank is a child process):
  python scripts/peer_phases.py --P 2 --n 67108864 [--iters 20] [--rocprof DIR]
--rocprof DIR wraps every rank in `rocprofv3 --kernel-trace --stats -d DIR/rank<r> --`, so the
kernel trace's average duration can be set beside the clocks; --pmc COUNTER (with --rocprof DIR)
collects one counter per dispatch instead (FETCH_SIZE or WRITE_SIZE, one pass each: the TCC
counters are device-wide, so each rank's dispatch counts every rank's traffic while their
kernels overlap).  Prints one JSON document.
"""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0
TICK_S = 1e-8  # s_memrealtime: 100 MHz


def worker(a):
    import ctypes

    import numpy as np
    import torch
    import torch.distributed as dist

    from hydra_amd import _lib, synth

    _lib.select_measure()  # the phase clocks exist in libhydra_measure.so only
    from hydra_amd.peer import PeerComm

    if a.variant:  # a measurement variant's kernel (2032: the push with dynamic slabs)
        _lib.lib().hydra_set_variant(a.variant)

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    dist.init_process_group("gloo", rank=a.rank, world_size=a.P)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    grid = a.blocks or max(1, 512 // a.P)  # every rank's grid resident at once on the one GPU
    peer = PeerComm(a.rank, a.P, 0, blocks=grid)
    L = _lib.lib()
    per_call = grid * _lib.PEER_STAMPS
    stamps = torch.zeros(per_call * (a.iters if a.back_to_back else 1), dtype=torch.int64,
                         device=dev)
    out = {"calls": []}
    try:
        x = synth.fill_at(synth.stress_at, a.P, a.rank, a.n, dev, torch.float32)
        peer.register(x)
        for _ in range(a.warmup):
            peer.allreduce_(x, algo=a.algo)
        torch.cuda.synchronize(dev)
        # the event-timed kernel without clocks (the shipped kernel exactly), then with them
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s = torch.cuda.current_stream(dev)
        e0.record(s)
        for _ in range(a.iters):
            peer.allreduce_(x, algo=a.algo)
        e1.record(s)
        torch.cuda.synchronize(dev)
        out["event_ms_plain"] = e0.elapsed_time(e1) / a.iters
        if a.back_to_back:  # steady state: each call its own stamp slice, no host barrier between
            dist.barrier()
            for i in range(a.iters):
                _lib.check(L.hydra_measure_peer_stamps(
                    peer._h, ctypes.c_void_p(stamps.data_ptr() + i * per_call * 8), grid))
                peer.allreduce_(x, algo=a.algo)
            torch.cuda.synchronize(dev)
            v = stamps.view(a.iters, grid, _lib.PEER_STAMPS).cpu().numpy()
            out["calls"] = [v[i].tolist() for i in range(a.iters)]
        else:
            _lib.check(L.hydra_measure_peer_stamps(peer._h, ctypes.c_void_p(stamps.data_ptr()),
                                                   grid))
        for _ in range(0 if a.back_to_back else a.iters):
            dist.barrier()
            peer.allreduce_(x, algo=a.algo)
            torch.cuda.synchronize(dev)
            out["calls"].append(stamps.view(grid, _lib.PEER_STAMPS).cpu().numpy().tolist())
        _lib.check(L.hydra_measure_peer_stamps(peer._h, None, 0))
        out["err"] = peer.error()
        out["grid"] = grid
        peer.unregister(x)
    finally:
        peer.close()
    dist.barrier()
    print("RESULT " + json.dumps(out), flush=True)
    dist.destroy_process_group()


def summarize(P, n, res, algo="peer2"):
    import numpy as np

    E = 4
    grid = res[0]["grid"]
    if algo == "peer2w":  # push: the fold writes every bucket; no copy phase
        fold_bytes = 2 * P * n * E         # all ranks: P reads + P writes of each owner block
        copy_bytes = 0
    else:
        fold_bytes = (P + 1) * n * E       # all ranks: P reads + 1 write of each owner block
        copy_bytes = 2 * (P - 1) * n * E   # all ranks: (P-1)/P n read + written, each
    total_bytes = fold_bytes + copy_bytes  # peer_bench.py's two-shot HBM bytes
    rows = []
    for c in range(len(res[0]["calls"])):
        t = np.array([r["calls"][c] for r in res], dtype=np.int64)  # [rank, wg, 6]
        span = (t[:, :, 5].max() - t[:, :, 0].min()) * TICK_S
        fold_w = (t[:, :, 2].max() - t[:, :, 1].min()) * TICK_S
        copy_w = (t[:, :, 4].max() - t[:, :, 3].min()) * TICK_S
        per_wg = {k: (t[:, :, i + 1] - t[:, :, i]) * TICK_S for i, k in
                  enumerate(("barrier1", "fold", "barrier2", "copy", "barrier3"))}
        rows.append({
            "span_us": span * 1e6,
            "rank_start_skew_us": float((t[:, :, 0].min(axis=1).max() -
                                         t[:, :, 0].min(axis=1).min()) * TICK_S * 1e6),
            "fold_window_us": fold_w * 1e6, "copy_window_us": copy_w * 1e6,
            # within one rank: how far apart its workgroups start (t0) and leave barrier 1 (t1)
            "wg_start_spread_us": float((t[:, :, 0].max(axis=1) - t[:, :, 0].min(axis=1)).max()
                                        * TICK_S * 1e6),
            "wg_barrier1_exit_spread_us": float((t[:, :, 1].max(axis=1) -
                                                 t[:, :, 1].min(axis=1)).max() * TICK_S * 1e6),
            "fold_GBps": fold_bytes / fold_w / 1e9,
            "copy_GBps": copy_bytes / copy_w / 1e9 if copy_w > 0 else 0.0,
            "span_GBps": total_bytes / span / 1e9,
            **{f"{k}_median_us": float(np.median(v)) * 1e6 for k, v in per_wg.items()},
            **{f"{k}_max_us": float(v.max()) * 1e6 for k, v in per_wg.items()},
        })
    med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
    plain = max(r["event_ms_plain"] for r in res)
    out = {
        "P": P, "algo": algo, "elements": n, "dtype": "f32", "workgroups_per_rank": grid,
        "calls": len(rows),
        "proxy": "all ranks on one GPU (IPC between processes on one device): remote reads are "
                 "local HBM reads; one clock for the whole GPU",
        "bytes": {"fold_all_ranks": fold_bytes, "copy_all_ranks": copy_bytes,
                  "total_all_ranks": total_bytes},
        "event_ms_plain_kernel": round(plain, 4),
        "event_frac_of_hbm": round(total_bytes / (plain * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "median_over_calls": {k: round(v, 2) for k, v in med.items()},
        "phase_frac_of_hbm": {"fold": round(med["fold_GBps"] / HBM_PEAK_GBS, 4),
                              "copy": round(med["copy_GBps"] / HBM_PEAK_GBS, 4),
                              "span": round(med["span_GBps"] / HBM_PEAK_GBS, 4)},
        "share_of_span": {k: round(med[f"{k}_median_us"] / med["span_us"], 4)
                          for k in ("barrier1", "fold", "barrier2", "copy", "barrier3")},
        "err": max(r["err"] for r in res),
    }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=2)
    ap.add_argument("--n", type=int, default=64 << 20)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--algo", default="peer2", choices=["peer2", "peer2w"])
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--back-to-back", action="store_true",
                    help="stamped calls issued back to back (steady state), not after host barriers")
    ap.add_argument("--rocprof", default="")
    ap.add_argument("--pmc", default="")
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
        cmd = ["python3", "-u", os.path.abspath(__file__), "--rank", str(r), "--port", str(port),
               "--P", str(a.P), "--n", str(a.n), "--iters", str(a.iters), "--warmup",
               str(a.warmup), "--blocks", str(a.blocks), "--algo", a.algo, "--variant", str(a.variant)] + (["--back-to-back"] if a.back_to_back else [])
        if a.rocprof:  # the profiler wraps the rank program itself (nothing in between)
            d = os.path.join(a.rocprof, f"rank{r}")
            mode = ["--pmc", a.pmc] if a.pmc else ["--kernel-trace", "--stats"]
            cmd = ["rocprofv3", *mode, "--output-format", "csv", "-d", d,
                   "-o", f"rank{r}", "--"] + cmd
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    res = []
    for p in procs:
        o, _ = p.communicate(timeout=600)
        o = o.decode(errors="replace")
        if p.returncode != 0:
            print(o[-3000:], file=sys.stderr)
            raise SystemExit(p.returncode)
        res.append(json.loads([ln for ln in o.splitlines() if ln.startswith("RESULT ")][-1][7:]))
    out = summarize(a.P, a.n, res, a.algo)
    out["variant"] = a.variant
    out["stamped_calls"] = "back to back (steady state)" if a.back_to_back else "each after a host barrier"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
