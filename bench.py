#!/usr/bin/env python3
"""bench.py -- hydra bucket-reduction hot path on MI355X.

Metric (BASELINE.json): chunk-sum GB/s (fp32) vs HBM peak; ring-allreduce GB/s at 1/2/4/8 GPU.

  N = 1  (BASELINE config 2): one step = one device-resident, in-place fp32 chunk-sum
         c = a + b over 64 Mi elements (gloo::sum<float>, math.h:15-23, in the ring's c == a
         form), HBM-resident: launch k works on buffer pair k mod 4 (2 GiB cycled, 8x the
         Infinity Cache).  value = 12 B/element x elements x steps / wall time of the timed
         region; roofline.mall_assisted reports one pair back to back beside it.
         The line carries config 2's 4 Ki..64 Mi size sweep (HBM-resident and MALL-assisted
         rates per size; --no-sweep skips it).
  N > 1  (BASELINE config 4): one step = one allreduce of a 64 Mi-element fp32 bucket per rank
         over xGMI in the reference's block ownership and fold order -- the fastest bit-exact
         schedule of RCCL p2p with the HIP sum fused per hop (DIRECT / A2A / RING), and last
         the peer-access kernel that reads the peers' blocks over xGMI and folds them in one
         pass (benchkit/allreduce.py over hydra_amd.ring / hydra_amd.peer; it becomes the
         headline when bit-exact and faster).  value = N x bucket bytes / time
         (whole-job bucket bytes reduced per second); algbw and busbw = algbw x 2(N-1)/N are
         reported beside it.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under torch.distributed.run.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBS = 153.0      # per xGMI link, per direction (task brief)
N_MICRO = 64 << 20         # config 2 largest size; config 4 bucket


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--elements", type=int, default=N_MICRO)
    p.add_argument("--dtype", default="f32", choices=["f32", "i32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true",
                   help="N=1: skip the host-buffer (PCIe-inclusive) context leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="bounded CPU-baseline sample (seconds of reference gloo::sum work)")
    p.add_argument("--no-sweep", action="store_true",
                   help="skip the 4 Ki..64 Mi size sweep (BASELINE config 2's range), e.g. so a "
                        "kernel trace of the command holds the headline size only")
    p.add_argument("--algo", default="auto", help="ring algorithm for N>1 (see hydra_amd.ring)")
    p.add_argument("--watchdog-s", type=float, default=420.0,
                   help="N>1: abort (exit 3) if the run exceeds this many seconds")
    p.add_argument("--no-config5", action="store_true", help="N>1: skip the bf16 config-5 leg")
    p.add_argument("--config5-elements", type=int, default=256 << 20,
                   help="N>1: bf16 elements of the config-5 leg (a multiple of 1 Mi; "
                        "BASELINE: 256 Mi)")
    p.add_argument("--peer", nargs="?", const="on", default="auto",
                   choices=["auto", "on", "off"],
                   help="N>1: the peer-access (IPC, reduce-on-read) leg, run last: auto (default) "
                        "when every peer GPU is reached over xGMI with peer access; on: always "
                        "(e.g. ranks sharing one GPU); off: never")
    p.add_argument("--extra-legs", action="store_true",
                   help="N>1: also check and time the schedules outside north_star's path "
                        "(old-style rings, BCUBE, halving-doubling, gloo::reduce to a root)")
    p.add_argument("--force-dist", action="store_true",
                   help="run the N>1 (RCCL) path even at world size 1 (code-path check)")
    # watchdog rehearsal hooks (tests): a stage that hangs for this many seconds
    p.add_argument("--stall-autotune-s", type=float, default=0.0, help=argparse.SUPPRESS)
    p.add_argument("--stall-context-s", type=float, default=0.0, help=argparse.SUPPRESS)
    return p.parse_args()


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


# ------------------------------------------------------------------------------- N = 1
ROTATE = 4  # buffer pairs the headline cycles through: 4 x 512 MiB >> the 256 MiB Infinity Cache


def kernel_src_hash():
    """sha256 of the chunk-sum kernel's sources: ties a committed PMC profile to the kernel it
    measured (roofline.traffic is reported only while they match)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("reduce_kernels.hip", "reduce_ops.h", "reduce_kernels.h"):
        with open(os.path.join(ROOT, "hydra_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def make_pairs(torch, dev, n, code, count):
    from hydra_amd import _lib
    from hydra_amd import synth

    pairs = []
    for i in range(count):
        if code == _lib.FLOAT32:
            a = torch.from_numpy(synth.bew_inputs(i, n)).to(dev)
            b = torch.from_numpy(synth.uniform_f32(n, 42 + i)).to(dev)
        else:
            a = torch.from_numpy(synth.int32_bucket(8, 2 * i, n)).to(dev)
            b = torch.from_numpy(synth.int32_bucket(8, 2 * i + 1, n)).to(dev)
        pairs.append((a, b))
    return pairs


def time_chunk_sum(torch, L, dev, pairs, code, steps, warmup, per_launch=0, cold_reps=0):
    """Launch k of every leg runs in place on pairs[k % len(pairs)].  Returns (wall seconds for
    the `steps` launches of the timed region, average launch ms = HIP-event span over that region
    / steps, per-launch event ms (each launch bracketed alone, `per_launch` of them), cold ms
    (each launch after a 1 GiB fill, `cold_reps` of them))."""
    from hydra_amd import _lib

    n = pairs[0][0].numel()
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    ptrs = [(a.data_ptr(), b.data_ptr()) for a, b in pairs]
    R = len(ptrs)

    def launch(k):
        pa, pb = ptrs[k % R]
        _lib.check(L.hydra_chunk_sum(code, pa, pa, pb, n, sp))

    if True:  # (the shipped kernel: libhydra_hip.so has no variants)
        for k in range(warmup):
            launch(k)
        torch.cuda.synchronize(dev)
        # timed region: exactly `steps` launches, synchronised on both sides, bracketed by HIP
        # events on the launch stream (average launch duration = event span / steps)
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        r0.record(s)
        for k in range(steps):
            launch(k)
        r1.record(s)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        region_ms = r0.elapsed_time(r1) / steps
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(per_launch)]
        for k, (e0, e1) in enumerate(ev):
            e0.record(s)
            launch(k)
            e1.record(s)
        torch.cuda.synchronize(dev)
        ms = [e0.elapsed_time(e1) for e0, e1 in ev]
        cold = []
        if cold_reps:
            flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
            evc = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                   for _ in range(cold_reps)]
            for k, (e0, e1) in enumerate(evc):
                flush.fill_(1.0)
                e0.record(s)
                launch(k)
                e1.record(s)
            torch.cuda.synchronize(dev)
            cold = [e0.elapsed_time(e1) for e0, e1 in evc]
            del flush
    return wall, region_ms, ms, cold


def hbm_ceiling(torch, dev, pairs, launches=40, rounds=3):
    """What THIS HBM delivers, measured in the same run under the headline's rotation: two
    pure read streams (2R) and a copy (1R1W) over the same buffer pairs, with the chunk-sum's
    launch shape (hydra_amd/libhydra_probe.so, measurement-only kernels).  GB/s of algorithmic
    bytes (8 B per element for both), median over `rounds`.  None if the probe library is
    absent.  The copy overwrites each pair's b with a, so it runs after every chunk-sum leg."""
    import ctypes

    path = os.path.join(ROOT, "hydra_amd", "libhydra_probe.so")
    if not os.path.exists(path):
        return None
    P = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    P.hydra_probe_launch.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_size_t, vp]
    n = pairs[0][0].numel()
    s = torch.cuda.current_stream(dev)
    sink = torch.empty(max(1, n // 1024), dtype=torch.float32, device=dev)
    out = {}
    for kind, name in ((0, "read_2R"), (1, "copy_1R1W")):
        rates = []
        for r in range(rounds + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for k in range(launches):
                a, b = pairs[k % len(pairs)]
                rc = P.hydra_probe_launch(kind, b.data_ptr(), a.data_ptr(), b.data_ptr(),
                                          sink.data_ptr(), n, s.cuda_stream)
                if rc:
                    raise RuntimeError(f"hydra_probe_launch({kind}) failed: hipError {rc}")
            e1.record(s)
            torch.cuda.synchronize(dev)
            if r:  # the first round warms up
                rates.append(8.0 * n / (e0.elapsed_time(e1) / launches * 1e-3) / 1e9)
        out[name] = round(float(np.median(rates)), 1)
    return out


SWEEP_POOL_BYTES = 1 << 30  # per operand: the HBM-resident sweep cycles 2 GiB (8x the MALL)


def sweep_leg(torch, L, dev, code, lo=12, hi=26):
    """BASELINE config 2's range (runner.cc:338-362 sweeps sizes the same way): the in-place
    chunk-sum at 4 Ki, 16 Ki, ..., 64 Mi elements, back-to-back launches on the headline's
    stream, timed by HIP events over each run (event span / launches: what a caller issuing one
    segment after another sees, launch gaps included).
      hbm_resident   launch k works on slot k of two 1 GiB pools (operands a, b), so no launch
                     reuses another's lines until the 2 GiB cycle wraps
      mall_assisted  one slot back to back (its operands stay in the 256 MiB Infinity Cache
                     while they fit)
    bound: "dispatch" when moving the launch's 12 B/element at the 8 TB/s peak would take less
    than the smallest size's per-launch time (the launch floor), else "hbm"."""
    from hydra_amd import _lib

    esz = 4
    pool_a = torch.empty(SWEEP_POOL_BYTES // esz, dtype=torch.float32, device=dev)
    pool_b = torch.empty_like(pool_a)
    pool_a.copy_(torch.arange(pool_a.numel(), device=dev, dtype=torch.float32) % 1024)
    pool_b.fill_(1.0)
    if code != _lib.FLOAT32:
        pool_a, pool_b = pool_a.view(torch.int32), pool_b.view(torch.int32)
    s = torch.cuda.current_stream(dev)
    sp = s.cuda_stream
    pa, pb = pool_a.data_ptr(), pool_b.data_ptr()

    def run(nn, launches, slots):
        step = nn * esz
        for k in range(8):  # warm-up (code, TLB, clocks)
            _lib.check(L.hydra_chunk_sum(code, pa + (k % slots) * step, pa + (k % slots) * step,
                                         pb + (k % slots) * step, nn, sp))
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for k in range(launches):
            off = (k % slots) * step
            _lib.check(L.hydra_chunk_sum(code, pa + off, pa + off, pb + off, nn, sp))
        e1.record(s)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / launches  # ms per launch

    def run_graph(nn, launches, slots):
        """The same launches captured into one hipGraph and replayed: no host enqueue cost
        between kernels (what a captured ring step sees), only the device's own launch gaps."""
        step = nn * esz
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            cs = torch.cuda.current_stream(dev).cuda_stream
            for k in range(launches):
                off = (k % slots) * step
                _lib.check(L.hydra_chunk_sum(code, pa + off, pa + off, pb + off, nn, cs))
        g.replay()  # warm-up
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        g.replay()
        e1.record(s)
        torch.cuda.synchronize(dev)
        del g
        return e0.elapsed_time(e1) / launches

    rows, floor_us = [], None
    for k in range(lo, hi + 1, 2):
        nn = 1 << k
        slots = max(1, SWEEP_POOL_BYTES // (nn * esz))
        launches = 400 if nn <= (1 << 20) else 200 if nn <= (1 << 22) else 100 if nn <= (1 << 24) \
            else 40
        hbm_ms = run(nn, launches, slots)
        mall_ms = run(nn, launches, 1)
        try:
            graph_ms = run_graph(nn, launches, slots)
        except Exception as e:  # context only
            graph_ms, graph_err = None, str(e)
        us = hbm_ms * 1e3
        floor_us = us if floor_us is None else floor_us
        ideal_us = 12.0 * nn / (HBM_PEAK_GBS * 1e9) * 1e6
        hbm_gbs = 12.0 * nn / (hbm_ms * 1e-3) / 1e9
        mall_gbs = 12.0 * nn / (mall_ms * 1e-3) / 1e9
        rows.append({"elements": nn, "launches": launches, "hbm_slots": min(slots, launches),
                     "hbm_resident": {"us_per_launch": round(us, 2), "GBps": round(hbm_gbs, 1),
                                      "frac_of_peak": round(hbm_gbs / HBM_PEAK_GBS, 4)},
                     "mall_assisted": {"us_per_launch": round(mall_ms * 1e3, 2),
                                       "GBps": round(mall_gbs, 1),
                                       "frac_of_peak": round(mall_gbs / HBM_PEAK_GBS, 4)},
                     "hbm_resident_graph": (
                         {"us_per_launch": round(graph_ms * 1e3, 2),
                          "GBps": round(12.0 * nn / (graph_ms * 1e-3) / 1e9, 1),
                          "frac_of_peak": round(12.0 * nn / (graph_ms * 1e-3) / 1e9 /
                                                HBM_PEAK_GBS, 4)}
                         if graph_ms else {"error": graph_err}),
                     "ideal_us_at_peak": round(ideal_us, 3),
                     "bound": "dispatch" if ideal_us < floor_us else "hbm"})
    del pool_a, pool_b
    return {"rows": rows, "launch_floor_us": round(floor_us, 2), "bytes_per_element": 12,
            "peak_GBps": HBM_PEAK_GBS,
            "timing": "HIP events around back-to-back launches on one stream (event span / "
                      "launches): launch gaps are included, which is what makes the small sizes "
                      "dispatch-bound; hbm_resident_graph = the same launches captured in one "
                      "hipGraph and replayed (no host enqueue between kernels)",
            "note": "context: the headline value is the 64 Mi line; hbm_resident cycles two "
                    "1 GiB pools, mall_assisted repeats one slot"}


def pmc_traffic():
    """HBM bytes per launch of the 64 Mi chunk-sum from the committed rocprofv3 PMC summary
    (profiles/pmc_chunk_sum.json, written by scripts/pmc_summary.py from separate --pmc
    FETCH_SIZE / WRITE_SIZE passes over this command: FETCH_SIZE x2 gfx950 correction +
    WRITE_SIZE, MI355X_MICROARCH.md §HBM).  Returned only while the profile's kernel-source hash
    equals the current sources, so a kernel change cannot inherit a stale figure."""
    p = os.path.join(ROOT, "profiles", "pmc_chunk_sum.json")
    info = {"file": "profiles/pmc_chunk_sum.json"}
    if not os.path.exists(p):
        return None, dict(info, status="absent")
    try:
        with open(p) as f:
            d = json.load(f)
    except Exception as e:
        return None, dict(info, status=f"unreadable: {e}")
    cur = kernel_src_hash()
    info.update(round=d.get("round"), kernel_src_sha256=d.get("kernel_src_sha256"),
                mode=d.get("mode"))
    if d.get("kernel_src_sha256") != cur:
        return None, dict(info, status="stale: profiled kernel sources differ from these")
    return d.get("hbm_bytes_per_launch"), dict(info, status="matches these kernel sources")


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpulist(text):
    out = []
    for part in (text or "").split(","):
        if "-" in part:
            lo, hi = part.split("-")
            out.extend(range(int(lo), int(hi) + 1))
        elif part.strip():
            out.append(int(part))
    return out


def gpu_numa_node(device_index=0):
    """NUMA node of the GPU (its PCI device's numa_node in sysfs), or None."""
    try:
        import torch

        pr = torch.cuda.get_device_properties(device_index)
        bus = "%04x:%02x:%02x.0" % (getattr(pr, "pci_domain_id", 0), pr.pci_bus_id,
                                    pr.pci_device_id)
        node = _read(f"/sys/bus/pci/devices/{bus}/numa_node")
        return int(node) if node is not None and int(node) >= 0 else None
    except Exception:
        return None


def baseline_cores(k, device_index=0, node=-1):
    """k host CPUs for the CPU baselines: on the GPU's NUMA node (as a rank process runs,
    DESIGN.md 6.3), never CPU 0 (the housekeeping / interrupt core) nor its SMT sibling, one
    logical CPU per physical core while there are enough; within this process's affinity.
    node: the GPU's NUMA node if the caller knows it (-1: look it up, which initialises HIP).
    Returns (cpus, node, note)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    if node == -1:
        node = gpu_numa_node(device_index)
    pool = [c for c in _cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist"))
            if c in aff] if node is not None else []
    note = f"GPU NUMA node {node}" if pool else "GPU NUMA node unknown: process affinity"
    pool = pool or aff
    avoid = {0} | set(_cpulist(_read("/sys/devices/system/cpu/cpu0/topology/thread_siblings_list")))
    cand = [c for c in pool if c not in avoid] or pool
    firsts, seen = [], set()
    for c in cand:  # one logical CPU per physical core first
        sib = tuple(_cpulist(_read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list"))
                    or [c])
        if sib not in seen:
            seen.add(sib)
            firsts.append(c)
    order = firsts + [c for c in cand if c not in firsts]
    return order[:max(1, k)], node, note


def _host_cpu():
    try:
        with open("/proc/cpuinfo") as f:
            return next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")),
                        None)
    except OSError:
        return None


def cpu_baseline(n, seconds):
    """The reference's own gloo::sum<float> (oracle/_ref, compiled from /root/reference) timed
    single-threaded on this host at the headline's size; falls back to the C restatement
    (oracle/liboracle.so).  Pinned to one core of the GPU's NUMA node (not CPU 0); three
    repetitions, every one reported."""
    from oracle import oracle as O

    kind = "reference" if O.ref_available() else "port"
    prev_aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    cores, node, note = baseline_cores(1)
    core = cores[0] if cores else None
    if core is not None:
        os.sched_setaffinity(0, {core})
    try:
        # the operands are first touched by the pinned core, so their pages are on its NUMA node:
        # the same loop reads 70-72 GB/s from local pages and 44-45 GB/s from the other socket's
        # (scripts/probe_cpu_baseline.py, profiles/r04za_cpu_baseline_numa.json), which is what
        # made rounds 3-4's baseline read ~45 or ~70 GB/s depending on where the process started
        a = np.arange(n, dtype=np.float32)
        b = np.ones(n, dtype=np.float32)
        # calibrate, then ~`seconds` of work as 3 timed repetitions (mean per call of each)
        reps = []
        if kind == "reference":
            per = O.ref_time_sum(6, a, a, b, 1, 1)
            iters = max(1, int(seconds / max(per, 1e-6) / 3))
            for _ in range(3):
                reps.append(O.ref_time_sum(6, a, a, b, iters, 1))
        else:
            per = 0.0
            t0 = time.perf_counter()
            O.orc().orc_op(0, 6, a.ctypes.data, a.ctypes.data, b.ctypes.data, n)
            iters = max(1, int(seconds / max(time.perf_counter() - t0, 1e-6) / 3))
            for _ in range(3):
                t0 = time.perf_counter()
                for _ in range(iters):
                    O.orc().orc_op(0, 6, a.ctypes.data, a.ctypes.data, b.ctypes.data, n)
                reps.append((time.perf_counter() - t0) / iters)
    finally:
        if core is not None and prev_aff:
            os.sched_setaffinity(0, prev_aff)
    rates = [12.0 * n / r / 1e9 for r in reps]
    per = float(np.median(reps))
    return {"value": round(12.0 * n / per / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": kind,
            "host_cpu": _host_cpu(), "host_logical_cpus": os.cpu_count(),
            "pinned_cpu": core, "numa_node": node, "placement": note,
            "repetitions_GBps": [round(r, 3) for r in rates],
            "spread": round((max(rates) - min(rates)) / float(np.median(rates)), 4),
            "sample": f"gloo::sum<float> in place over {n} fp32 elements (the headline's size, "
                      f"12 B/element), single thread pinned to host CPU {core} ({note}), "
                      "operands first-touched by that core (NUMA-local pages), "
                      f"{iters} calls x 3 repetitions (~{seconds:.0f} s); value = the median "
                      "repetition",
            "per_call_ms": round(per * 1e3, 3)}


def host_path_leg(n=16 << 20, calls=5):
    """Context: the same chunk-sum on HOST buffers through
    hydra_reduce_host, c == a in place as the ring calls it -- the PCIe-inclusive rate, never
    `value`.  pinned: hipHostMalloc'd operands read and written in place over PCIe (zero-copy);
    pageable: plain heap operands, copied by the CPU through the context's pinned staging.  GB/s
    of algorithmic bytes (12 B/element), median of `calls` calls after one untimed call."""
    from hydra_amd import _lib
    from hydra_amd.reduce import HostContext

    L = _lib.lib()
    out = {"elements": n, "bytes_per_element": 12, "calls": calls,
           "note": "operands in host memory: bound by PCIe (DESIGN.md 6.3), context only"}
    # as a rank process runs: on CPUs of the GPU's NUMA node, operands allocated
    # there (the copy helpers the staged path starts inherit the placement)
    prev_aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    cores, node, note = baseline_cores(8)
    if cores:
        os.sched_setaffinity(0, set(cores))
        out["placement"] = {"cpus": cores, "numa_node": node, "note": note}
    try:
        return _host_path_calls(L, HostContext, n, calls, out)
    finally:
        if cores and prev_aff:
            os.sched_setaffinity(0, prev_aff)


def _host_path_calls(L, HostContext, n, calls, out):
    import ctypes

    from hydra_amd import _lib

    ctx = HostContext(0)
    blocks = []
    try:
        def alloc_pinned():
            p = ctypes.c_void_p()
            _lib.check(L.hydra_malloc_host(n * 4, ctypes.byref(p)))
            blocks.append(p)
            return np.frombuffer((ctypes.c_char * (n * 4)).from_address(p.value), np.float32)

        kinds = {"pinned_zero_copy": (alloc_pinned(), alloc_pinned()),
                 "pageable_staged": (np.empty(n, np.float32), np.empty(n, np.float32))}
        for name, (a, b) in kinds.items():
            a[:] = np.arange(n, dtype=np.float32) % 1024
            b[:] = 1.0
            _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                           b.ctypes.data, n))
            ok = bool(np.array_equal(a, (np.arange(n, dtype=np.float32) % 1024) + 1.0))
            ts = []
            for _ in range(calls):
                t0 = time.perf_counter()
                _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                               b.ctypes.data, n))
                ts.append(time.perf_counter() - t0)
            med = float(np.median(ts))
            out[name] = {"ms_per_call": round(med * 1e3, 3),
                         "GBps": round(12.0 * n / med / 1e9, 2), "first_call_exact": ok}
    finally:
        ctx.close()
        for p in blocks:
            L.hydra_free_host(p)
    return out


def run_single(args):
    import torch

    from hydra_amd import _lib

    L = _lib.lib()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    code = _lib.FLOAT32 if args.dtype == "f32" else _lib.INT32
    n = args.elements
    algo_bytes = 12.0 * n
    pairs = make_pairs(torch, dev, n, code, ROTATE)
    # headline: HBM-resident launches, each on the next of ROTATE buffer pairs, so no launch
    # finds its operands in the 256 MiB Infinity Cache (2 GiB cycled between reuses)
    wall, region_ms, ms, cold = time_chunk_sum(torch, L, dev, pairs, code, args.steps,
                                               args.warmup, per_launch=min(100, args.steps),
                                               cold_reps=20)
    # context: one pair back to back -- part of its 512 MiB stays in the Infinity Cache
    mwall, mregion, _, _ = time_chunk_sum(torch, L, dev, pairs[:1], code, 20, 2)
    value = algo_bytes * args.steps / wall / 1e9
    achieved = algo_bytes / (region_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic()
    out = {
        "metric": "chunk-sum GB/s (fp32) vs HBM peak; ring-allreduce GB/s at 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32" if code == _lib.FLOAT32 else "i32", "data": "synthetic",
        "config": {"workload": "device-resident in-place chunk sum c=a+b (gloo::sum<float> "
                               "ring form), BASELINE config 2, HBM-resident: launch k runs on "
                               f"buffer pair k mod {ROTATE} ({ROTATE} x 512 MiB cycled)",
                   "elements": n, "bytes_per_element": 12, "buffer_pairs": ROTATE,
                   "parallelism": "single GPU"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_ms_avg": round(region_ms, 5),
                     "timing": "HIP events on the launch stream over the timed region "
                               "(event span / steps), HBM-resident rotation",
                     "per_launch_event_ms_median": round(float(np.median(ms)), 5),
                     "frac_of_measured_copy_ceiling": round(achieved / 6290.0, 4),
                     "copy_ceiling_note": "6.29 TB/s = best float4 HBM copy measured on MI355X "
                                          "(MI355X_MICROARCH.md); spec peak 8 TB/s",
                     "cold_achieved": round(algo_bytes / (float(np.median(cold)) * 1e-3) / 1e9, 1),
                     "cold_note": "median over 20 launches, each after a 1 GiB fill that "
                                  "evicts the 256 MiB Infinity Cache",
                     "mall_assisted": {
                         "achieved": round(algo_bytes / (mregion * 1e-3) / 1e9, 1),
                         "frac": round(algo_bytes / (mregion * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "kernel_ms_avg": round(mregion, 5),
                         "note": "context only: ONE buffer pair launched back to back (20 "
                                 "launches); part of its 512 MiB working set is served by the "
                                 "256 MiB Infinity Cache, so this is not an HBM rate"}},
    }
    try:  # the ceiling this HBM delivers, same run, same rotation (after every chunk-sum leg)
        ceil = hbm_ceiling(torch, dev, pairs)
    except Exception as e:  # context for the roofline, never the product
        ceil = {"error": str(e)}
    if ceil and "read_2R" in ceil:
        out["roofline"]["measured_ceiling"] = dict(
            ceil, unit="GB/s", note="same run, same 4-pair rotation: two pure read streams and "
                                   "a copy with the chunk-sum's launch shape "
                                   "(hydra_amd/csrc/probe_kernels.hip); a 2-read + 1-write "
                                   "stream cannot exceed the pure-read rate")
        out["roofline"]["frac_of_measured_read_ceiling"] = round(achieved / ceil["read_2R"], 4)
        if ceil.get("copy_1R1W"):
            # per-byte cost model fitted to the two probes: a read byte costs 1/read_2R, a
            # written byte (8/copy - 4/read_2R)/4, so the chunk-sum's mix of 8 read + 4 written
            # bytes per element is bounded by 12 / (4/read_2R + 8/copy_1R1W)
            mix = 12.0 / (4.0 / ceil["read_2R"] + 8.0 / ceil["copy_1R1W"])
            out["roofline"]["measured_ceiling"]["mix_2R1W_model"] = round(mix, 1)
            out["roofline"]["frac_of_measured_mix_ceiling"] = round(achieved / mix, 4)
    elif ceil:
        out["roofline"]["measured_ceiling"] = ceil
    del pairs
    if not args.no_sweep:
        # config 2's whole size range (context: the headline is the 64 Mi line above), for the
        # line's dtype and for int32 (the microbench runs fp32 and int32)
        other = _lib.INT32 if code == _lib.FLOAT32 else _lib.FLOAT32
        for key, c in (("sweep", code), ("sweep_" + ("int32" if other == _lib.INT32 else "f32"),
                                         other)):
            try:
                out[key] = sweep_leg(torch, L, dev, c)
            except Exception as e:
                out[key] = {"error": str(e)}
    if not args.no_host_path:
        try:  # row N2: the PCIe-inclusive host-buffer rate beside the HBM one (context only)
            out["host_path"] = host_path_leg()
        except Exception as e:  # context, never the product's headline
            out["host_path"] = {"error": str(e)}
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds)
        except Exception as e:  # the baseline is reported, never the product
            out["cpu_baseline"] = {"value": None, "error": str(e)}
    print(json.dumps(out), flush=True)


# ------------------------------------------------------------------------------- N > 1
def ring_cpu_baseline(P, n, seconds):
    """The reference's own new_allreduce_ring benchmark body (oracle/_ref: gloo::allreduce RING
    with gloo::sum<float>, compiled from /root/reference; benchmark/main.cc:321-358) on P
    thread-ranks over loopback TCP on this host, n fp32 elements per rank, per-iteration wall
    time of rank 0 as runner.cc:683-702 measures it.  A bounded sample: one calibration
    allreduce, then as many as fit in ~`seconds` (1..20).  Falls back to nothing (an error
    entry) when the reference library was not built -- never to the product."""
    from oracle import oracle as O

    if not O.ref_available():
        raise RuntimeError("oracle/_ref (the reference built from its sources) is not present")
    # the 2P threads (1 user + 1 event loop per rank) on 2P CPUs of the GPU's NUMA node, not
    # CPU 0 (the reference's threads inherit the process affinity)
    prev_aff = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    cores, node, note = baseline_cores(2 * P)
    if cores:
        os.sched_setaffinity(0, set(cores))
    try:
        t0 = time.perf_counter()
        O.ref_bench_ring(P, n, 0, 1)  # calibration (connect + one allreduce)
        per = max(time.perf_counter() - t0, 1e-3)
        iters = int(max(1, min(20, seconds / per)))
        s = O.ref_bench_ring(P, n, 1, iters) * 1e-9  # seconds per iteration, rank 0
    finally:
        if cores and prev_aff:
            os.sched_setaffinity(0, prev_aff)
    avg = float(np.mean(s))
    model = _host_cpu()
    return {"value": round(P * 4.0 * n / avg / 1e9, 3), "unit": "GB/s", "cores": 2 * P,
            "kind": "reference", "pinned_cpus": cores, "numa_node": node, "placement": note,
            "sample": f"{iters} allreduces (after 1 warm-up) of the reference's gloo::allreduce "
                      f"RING + gloo::sum<float> over {n} fp32 elements per rank on {P} "
                      "thread-ranks, loopback TCP (1 user + 1 event-loop thread per rank), "
                      f"pinned to CPUs {cores} ({note})",
            "value_def": "P x n x 4 B / mean per-iteration time (the same whole-job definition "
                         "as this line's value)",
            "ms_p50": round(float(np.percentile(s, 50)) * 1e3, 3),
            "ms_avg": round(avg * 1e3, 3),
            "GiBps_runner": round(4.0 * n / avg / 2 ** 30, 4),
            "host_cpu": model, "host_logical_cpus": os.cpu_count()}


def run_multi(args):
    import torch
    import torch.distributed as dist

    from benchkit import allreduce as bench_ar

    ws, rank, local = dist_env()
    if ws == 1:  # --force-dist without a launcher
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    # Rehearsal on a one-GPU box (never the driver's run): every rank on GPU 0, each with its own
    # RCCL host identity, so RCCL accepts N ranks on one GPU and links them over loopback
    # sockets.  The whole N>1 path runs with real RCCL ranks; the rates are socket rates.
    rehearse = os.environ.get("HYDRA_BENCH_SHARED_GPU") == "1"
    if rehearse:
        local = 0
        os.environ["NCCL_HOSTID"] = f"hydra-rehearsal-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    try:
        base = None
        if not args.no_cpu_baseline:
            def base(P, n):
                return ring_cpu_baseline(P, n, args.cpu_seconds)
        res = bench_ar.bench_allreduce(args, dev, cpu_baseline=base)
    finally:
        dist.destroy_process_group()
    if rehearse:
        res["rehearsal"] = ("HYDRA_BENCH_SHARED_GPU=1: all ranks on one GPU, RCCL over loopback "
                            "sockets -- a code-path check, not an xGMI rate")
    if rank == 0:
        print(json.dumps(res), flush=True)


def main():
    args = parse()
    ws, _, _ = dist_env()
    if ws != args.gpus and not (ws == 1 and args.gpus == 1):
        if ws == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with "
                             f"--nproc-per-node {args.gpus}")
    if ws > 1 or args.force_dist:
        run_multi(args)
    else:
        run_single(args)


if __name__ == "__main__":
    main()
