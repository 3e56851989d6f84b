"""The N>1 bench (bench.py --gpus N): BASELINE config 4 / 5 allreduces over the product's
communicators (hydra_amd.ring.XgmiComm, hydra_amd.peer.PeerComm), timed per the bench contract,
with parity self-checks, the autotune, context legs, the peer-access leg and the JSON line.

Bench-side code (not the product): the product package hydra_amd/ holds only the allreduce's
Python face; this module drives it.  The schedules' self-check expectations below restate the
reference's fold orders for the bench's own gate (the oracle is the tests' checker).
"""
from __future__ import annotations

import os
import time

import numpy as np

from hydra_amd import _lib
from hydra_amd._lib import HydraError
from hydra_amd.ring import XgmiComm, exchange_unique_id, split_elements

def max_over_ranks(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(run_step, steps: int, warmup: int, sync, barrier) -> float:
    """warmup untimed, then exactly `steps` bracketed by barrier + sync on both sides."""
    for _ in range(warmup):
        run_step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        run_step()
    sync()
    barrier()
    return time.perf_counter() - t0


def expected_fold_f32(xs: list[np.ndarray], max_segment: int = 1 << 20) -> np.ndarray:
    """Self-check for the bench (not the oracle): the reference ring's result for in-place
    fp32 buckets -- block q = [qS*sb, (q+1)S*sb) folded x_q + (x_{q+1} + (... + x_{q-1}))."""
    P, n = len(xs), xs[0].size
    ns, sb, S = _lib.ring_plan(P, n, 4, max_segment)
    out = np.empty(n, np.float32)
    for q in range(P):
        lo, hi = min(n, q * S * sb // 4), min(n, (q + 1) * S * sb // 4)
        if lo >= hi:
            continue
        acc = xs[(q + P - 1) % P][lo:hi].astype(np.float32)
        for d in range(P - 2, -1, -1):
            acc = xs[(q + d) % P][lo:hi] + acc
        out[lo:hi] = acc
    return out


def expected_fold_at(P: int, n: int, idx: np.ndarray, gen, esize: int = 4,
                     max_segment: int = 1 << 20) -> np.ndarray:
    """Self-check for the bench's full-size gate (not the oracle): the reference ring's result at
    element indices idx of an n-element bucket whose rank-r values are gen(P, r, idx)
    (synth.stress_at: fp32; synth.stress_cancel_at with esize 2: bf16 values accumulated in fp32
    and rounded once, config 5).  Owner block q = [qS*sb, (q+1)S*sb) in elements (allreduce.cc:
    199-221), folded x_q + (x_{q+1} + (... + x_{q-1})) in fp32.  Returns fp32 (esize 4) or the
    bf16 bit patterns (esize 2)."""
    from hydra_amd import synth

    _, sb, S = _lib.ring_plan(P, n, esize, max_segment)
    owner = np.minimum(idx // (S * sb // esize), P - 1)
    vals = [gen(P, r, idx).astype(np.float32) for r in range(P)]
    if esize == 2:  # the bucket holds bf16: the values each rank contributes, widened
        vals = [synth.bf16_to_f32(synth.bf16_bits(v)) for v in vals]
    out = np.empty(idx.size, np.float32)
    for q in range(P):
        sel = owner == q
        acc = vals[(q + P - 1) % P][sel].copy()
        for d in range(P - 2, -1, -1):
            acc = vals[(q + d) % P][sel] + acc
        out[sel] = acc
    return synth.bf16_bits(out) if esize == 2 else out


def sample_indices(n: int, count: int = 1 << 20, seed: int = 7) -> np.ndarray:
    """The bench gate's sample: every 1 MiB-segment edge region, both bucket ends, `count`
    seeded random indices."""
    seg = 1 << 18  # fp32 elements per 1 MiB segment (bf16: every second edge)
    edges = np.concatenate([np.arange(0, n + seg, seg, dtype=np.int64) + d for d in (-1, 0)])
    rnd = np.random.default_rng(seed).integers(0, n, min(count, n), dtype=np.int64)
    idx = np.unique(np.concatenate([edges, rnd, [0, n - 1]]))
    return idx[(idx >= 0) & (idx < n)]


def reduce_geometry(P: int, n: int, esize: int, max_segment: int = 1 << 20):
    """gloo::reduce's segment geometry (reduce.cc:87-135) -> (numSegments, segmentBytes, S)."""
    total = n * esize
    msb = esize * (max_segment // esize)
    sb = min((total + 2 * P - 1) // (2 * P), msb)
    sb = -(-sb // esize) * esize
    ns = max(-(-total // sb), 2 * P)
    ns = -(-ns // P) * P
    return ns, sb, ns // P


def expected_reduce_f32(xs: list[np.ndarray], max_segment: int = 1 << 20) -> np.ndarray:
    """Self-check for the bench: gloo::reduce's root result for fp32 buckets -- the ring fold
    over gloo::reduce's own blocks."""
    P, n = len(xs), xs[0].size
    ns, sb, S = reduce_geometry(P, n, 4, max_segment)
    out = np.empty(n, np.float32)
    for q in range(P):
        lo, hi = min(n, q * S * sb // 4), min(n, (q + 1) * S * sb // 4)
        if lo >= hi:
            continue
        acc = xs[(q + P - 1) % P][lo:hi].astype(np.float32)
        for d in range(P - 2, -1, -1):
            acc = xs[(q + d) % P][lo:hi] + acc
        out[lo:hi] = acc
    return out


def expected_old_ring_f32(xs: list[np.ndarray], rank: int) -> np.ndarray:
    """Self-check for the bench: the old-style AllreduceRing<T> result on `rank` -- its own left
    fold x_r + x_{r-1} + ... + x_{r-P+1} (allreduce_ring.h:71-106)."""
    P = len(xs)
    acc = xs[rank].astype(np.float32)
    for d in range(1, P):
        acc = acc + xs[(rank - d) % P]
    return acc


def expected_chunked_ring_f32(xs: list[np.ndarray]) -> np.ndarray:
    """Self-check for the bench: AllreduceRingChunked<T>'s result -- chunk c (2P chunks of
    max(256, ceil(n/2P))) seeded by s = c/2 and folded x_{s+1} + x_s, x_{s+2} + (...), ..."""
    P, n = len(xs), xs[0].size
    ce = max(256, -(-n // (2 * P)))
    out = np.empty(n, np.float32)
    for c in range(2 * P):
        lo, hi = min(n, c * ce), min(n, (c + 1) * ce)
        if lo >= hi:
            continue
        s = c // 2
        acc = xs[s][lo:hi].astype(np.float32)
        for d in range(1, P):
            acc = xs[(s + d) % P][lo:hi] + acc
        out[lo:hi] = acc
    return out


def expected_bcube_f32(xs: list[np.ndarray]) -> np.ndarray:
    """Self-check for the bench: gloo's BCUBE result (allreduce.cc:423-700) -- per step, each
    rank folds its group's partials into its chunk, own value first, peers in group order."""
    P, n = len(xs), xs[0].size
    part = [x.astype(np.float32).copy() for x in xs]
    sizes, left = [], P
    while left % 2 == 0:
        sizes.append(2)
        left //= 2
    if left > 1:
        sizes.append(left)
    rng = [(0, n)] * P
    dist = 1
    for g in sizes:
        snap = [p.copy() for p in part]
        new = []
        for r in range(P):
            grank = (r // dist) % g
            base = r - grank * dist
            off, ln = rng[r]
            ch = -(-ln // g)
            mo, ml = off + grank * ch, max(0, min(ch, ln - grank * ch))
            for i in range(g):
                peer = base + i * dist
                if peer != r and ml:
                    part[r][mo:mo + ml] = part[r][mo:mo + ml] + snap[peer][mo:mo + ml]
            new.append((mo, ml))
        rng = new
        dist *= g
    out = np.empty(n, np.float32)
    for r in range(P):
        mo, ml = rng[r]
        out[mo:mo + ml] = part[r][mo:mo + ml]
    return out


HBM_PEAK_GBS = 8000.0
XGMI_LINK_GBS = 153.0


def _sig(x: float, digits: int = 4) -> float:
    """x rounded to `digits` significant digits (slow test transports must not round to 0)."""
    from math import floor, log10

    return 0.0 if x == 0 else round(x, digits - 1 - int(floor(log10(abs(x)))))


def phase_report(ph: dict, P: int, n: int, esize: int) -> dict:
    """The N>1 line's own roofline evidence from one profiled (untimed) allreduce: comm-stream
    (link) vs compute-stream (fold) busy time, their overlap, per-link GB/s against one xGMI
    link, and the fold kernels' HBM fraction.  Algorithmic bytes: per-rank link bytes
    2(P-1)/P*n*E and fused-sum HBM bytes (P-1)/P*n*3E (12 B/element for fp32);
    the fold kernels' own algorithmic bytes ((nsrc+1) x block per FOLD, 3 x segment per REDUCE)
    beside them."""
    calls = max(1, int(ph.get("calls", 0)))
    link, fold, span = ph["link_ms"] / calls, ph["fold_ms"] / calls, ph["span_ms"] / calls
    sent = ph["sent_bytes"] / calls
    peers = max(1, int(ph.get("peers", 0)))
    fused = (P - 1) / P * n * 3 * esize
    kern = ph["fold_hbm_bytes"] / calls
    out = {
        "calls": int(ph.get("calls", 0)),
        "link_ms": round(link, 4), "fold_ms": round(fold, 4), "span_ms": round(span, 4),
        "overlap_ms": round(max(0.0, link + fold - span), 4),
        "bound": "link" if link >= fold else "fold",
        "link": {"sent_bytes": int(sent), "recv_bytes": int(ph["recv_bytes"] / calls),
                 "algorithmic_bytes": int(2 * (P - 1) / P * n * esize), "peers": peers,
                 "ops": int(ph["link_ops"] / calls),
                 "aggregate_GBps": _sig(sent / (link * 1e-3) / 1e9) if link > 0 else None,
                 "per_link_GBps": (_sig(sent / peers / (link * 1e-3) / 1e9)
                                   if link > 0 else None),
                 "link_peak_GBps": XGMI_LINK_GBS},
        "fold": {"kernel_hbm_bytes": int(kern), "fused_sum_bytes": int(fused),
                 "ops": int(ph["fold_ops"] / calls),
                 "kernel_GBps": _sig(kern / (fold * 1e-3) / 1e9) if fold > 0 else None,
                 "hbm_peak_GBps": HBM_PEAK_GBS},
    }
    if out["link"]["per_link_GBps"] is not None:
        out["link"]["frac_of_link"] = _sig(out["link"]["per_link_GBps"] / XGMI_LINK_GBS)
    if out["fold"]["kernel_GBps"] is not None:
        out["fold"]["frac_of_hbm"] = _sig(out["fold"]["kernel_GBps"] / HBM_PEAK_GBS)
    return out


def _peer_mode(args) -> str:
    """bench.py --peer: "auto" (default: the peer leg runs when every peer GPU of this node is
    reached over xGMI with peer access), "on" (always: e.g. the one-GPU rehearsal, where the
    ranks share a GPU) or "off".  (A bool from older callers: True = on, False = off.)"""
    v = getattr(args, "peer", "auto")
    if v is True:
        return "on"
    if v is False or v is None:
        return "off"
    return str(v)


def bench_allreduce(args, dev, make_comm=None, sync=None, cpu_baseline=None,
                    make_peer=None) -> dict:
    """bench.py --gpus N (N > 1): BASELINE config 4 (fp32 64 Mi per rank) on this rank.

    make_comm() -> a communicator with XgmiComm's allreduce_ / reduce_ / apipe_allreduce_ /
    close (default: an RCCL XgmiComm over this rank's GPU, its unique id broadcast over the
    process group); sync() waits for this rank's enqueued work (default: the device);
    make_peer() -> the peer-access group of the last leg (default: hydra_amd.peer.PeerComm).  The
    hooks let tests/test_bench_gloo.py run this whole orchestration -- parity self-checks,
    autotune, timed region, context legs, the peer leg, JSON line -- at world size 2 to 8 on the
    CPU, with the same plans executed over gloo p2p."""
    import torch
    import torch.distributed as dist

    from hydra_amd import synth

    rank, world = dist.get_rank(), dist.get_world_size()
    # a hung collective must fail the run, not stall it: hard exit (status 3) after `watchdog_s`,
    # printing the measured headline flagged when there is one (benchkit/watchdog.py)
    from . import watchdog

    state = {}  # "result": builds the JSON line once the headline measurement is complete
    dog = watchdog.start(rank, float(getattr(args, "watchdog_s", 420)), state)
    if make_comm is None:
        def make_comm():
            return XgmiComm(rank, world, dev.index, exchange_unique_id(rank, dev))
    if sync is None:
        def sync():
            torch.cuda.synchronize(dev)
    comm = make_comm()
    rail2 = make_comm()  # apipe's 2nd rail
    # what RCCL itself reports for the communicator (ncclCommCount / UserRank / CuDevice): the
    # line shows that RCCL saw N ranks, and that every rank agrees
    try:
        info = comm.info()
    except HydraError as e:
        info = {"error": str(e)}
    cnt = float(info.get("nccl_comm_count", -1))
    comm_seen = {"nccl_comm_count": int(cnt),
                 "min_over_ranks": int(-max_over_ranks(-cnt, dev)),
                 "max_over_ranks": int(max_over_ranks(cnt, dev)),
                 "user_rank": info.get("nccl_user_rank"), "device": info.get("nccl_device"),
                 "backend": info.get("backend", "rccl")}
    if "error" in info:
        comm_seen["error"] = info["error"]
    # the fabric between this rank's GPU and the node's others (xGMI vs PCIe, hops, peer
    # access): the line shows what its links were (empty when the process sees one GPU)
    try:
        comm_seen["links_from_device"] = (_lib.device_links(dev.index)
                                          if getattr(dev, "type", "") == "cuda" else [])
    except (HydraError, RuntimeError) as e:
        comm_seen["links_from_device"] = f"n/a: {e}"
    extra_legs = bool(getattr(args, "extra_legs", False))
    cpu_base = None
    if make_peer is None:
        def make_peer():
            from hydra_amd.peer import PeerComm

            return PeerComm(rank, world, dev.index)

    # IPC-mapped buckets, one kernel per allreduce: set up in the LAST leg only (7 below), after
    # every other field of the line is measured
    pg = {"peer": None, "err": "not set up yet"}
    peer_leg = {}
    n = args.elements
    algo = getattr(args, "algo", "auto")

    # ranks sharing ONE GPU (the rehearsal, HYDRA_BENCH_SHARED_GPU=1): the peer kernel's
    # barriers need every rank's grid resident at once, and a GPU holds 512 of its workgroups
    # (two per CU at its register count), so each rank's grid is capped at 512 / world there
    shared_cap = max(1, 512 // world) if os.environ.get("HYDRA_BENCH_SHARED_GPU") == "1" else 0

    def run(a, t, ch=0, **kw):
        """ch: RCCL plans' pipelining chunk in bytes; peer algorithms' workgroup count."""
        if a in _lib.PEER_ALGOS:
            if pg["peer"] is None:
                raise HydraError(3, f"peer group unavailable: {pg['err']}")
            if shared_cap:
                ch = min(ch, shared_cap) if ch else shared_cap
            pg["peer"].set_option(_lib.PEER_OPT_BLOCKS, ch)
            pg["peer"].allreduce_(t, algo=a, **kw)
        else:
            comm.allreduce_(t, algo=a, chunk_bytes=ch, **kw)

    try:
        # 1) parity self-check on fold-order-sensitive inputs (small bucket), every algorithm
        pn = 1 << 20  # equal blocks at P = 2..8, so A2A is checked too
        xs = [synth.stress_f32(world, r, pn) for r in range(world)]
        exp = expected_fold_f32(xs)
        parity = {}
        tp = torch.empty(pn, dtype=torch.float32, device=dev)
        for a in ("direct", "ring", "a2a"):
            tp.copy_(torch.from_numpy(xs[rank]))
            try:
                run(a, tp)
            except HydraError as e:  # e.g. A2A with unequal blocks at this P
                parity[a] = f"n/a: {e}"
                continue
            sync()
            ok = bool(np.array_equal(tp.cpu().numpy().view(np.uint32), exp.view(np.uint32)))
            ok_all = max_over_ranks(0.0 if ok else 1.0, dev) == 0.0
            parity[a] = "bit-exact" if ok_all else "MISMATCH"
        # 2) exactness at full size on fold-order-sensitive values (synth.stress_at: the fp32
        #    result depends on block ownership and fold order).  DIRECT -- the schedule the tests
        #    pin at this size against the reference -- runs first: its bucket is this run's
        #    reference result, checked against the reference fold on sampled indices and its
        #    sha256 compared across ranks.  Every other schedule must reproduce it bit for bit on
        #    every rank before it is timed or promoted.
        x0 = synth.fill_at(synth.stress_at, world, rank, n, dev, torch.float32)
        x = x0.clone()
        ref = x0.clone()
        run("direct", ref)
        sync()
        gate = _full_size_gate(ref, world, n, synth.stress_at, 4, dev)

        def full_exact(a, ch=0):
            x.copy_(x0)
            run(a, x, ch)
            sync()
            good = bool(torch.equal(x.view(torch.int32), ref.view(torch.int32)))
            return gate["ok"] and max_over_ranks(0.0 if good else 1.0, dev) == 0.0

        full_ok = {"direct": gate["ok"]}
        def measure(a, ch, runner=None):
            """The timed region (exactly `steps` allreduces, barrier + sync on both sides, max
            over ranks) and the per-iteration latency as the reference's benchmark reports it
            (runner.cc:693-697: wall time around each run(), p50/p99), outside the region.
            runner: run() by default (the peer leg passes one that records errors instead of
            raising, so every rank still issues the same collectives)."""
            go = runner or run

            def step():
                go(a, x, ch)

            wall = max_over_ranks(timed_steps(step, args.steps, args.warmup, sync, dist.barrier),
                                  dev)
            lat = []
            for _ in range(max(5, min(50, args.steps))):
                sync()
                dist.barrier()
                sync()
                t0 = time.perf_counter()
                step()
                sync()
                lat.append(time.perf_counter() - t0)
            return wall / args.steps * 1e3, {
                "p50": round(max_over_ranks(float(np.percentile(lat, 50)), dev) * 1e3, 4),
                "p99": round(max_over_ranks(float(np.percentile(lat, 99)), dev) * 1e3, 4),
                "samples": len(lat), "note": "per step, synchronised, max over ranks"}

        tuning = {}
        if algo == "auto" and full_ok["direct"]:
            # a safe headline first (DIRECT, default chunk): if a later candidate hangs, the
            # watchdog still reports a measured bit-exact schedule
            ms_safe, lat_safe = measure("direct", 0)
            state["result"] = lambda: _bench_result(
                n, world, args, "direct", 0, dict(tuning), parity, full_ok, ms_safe, lat_safe,
                {}, None, comm_seen, gate=gate)
        # 3) pick the algorithm: "auto" = the fastest bit-exact RCCL schedule on this node
        #    (DIRECT / A2A / RING), chosen on a few untimed steps; the peer-access kernel is
        #    checked and timed last (7) and replaces this headline only if it is faster
        chosen, chunk = algo, 0
        stall = float(getattr(args, "stall_autotune_s", 0.0) or 0.0)
        if stall > 0:  # rehearsal hook (bench.py --stall-autotune-s): an autotune candidate hangs
            time.sleep(stall)
        if algo == "auto":
            best = None
            for a, ch in (("direct", 1 << 20), ("direct", 4 << 20), ("direct", 16 << 20),
                          ("direct", 64 << 20), ("a2a", 0), ("ring", 4 << 20)):
                if parity.get(a) != "bit-exact":
                    continue  # only schedules that reproduced the reference are eligible
                try:
                    def tstep(a=a, ch=ch):
                        run(a, x, ch)

                    tw = max_over_ranks(timed_steps(tstep, 5, 2, sync, dist.barrier), dev) / 5
                except _lib.HydraError:
                    continue
                tuning[f"{a}/{ch >> 20}MiB"] = round(tw * 1e3, 4)
                if best is None or tw < best[0]:
                    best = (tw, a, ch)
            chosen, chunk = (best[1], best[2]) if best is not None else ("direct", 0)
        if chosen not in full_ok:
            full_ok[chosen] = full_exact(chosen, chunk)
            if not full_ok[chosen]:  # never time a schedule that missed the reference bits
                chosen, chunk = "direct", 0
        ms, lat_ms = measure(chosen, chunk)
        phases = {}

        def profile_step(name, a, t, ch, esize, **kw):
            """One untimed, profiled allreduce after the timed region (the executor's own
            timing events on its comm and compute streams): the line's per-phase evidence."""
            if a in _lib.PEER_ALGOS:
                phases[name] = "n/a: one peer-access kernel (no separate link / fold phases)"
                return
            err = None
            try:
                comm.profile(True)
                try:
                    run(a, t, ch, **kw)
                    sync()
                    ph = comm.phases()
                finally:
                    comm.profile(False)
                phases[name] = dict(phase_report(ph, world, t.numel(), esize), algo=a,
                                    chunk_bytes=ch)
            except HydraError as e:
                err = str(e)
            if any_rank_failed(err):
                phases[name] = f"n/a: {err or 'another rank failed'}"

        def any_rank_failed(err):
            return max_over_ranks(1.0 if err else 0.0, dev) > 0

        profile_step("config4", chosen, x, chunk, 4)
        # 4) context: the other algorithms on the same bucket (fewer steps)
        others = {}
        c5 = None

        def _result(ms_, lat_, others_, c5_):
            return _bench_result(n, world, args, chosen, chunk, tuning, parity, full_ok, ms_,
                                 lat_, dict(others_), c5_, comm_seen, cpu_base, phases,
                                 dict(peer_leg), gate=gate)

        # the reference's own ring on this host's cores (bench.py's baseline leg: rank 0 only,
        # outside every timed region; the other ranks wait at the barrier)
        if cpu_baseline is not None:
            if rank == 0:
                try:
                    cpu_base = cpu_baseline(world, n)
                except Exception as e:  # a reported baseline, never the product
                    cpu_base = {"value": None, "error": str(e)}
            dist.barrier()

        state["result"] = lambda: _result(ms, lat_ms, others, c5)
        stall = float(getattr(args, "stall_context_s", 0.0) or 0.0)
        if stall > 0:  # rehearsal hook (bench.py --stall-context-s): a context phase hangs
            time.sleep(stall)
        # Everything after the headline is context: every wait is bounded (past
        # `context_timeout_s` the RCCL communicator is aborted and the rest of the legs fail
        # fast on it), an error is recorded in the line instead of failing the run, and every
        # rank runs the same collectives whatever happened locally, so one rank's failure
        # cannot strand the others in a barrier.
        ctx_timeout_ms = int(float(getattr(args, "context_timeout_s", 60.0)) * 1000)

        def bounded_wait():
            comm.wait(ctx_timeout_ms)

        def any_rank(err):
            """Collective: did any rank fail?  (err: this rank's error message or None)"""
            return max_over_ranks(1.0 if err else 0.0, dev) > 0

        def context_leg(step, k, warm=3, wait=bounded_wait):
            """ms per call of `step` over k timed calls after `warm` untimed ones, max over
            ranks; or 'n/a: <why>' on every rank if any rank failed."""
            err, t0, t1 = None, 0.0, 0.0
            try:
                for _ in range(warm):
                    step()
                wait()
            except HydraError as e:
                err = str(e)
            if any_rank(err):  # (also the barrier before the timed calls)
                return f"n/a: {err or 'another rank failed'}"
            try:
                t0 = time.perf_counter()
                for _ in range(k):
                    step()
                wait()
                t1 = time.perf_counter()
            except HydraError as e:
                err = str(e)
            failed = any_rank(err)
            wall = max_over_ranks(t1 - t0, dev)
            return f"n/a: {err or 'another rank failed'}" if failed else round(wall / k * 1e3, 4)

        # parity of the schedules the headline does not use
        def check_parity(name, call, expect, wait=bounded_wait):
            err, ok = None, False
            try:
                t = torch.from_numpy(xs[rank].copy()).to(dev)
                call(t)
                wait()
                ok = expect is None or bool(np.array_equal(t.cpu().numpy().view(np.uint32),
                                                           expect.view(np.uint32)))
            except HydraError as e:
                err = str(e)
            if any_rank(err):
                parity[name] = f"n/a: {err or 'another rank failed'}"
                return
            parity[name] = ("bit-exact" if max_over_ranks(0.0 if ok else 1.0, dev) == 0.0
                            else "MISMATCH")

        # --extra-legs: the schedules outside north_star's path (old-style rings, BCUBE,
        # halving-doubling, gloo::reduce to a root) -- parity and timings; off by default
        if extra_legs:
            check_parity("ring_old", lambda t: comm.allreduce_(t, algo="ring_old"),
                         expected_old_ring_f32(xs, rank))
            check_parity("ring_chunked", lambda t: comm.allreduce_(t, algo="ring_chunked"),
                         expected_chunked_ring_f32(xs))
            check_parity("bcube", lambda t: comm.allreduce_(t, algo="bcube"),
                         expected_bcube_f32(xs))
            # gloo::reduce to the last rank (hydra_reduce_root): only the root's bucket is defined
            check_parity("reduce_root", lambda t: comm.reduce_(t, world - 1),
                         expected_reduce_f32(xs) if rank == world - 1 else None)
        k = max(5, args.steps // 4)
        # context: RCCL's own allreduce and its own reduce-scatter + all-gather
        legs = ("ring", "direct", "a2a", "rccl", "rccl_rs_ag")
        if extra_legs:
            legs += ("ring_old", "ring_chunked", "bcube", "halving_doubling")
        for a in legs:
            if a == chosen:
                continue

            def ostep(a=a):
                run(a, x)

            others[a] = context_leg(ostep, k)

        if extra_legs:
            def rstep():
                comm.reduce_(x, 0)

            # gloo::reduce of the same bucket to rank 0 (context: no all-gather half)
            others["reduce_root0"] = context_leg(rstep, k)

        # 5) BASELINE config 5: bf16 bucket of 256 Mi elements, fp32 accumulation
        c5_ref = {}  # its gated DIRECT bucket, for the peer leg's config-5 schedule (7)
        if not getattr(args, "no_config5", False):
            n5 = int(getattr(args, "config5_elements", 256 << 20))
            # fold-order-sensitive bf16 values (+-2^k pivots that cancel: the one bf16 rounding
            # after the fp32 fold does not hide the order), generated on the device
            xb = synth.fill_at(synth.stress_cancel_at, world, rank, n5, dev,
                               torch.bfloat16).view(torch.int16)

            c5_algo = chosen if chosen in ("direct", "a2a") else "direct"

            def bstep():
                run(c5_algo, xb, chunk if c5_algo == "direct" else 0,
                    dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)

            k5 = max(5, args.steps // 10)
            # full-size check first: every rank's bucket equals the reference ring's fp32 fold
            # of the widened values, rounded once, on >= 1 Mi sampled indices, and the buckets
            # agree across ranks (sha256); the timed steps then keep folding in place
            err, g5 = None, None
            try:
                bstep()
                bounded_wait()
            except HydraError as e:
                err = str(e)
            if any_rank(err):
                c5 = {"elements": n5, "algo": c5_algo, "error": err or "another rank failed"}
            else:
                g5 = _full_size_gate(xb, world, n5, synth.stress_cancel_at, 2, dev)
                full_ok["config5_bf16_acc32"] = g5["ok"]
                if g5["ok"]:  # the gated bucket: the peer leg's config-5 schedule must equal it
                    c5_ref.update(n5=n5, ref=xb.clone(), k5=k5)
                r5 = context_leg(bstep, k5, warm=2)
                if not isinstance(r5, str):
                    profile_step("config5", c5_algo, xb, chunk if c5_algo == "direct" else 0, 2,
                                 dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
                if isinstance(r5, str):
                    c5 = {"elements": n5, "algo": c5_algo, "error": r5}
                else:
                    b_alg = 2.0 * n5 / (r5 * 1e-3) / 1e9
                    c5 = {"elements": n5, "dtype": "bf16 (fp32 accumulate, one rounding)",
                          "algo": c5_algo, "ms": r5, "algbw_GBps": round(b_alg, 2),
                          "busbw_GBps": round(b_alg * 2 * (world - 1) / world, 2),
                          "full_size_gate": g5}
                    c5_ref["rccl_ms"] = r5
            state["result"] = lambda: _result(ms, lat_ms, others, c5)
            del xb
        # 6) two rails (bew_allreduce_a, calculateElements_AA, DIRECT on each): the only leg in
        #    which two RCCL communicators run at once (pipeallreduce-a.cc:32-50's two threads).
        #    Last, and every wait bounded: a stall between the communicators aborts both (and
        #    ends this leg on every rank, each by its own timeout) instead of wedging the run.
        def rails_wait():  # past the bound BOTH rails are aborted
            try:
                comm.wait(ctx_timeout_ms)
            except HydraError:
                try:
                    rail2.wait(1)
                except HydraError:
                    pass
                raise

        e1, _ = split_elements(0, world, pn)
        exp2 = np.concatenate([expected_fold_f32([v[:e1] for v in xs]) if e1 else
                               np.empty(0, np.float32),
                               expected_fold_f32([v[e1:] for v in xs]) if e1 < pn else
                               np.empty(0, np.float32)])
        check_parity("apipe", lambda t: comm.apipe_allreduce_(rail2, t, algo="direct"), exp2,
                     wait=rails_wait)
        others["apipe_direct"] = (
            parity["apipe"] if parity["apipe"].startswith("n/a") else
            context_leg(lambda: comm.apipe_allreduce_(rail2, x, algo="direct"), k,
                        wait=rails_wait))
        state["result"] = lambda: _result(ms, lat_ms, others, c5)

        # 7) the reduce-on-read schedule (precedent cuda_collectives_native.h:
        #    63-120): ONE gfx950 kernel per allreduce reads the peers' IPC-mapped blocks over
        #    xGMI and folds them in the reference order.  On by default when every peer GPU is
        #    reached over xGMI with peer access; last, so every field above is already measured.
        #    Its barriers are bounded on the device (a peer that never arrives ends the kernel
        #    with an error word, hydra_peer_error) and every step's outcome is agreed over the
        #    ranks: a failure becomes an error entry of this leg, never a failed line.
        peer_leg.update(_peer_eligibility(args, comm_seen, world, dev))
        if shared_cap:
            peer_leg["shared_gpu_workgroup_cap"] = shared_cap
        if peer_leg["enabled"]:
            pr = _peer_leg(make_peer, pg, run, measure, sync, dev, rank, world, xs, exp, x, x0,
                           ref, gate, tp, peer_leg, c5_ref)
            c5_ref.clear()
            peer_leg["headline_ms"] = round(ms, 4)
            # promoted only when bit-exact with this run's DIRECT bucket at full size on the
            # order-sensitive data (the gate) and faster
            peer_leg["promoted"] = bool(pr is not None and peer_leg.get("full_size_exact")
                                        and pr[2] < ms)
            if peer_leg["promoted"]:  # the new headline: its own phases and parity entries
                others[chosen] = round(ms, 4)
                phases["config4_demoted_" + chosen] = phases.get("config4")
                chosen, chunk, ms, lat_ms = pr
                full_ok[chosen] = True
                phases["config4"] = peer_leg.get("phases")
                parity.update(peer_leg.get("parity_fold_order_1M", {}))
        state["result"] = lambda: _result(ms, lat_ms, others, c5)
    finally:
        errs = []
        for closer in ((pg["peer"].close if pg["peer"] is not None else None), comm.close,
                       rail2.close):
            if closer is None:
                continue
            try:
                closer()
            except HydraError as e:  # a teardown fault fails the run, after every close ran
                errs.append(e)
        dog.cancel()  # (after the closes: a hung communicator teardown is still caught)
        if errs:
            raise errs[0]
    return _result(ms, lat_ms, others, c5)


def _full_size_gate(t, world, n, gen, esize, dev) -> dict:
    """The full-size gate on this run's DIRECT bucket t (collective): t at >= 1 Mi sampled
    indices equals the reference fold (expected_fold_at) on every rank, and every rank's bucket
    has the same sha256.  Returns {"ok": ..., evidence}."""
    import hashlib

    import torch
    import torch.distributed as dist

    idx = sample_indices(n)
    want = expected_fold_at(world, n, idx, gen, esize=esize)
    it = torch.from_numpy(idx).to(t.device)
    if esize == 4:
        got = t.view(torch.int32)[it].cpu().numpy().view(np.uint32)
        ok = bool(np.array_equal(got, want.view(np.uint32)))
    else:
        got = t.view(torch.int16)[it].cpu().numpy().view(np.uint16)
        ok = bool(np.array_equal(got, want))
    digest = hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()
    digests = [None] * world
    dist.all_gather_object(digests, digest)
    agree = len(set(digests)) == 1
    sampled_ok = max_over_ranks(0.0 if ok else 1.0, dev) == 0.0
    return {"ok": bool(sampled_ok and agree), "data": getattr(gen, "__name__", str(gen)),
            "schedule": "direct", "sampled_indices": int(idx.size),
            "sampled_equal_reference_fold": sampled_ok, "sha256_equal_across_ranks": agree,
            "sha256": digest[:16],
            "rule": "every other schedule (and the peer leg) must equal this bucket bit for bit "
                    "on every rank to be timed or promoted"}


def _peer_eligibility(args, comm_seen, world, dev) -> dict:
    """Whether the peer leg runs on this node, agreed over the ranks: --peer on / off, or (auto)
    every other rank's GPU reached from this one over xGMI with peer access
    (rccl_comm.links_from_device: hydra_device_link)."""
    mode = _peer_mode(args)
    if mode == "off":
        return {"enabled": False, "mode": mode, "reason": "disabled (--peer off)"}
    if mode == "on":
        return {"enabled": True, "mode": mode, "reason": "forced (--peer on)"}
    import torch.distributed as dist

    links = comm_seen.get("links_from_device")
    # the GPUs the other ranks run on (a rank's device index need not equal its rank: a
    # CUDA_VISIBLE_DEVICES offset, a subset of the node's GPUs)
    devs = [None] * world
    dist.all_gather_object(devs, getattr(dev, "index", None))
    others = {d for i, d in enumerate(devs) if d is not None and d != getattr(dev, "index", None)}
    reason = None
    if world < 2:
        reason = "one rank: no peer to read from"
    elif not isinstance(links, list) or getattr(dev, "type", "") != "cuda":
        reason = "no GPU peer links visible to this process"
    else:
        mine = [lk for lk in links if lk.get("peer", -1) in others]
        if len(others) < world - 1 or len(mine) < world - 1:
            reason = (f"this process sees {len(links) + 1} GPU(s) for {world} ranks (ranks share "
                      "a GPU: no xGMI between them)")
        elif not all(lk.get("link") == "xgmi" and lk.get("peer_access") for lk in mine):
            reason = "not every peer GPU is reached over xGMI with peer access: " + \
                     ", ".join(f"{lk.get('peer')}:{lk.get('link')}/"
                               f"{'peer' if lk.get('peer_access') else 'no-peer'}" for lk in mine)
    bad = max_over_ranks(1.0 if reason else 0.0, dev) > 0
    if not bad:
        return {"enabled": True, "mode": mode,
                "reason": "every peer GPU over xGMI with peer access (hydra_device_link)"}
    return {"enabled": False, "mode": mode,
            "reason": f"skipped: {reason or 'another rank has no xGMI peer access'}"}


def _peer_leg(make_peer, pg, run, measure, sync, dev, rank, world, xs, exp, x, x0, ref, gate, tp,
              leg, c5_ref=None):
    """The peer leg's steps, each agreed over the ranks before the next: set up the IPC group,
    register the two buckets, parity of both schedules on the fold-order stress bucket, exactness
    at full size, a workgroup-count autotune, the timed region (bench.py's contract: exactly
    `steps` allreduces, barrier + sync on both sides, max over ranks) and one event-timed call as
    its phase entry.  Fills `leg`; returns (algo, workgroups, ms, latency) when the schedule is
    bit-exact and faster than the RCCL headline (the caller promotes it), else None."""
    import torch
    import torch.distributed as dist

    def agreed(err):
        return max_over_ranks(1.0 if err else 0.0, dev) == 0.0

    def peer_ok():
        p = pg["peer"]
        return max_over_ranks(float(p.error()) if p is not None else 1.0, dev) == 0.0

    failed = []  # inside a timed loop: a local error is recorded and the rank's later calls are
    # skipped, so every rank still issues the same collectives (barriers, max over ranks)

    def guarded(a, t, ch=0, **kw):
        if failed:
            return
        try:
            run(a, t, ch, **kw)
        except Exception as e:
            failed.append(str(e))

    err = None
    try:
        pg["peer"] = make_peer()  # collective; fails on every rank together
    except Exception as e:  # (any failure: recorded, ranks stay in step)
        err = str(e)
    if not agreed(err):
        pg["peer"] = None
        leg["error"] = f"setup: {err or 'another rank failed'}"
        return None
    try:
        for t in (tp, x):
            try:
                pg["peer"].register(t)
            except Exception as e:
                err = str(e)
            if not agreed(err):
                leg["error"] = f"register: {err or 'another rank failed'}"
                return None
        par = {}
        for a in ("peer2", "peer2w", "peer1"):
            ok = False
            try:
                tp.copy_(torch.from_numpy(xs[rank]))
                run(a, tp)
                sync()
                ok = bool(np.array_equal(tp.cpu().numpy().view(np.uint32), exp.view(np.uint32)))
            except Exception as e:
                err = str(e)
            if not agreed(err) or not peer_ok():
                par[a] = f"n/a: {err or 'a barrier expired or another rank failed'}"
                err = None
                continue
            par[a] = "bit-exact" if max_over_ranks(0.0 if ok else 1.0, dev) == 0.0 else "MISMATCH"
        leg["parity_fold_order_1M"] = par
        # the two-shot schedules (pull: peer2; push: peer2w) are the candidates for config 4's
        # bucket; only those that reproduced the reference bits go on
        algos = [a for a in ("peer2w", "peer2") if par.get(a) == "bit-exact"]
        if not algos:
            leg["error"] = "no two-shot schedule reproduced the reference bits; not timed"
            return None
        # the full-size gate: this run's DIRECT bucket on the order-sensitive data (_full_size_gate
        # pinned it to the reference fold), bit for bit, on every rank -- per schedule
        exact = {}
        for a in algos:
            good = False
            try:
                x.copy_(x0)
                run(a, x)
                sync()
                good = bool(torch.equal(x.view(torch.int32), ref.view(torch.int32)))
            except Exception as e:
                err = str(e)
            if not agreed(err) or not peer_ok():
                leg["error"] = f"full size: {err or 'a barrier expired or another rank failed'}"
                return None
            exact[a] = bool(gate["ok"]) and max_over_ranks(0.0 if good else 1.0, dev) == 0.0
        leg["full_size_exact_by_algo"] = exact
        algos = [a for a in algos if exact[a]]
        leg["full_size_exact"] = bool(algos)
        leg["full_size_gate"] = "equal to this run's DIRECT bucket (synth.stress_at), every rank"
        if not algos:
            return None
        tune = {}
        # 0: derived from the bucket (one per slab, <= 256, one per CU).  With a GPU per rank,
        # 512 too: two per CU, still all resident at the fold's register count (peer_allreduce.cpp),
        # twice the remote loads in flight for xGMI's longer read latency.  Ranks sharing one GPU
        # (the rehearsal) are capped at 512 / world by run(), so 512 is not a candidate there.
        cands = (0, 128, 64) if leg.get("shared_gpu_workgroup_cap") else (0, 512, 128, 64)
        for a in algos:
            for wg in cands:
                tw = None
                try:
                    def tstep(a=a, wg=wg):
                        guarded(a, x, wg)

                    tw = max_over_ranks(timed_steps(tstep, 5, 2, sync, dist.barrier), dev) / 5
                except Exception as e:
                    err = str(e)
                err = err or (failed[0] if failed else None)
                if not agreed(err) or not peer_ok():
                    leg["error"] = f"autotune: {err or 'a barrier expired or another rank failed'}"
                    return None
                tune[f"{a}/{wg}wg"] = round(tw * 1e3, 4)
        leg["autotune_ms"] = tune
        best = min(tune, key=tune.get)
        algo, wg = best.split("/")[0], int(best.split("/")[1][:-2])
        try:
            ms_p, lat_p = measure(algo, wg, runner=guarded)
        except Exception as e:
            err = str(e)
        err = err or (failed[0] if failed else None)
        if not agreed(err) or not peer_ok():
            leg["error"] = f"timed region: {err or 'a barrier expired or another rank failed'}"
            return None
        leg.update(algo=algo, workgroups=wg, ms_per_step=round(ms_p, 4), latency_ms=lat_p)
        leg["phases"] = _peer_phases(run, sync, dev, x, wg, world, algo)
        if c5_ref and c5_ref.get("ref") is not None:  # config 5 through the same schedule
            leg["config5"] = _peer_config5(pg, run, guarded, failed, sync, dev, rank, world,
                                           algo, wg, c5_ref, agreed, peer_ok)
        return algo, wg, ms_p, lat_p
    finally:
        p, pg["peer"] = pg["peer"], None
        if p is not None:
            try:
                p.close()
            except Exception as e:  # a teardown failure is reported, after every rank closed
                leg.setdefault("error", f"teardown: {e}")


def _peer_config5(pg, run, guarded, failed, sync, dev, rank, world, algo, wg, c5, agreed,
                  peer_ok) -> dict:
    """BASELINE config 5 (bf16, fp32 accumulation) through the peer leg's schedule: a fresh
    bucket of the same stress_cancel_at values, registered, allreduced once and compared bit
    for bit with the config-5 leg's gated DIRECT bucket on every rank; only then timed (k5
    allreduces, barrier + sync on both sides, max over ranks).  Every step agreed over the
    ranks; a failure becomes this entry's error."""
    import torch
    import torch.distributed as dist

    from hydra_amd import synth

    n5, kw = c5["n5"], dict(dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    out = {"algo": algo, "workgroups": wg, "elements": n5,
           "gate": "equal to this run's config-5 DIRECT bucket (synth.stress_cancel_at), every rank"}
    err, t5 = None, None
    try:
        t5 = synth.fill_at(synth.stress_cancel_at, world, rank, n5, dev,
                           torch.bfloat16).view(torch.int16)
    except Exception as e:
        err = str(e)
    if not agreed(err):
        return dict(out, error=f"inputs: {err or 'another rank failed'}")
    try:
        pg["peer"].register(t5)  # collective
    except Exception as e:
        err = str(e)
    if not agreed(err):
        return dict(out, error=f"register: {err or 'another rank failed'}")
    good = False
    try:
        run(algo, t5, wg, **kw)
        sync()
        good = bool(torch.equal(t5, c5["ref"]))
    except Exception as e:
        err = str(e)
    if not agreed(err) or not peer_ok():
        return dict(out, error=f"full size: {err or 'a barrier expired or another rank failed'}")
    out["full_size_exact"] = max_over_ranks(0.0 if good else 1.0, dev) == 0.0
    if not out["full_size_exact"]:
        return out
    tw = None
    try:
        tw = max_over_ranks(timed_steps(lambda: guarded(algo, t5, wg, **kw), c5["k5"], 2, sync,
                                        dist.barrier), dev) / c5["k5"]
    except Exception as e:
        err = str(e)
    err = err or (failed[0] if failed else None)
    if not agreed(err) or not peer_ok():
        return dict(out, error=f"timed: {err or 'a barrier expired or another rank failed'}")
    b_alg = 2.0 * n5 / tw / 1e9
    out.update(ms=round(tw * 1e3, 4), algbw_GBps=round(b_alg, 2),
               busbw_GBps=round(b_alg * 2 * (world - 1) / world, 2), rccl_ms=c5.get("rccl_ms"))
    return out


def _peer_phases(run, sync, dev, x, wg, world, algo="peer2") -> dict:
    """One event-timed peer allreduce (untimed otherwise): the kernel IS both phases -- it reads
    the peers' blocks over xGMI (link) and folds them as they arrive (fold) -- so the entry gives
    the one kernel's time against both rooflines: per-rank link bytes 2(P-1)/P x n x E (the
    owner block's P-1 remote reads + the P-1 finished blocks pulled back, or pushed: peer2w)
    over P-1 links, and the fused sum's algorithmic HBM bytes (P-1)/P x n x 3E (SURVEY.md
    8(d))."""
    import torch

    n, esize = x.numel(), x.element_size()
    local, err = -1.0, None
    try:
        if getattr(dev, "type", "") == "cuda":
            s = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            sync()
            e0.record(s)
            run(algo, x, wg)
            e1.record(s)
            sync()
            local = e0.elapsed_time(e1)
        else:  # (the CPU rehearsal: wall time of one synchronous call)
            sync()
            t0 = time.perf_counter()
            run(algo, x, wg)
            sync()
            local = (time.perf_counter() - t0) * 1e3
    except Exception as e:  # every rank still reaches the collective below
        err = str(e)
    failed = max_over_ranks(1.0 if err else 0.0, dev) > 0
    ms = max_over_ranks(local, dev)
    if failed:
        return {"error": err or "another rank failed"}
    link_bytes = 2 * (world - 1) / world * n * esize
    fused = (world - 1) / world * n * 3 * esize
    links = max(1, world - 1)
    per_link = link_bytes / links / (ms * 1e-3) / 1e9 if ms > 0 else None
    kern = fused / (ms * 1e-3) / 1e9 if ms > 0 else None
    return {"calls": 1, "algo": algo, "kernel_ms": round(ms, 4), "link_ms": round(ms, 4),
            "fold_ms": round(ms, 4), "span_ms": round(ms, 4), "overlap_ms": round(ms, 4),
            "note": "one kernel: link reads and folds overlap completely (link = fold = span)",
            "link": {"algorithmic_bytes": int(link_bytes), "peers": links,
                     "per_link_GBps": _sig(per_link) if per_link else None,
                     "frac_of_link": _sig(per_link / XGMI_LINK_GBS) if per_link else None,
                     "link_peak_GBps": XGMI_LINK_GBS},
            "fold": {"fused_sum_bytes": int(fused),
                     "kernel_GBps": _sig(kern) if kern else None,
                     "frac_of_hbm": _sig(kern / HBM_PEAK_GBS) if kern else None,
                     "hbm_peak_GBps": HBM_PEAK_GBS}}


def _bench_result(n, world, args, chosen, chunk, tuning, parity, full_ok, ms, lat_ms, others,
                  c5, comm_seen=None, cpu_base=None, phases=None, peer_leg=None,
                  gate=None) -> dict:
    """The N>1 bench JSON line (bench_allreduce; also printed by its watchdog once the headline
    is measured)."""
    bucket = 4.0 * n
    algbw = bucket / (ms * 1e-3) / 1e9
    busbw = algbw * 2 * (world - 1) / world
    link = 153.0
    return {
        "metric": "chunk-sum GB/s (fp32) vs HBM peak; ring-allreduce GB/s at 1/2/4/8 GPU",
        "value": round(world * algbw, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"in-place allreduce of a {n}-element fp32 bucket per rank over "
                               "xGMI, reference ring block ownership and fold order, "
                               + ("ONE gfx950 kernel reading the peers' IPC-mapped blocks"
                                  if chosen.startswith("peer") else
                                  "RCCL p2p with the HIP sum fused per hop")
                               + " (BASELINE config 4)", "elements": n, "algo": chosen,
                   ("peer_workgroups" if chosen in _lib.PEER_ALGOS else "chunk_bytes"): chunk,
                   "autotune_ms": tuning,
                   "parallelism": f"dp{world}",
                   "scaling_note": "value = N x allreduce algbw of a fixed per-rank bucket "
                                   "(weak scaling, xGMI-bound); bench.py at N = 1 reports the "
                                   "HBM chunk-sum instead (BASELINE's metric names both), so "
                                   "the N = 1 value is not the base of an allreduce efficiency "
                                   "(DESIGN.md 7)"},
        "algbw_GBps": round(algbw, 2), "busbw_GBps": round(busbw, 2),
        "roofline": {"bound": "xgmi", "achieved": round(busbw, 2),
                     "peak": round(link * max(1, world - 1), 1), "unit": "GB/s",
                     "frac": round(busbw / (link * max(1, world - 1)), 4),
                     "traffic": int((world - 1) / world * n * 12),
                     "traffic_kind": "algorithmic, not measured: the fused-sum HBM bytes per "
                                     "rank per allreduce, (P-1)/P x n x 12 (SURVEY.md 8(d)); no "
                                     "PMC pass runs at N > 1",
                     "phases": (phases or {}).get("config4"),
                     "note": "busbw vs (P-1) xGMI links x 153 GB/s; a single ring is bound by "
                             "1 link (153 GB/s); phases = one profiled untimed allreduce after "
                             "the timed region (link = comm-stream busy time, fold = compute-"
                             "stream busy time)"},
        "latency_ms": lat_ms,
        "other_algos_ms": others,
        "other_algos_busbw_GBps": {a: round(bucket / (v * 1e-3) / 1e9 * 2 * (world - 1) / world, 2)
                                   for a, v in others.items()
                                   if isinstance(v, float) and a != "reduce_root0"},
        "config5_bf16": (dict(c5, phases=(phases or {}).get("config5"),
                              peer=(peer_leg or {}).get("config5"))
                         if isinstance(c5, dict) else c5),
        "parity": {"fold_order_1M": parity, "full_size_exact": full_ok,
                   "full_size_gate": gate},
        "rccl_comm": comm_seen,
        "cpu_baseline": cpu_base,
        "peer_leg": peer_leg or {"enabled": False, "reason": "not reached"},
    }
