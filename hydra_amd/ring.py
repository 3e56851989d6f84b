"""Multi-GPU bucket allreduce (RCCL over xGMI + fused HIP reductions) -- Python face.

Mirrors gloo::allreduce(AllreduceOptions) with Algorithm::RING (gloo/gloo/allreduce.h:89-201,
allreduce.cc:99-422) for device-resident buckets, one process per GPU.  The schedule, the
kernels and the RCCL calls all live in libhydra_hip.so (hydra_amd/csrc/xgmi_*.{h,cpp}); this
module exchanges the RCCL unique id over torch.distributed and hands tensors over.
"""
from __future__ import annotations

import ctypes
import sys
import time

import numpy as np

from . import _lib
from ._lib import ALGOS, HydraError, OPS, check

_is_finalizing = sys.is_finalizing


def plan(algo: str, P: int, rank: int, n: int, esize: int, max_segment: int = 0,
         chunk_bytes: int = 0):
    """The op list rank `rank` executes, as a list of dicts, plus its scratch bytes."""
    L = _lib.lib()
    cnt, scr = ctypes.c_size_t(), ctypes.c_size_t()
    check(L.hydra_plan(ALGOS[algo], P, rank, n, esize, max_segment, chunk_bytes, None, 0,
                       ctypes.byref(cnt), ctypes.byref(scr)))
    arr = (_lib.PlanOp * max(1, cnt.value))()
    check(L.hydra_plan(ALGOS[algo], P, rank, n, esize, max_segment, chunk_bytes, arr, cnt.value,
                       ctypes.byref(cnt), ctypes.byref(scr)))
    ops = [{f: getattr(arr[i], f) for f, _ in _lib.PlanOp._fields_} for i in range(cnt.value)]
    return ops, scr.value


def plan_reduce(root: int, P: int, rank: int, n: int, esize: int, max_segment: int = 0,
                chunk_bytes: int = 0):
    """hydra_reduce_root's op list for `rank` (gloo::reduce to `root`), plus its scratch bytes."""
    L = _lib.lib()
    cnt, scr = ctypes.c_size_t(), ctypes.c_size_t()
    check(L.hydra_reduce_root_plan(root, P, rank, n, esize, max_segment, chunk_bytes, None, 0,
                                   ctypes.byref(cnt), ctypes.byref(scr)))
    arr = (_lib.PlanOp * max(1, cnt.value))()
    check(L.hydra_reduce_root_plan(root, P, rank, n, esize, max_segment, chunk_bytes, arr,
                                   cnt.value, ctypes.byref(cnt), ctypes.byref(scr)))
    ops = [{f: getattr(arr[i], f) for f, _ in _lib.PlanOp._fields_} for i in range(cnt.value)]
    return ops, scr.value


def simulate_reduce(bufs, root: int, op: str = "sum", dtype_code: int | None = None,
                    flags: int = 0, max_segment: int = 0, chunk_bytes: int = 0) -> None:
    """hydra_reduce_root for len(bufs) ranks on ONE GPU; bufs[root] ends with the reduction."""
    from .reduce import _torch_dtype_code

    P = len(bufs)
    code = dtype_code if dtype_code is not None else _torch_dtype_code(bufs[0])
    n = _count(bufs[0], code)
    for b in bufs:
        if _count(b, code) != n or not b.is_contiguous():
            raise HydraError(1, "simulate_reduce: buckets must be contiguous and equally sized")
    ptrs = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
    check(_lib.lib().hydra_reduce_root_simulate(root, OPS[op], code, flags, P, ptrs, n,
                                                max_segment, chunk_bytes))


def simulate(bufs, algo: str = "auto", op: str = "sum", dtype_code: int | None = None,
             flags: int = 0, max_segment: int = 0, chunk_bytes: int = 0) -> None:
    """Run all len(bufs) ranks' plans on ONE GPU (device tensors, modified in place)."""
    from .reduce import _torch_dtype_code

    P = len(bufs)
    code = dtype_code if dtype_code is not None else _torch_dtype_code(bufs[0])
    n = _count(bufs[0], code)
    for b in bufs:
        if _count(b, code) != n or not b.is_contiguous():
            raise HydraError(1, "simulate: buckets must be contiguous and equally sized")
    ptrs = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
    check(_lib.lib().hydra_allreduce_simulate(ALGOS[algo], OPS[op], code, flags, P, ptrs, n,
                                              max_segment, chunk_bytes))


def split_elements(table: int, P: int, n: int) -> tuple[int, int]:
    """calculateElements_AA (table 0) / _AG (1): (e1 for rail 1, e2 for rail 2)."""
    e1, e2 = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.lib().hydra_split_elements(table, P, n, ctypes.byref(e1), ctypes.byref(e2))
    return e1.value, e2.value


def simulate_apipe(bufs, table: int = 0, algo: str = "auto", op: str = "sum",
                   dtype_code: int | None = None, flags: int = 0, max_segment: int = 0,
                   chunk_bytes: int = 0) -> None:
    """hydra_apipe_allreduce on len(bufs) simulated ranks of one GPU (in place)."""
    from .reduce import _torch_dtype_code

    P = len(bufs)
    code = dtype_code if dtype_code is not None else _torch_dtype_code(bufs[0])
    n = _count(bufs[0], code)
    for b in bufs:
        if _count(b, code) != n or not b.is_contiguous():
            raise HydraError(1, "simulate_apipe: buckets must be contiguous and equally sized")
    ptrs = (ctypes.c_void_p * P)(*[b.data_ptr() for b in bufs])
    check(_lib.lib().hydra_apipe_allreduce_simulate(table, ALGOS[algo], OPS[op], code, flags, P,
                                                    ptrs, n, max_segment, chunk_bytes))


def _count(t, code: int) -> int:
    """elements of dtype `code` in tensor t (t may hold the bits in another dtype)."""
    if code not in _lib.ESIZE:
        raise HydraError(1, f"invalid dtype code {code}")
    nbytes = t.numel() * t.element_size()
    if nbytes % _lib.ESIZE[code]:
        raise HydraError(1, "tensor size is not a multiple of the element size")
    return nbytes // _lib.ESIZE[code]


def _rccl_unique_id() -> bytes:
    buf = np.zeros(_lib.UNIQUE_ID_BYTES, dtype=np.uint8)
    check(_lib.lib().hydra_comm_get_unique_id(buf.ctypes.data))
    return buf.tobytes()


def exchange_unique_id(rank: int, device=None, make_id=_rccl_unique_id) -> bytes:
    """Rank 0 creates the RCCL unique id; every rank gets it via torch.distributed broadcast
    (works on nccl -- device tensor -- and gloo -- host tensor -- process groups)."""
    import torch
    import torch.distributed as dist

    buf = np.zeros(_lib.UNIQUE_ID_BYTES, dtype=np.uint8)
    if rank == 0:
        buf[:] = np.frombuffer(make_id(), dtype=np.uint8)
    t = torch.from_numpy(buf)
    if dist.get_backend() == "nccl":
        t = t.to(device)
    dist.broadcast(t, 0)
    return bytes(t.cpu().numpy().tobytes())


class XgmiComm:
    """One RCCL communicator + comm/compute streams + scratch (hydra_comm_t)."""

    def __init__(self, rank: int, world: int, device_index: int, uid: bytes):
        h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(uid, _lib.UNIQUE_ID_BYTES)
        check(_lib.lib().hydra_comm_init(ctypes.byref(h), world, rank, idbuf, device_index))
        self._h = h
        self.rank, self.world = rank, world

    def info(self) -> dict:
        """What RCCL itself reports: ncclCommCount / ncclCommUserRank / ncclCommCuDevice."""
        cnt, r, d = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(_lib.lib().hydra_comm_info(self._h, ctypes.byref(cnt), ctypes.byref(r),
                                         ctypes.byref(d)))
        return {"nccl_comm_count": cnt.value, "nccl_user_rank": r.value, "nccl_device": d.value}

    def allreduce_(self, t, algo: str = "auto", op: str = "sum", dtype_code: int | None = None,
                   flags: int = 0, max_segment: int = 0, chunk_bytes: int = 0,
                   stream: int | None = None) -> None:
        """In-place allreduce of device tensor t on the current (or given) stream."""
        import torch

        from .reduce import _torch_dtype_code

        code = dtype_code if dtype_code is not None else _torch_dtype_code(t)
        if not t.is_contiguous():
            raise HydraError(1, "allreduce_: contiguous tensor required")
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        check(_lib.lib().hydra_allreduce(self._h, ALGOS[algo], OPS[op], code, flags,
                                         t.data_ptr(), _count(t, code), max_segment,
                                         chunk_bytes, s))

    def reduce_(self, t, root: int, op: str = "sum", dtype_code: int | None = None,
                flags: int = 0, max_segment: int = 0, chunk_bytes: int = 0,
                stream: int | None = None) -> None:
        """gloo::reduce of device tensor t to `root`, in place (only the root's t is defined)."""
        import torch

        from .reduce import _torch_dtype_code

        code = dtype_code if dtype_code is not None else _torch_dtype_code(t)
        if not t.is_contiguous():
            raise HydraError(1, "reduce_: contiguous tensor required")
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        check(_lib.lib().hydra_reduce_root(self._h, root, OPS[op], code, flags, t.data_ptr(),
                                           _count(t, code), max_segment, chunk_bytes, s))

    def apipe_allreduce_(self, rail2: "XgmiComm", t, table: int = 0, algo: str = "auto",
                         op: str = "sum", dtype_code: int | None = None, flags: int = 0,
                         max_segment: int = 0, chunk_bytes: int = 0,
                         stream: int | None = None) -> None:
        """bew_allreduce_a on device: split t per calculateElements (table 0 = _AA, 1 = _AG),
        [0, e1) on this communicator and [e1, n) on rail2, concurrently."""
        import torch

        from .reduce import _torch_dtype_code

        code = dtype_code if dtype_code is not None else _torch_dtype_code(t)
        if not t.is_contiguous():
            raise HydraError(1, "apipe_allreduce_: contiguous tensor required")
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        check(_lib.lib().hydra_apipe_allreduce(self._h, rail2._h, table, ALGOS[algo], OPS[op],
                                               code, flags, t.data_ptr(), _count(t, code),
                                               max_segment, chunk_bytes, s))

    def profile(self, enable: bool) -> None:
        """hydra_comm_profile: time every op of the following allreduces (measurement only)."""
        check(_lib.lib().hydra_comm_profile(self._h, 1 if enable else 0))

    def phases(self) -> dict:
        """hydra_comm_phases: per-phase totals of the allreduces since profile(True)."""
        ph = _lib.CommPhases()
        check(_lib.lib().hydra_comm_phases(self._h, ctypes.byref(ph)))
        return {f: getattr(ph, f) for f, _ in _lib.CommPhases._fields_ if f != "reserved"}

    def wait(self, timeout_ms: int, stream: int | None = None) -> None:
        """Block until the work enqueued on `stream` (default: current) is done; past timeout_ms
        the communicator is aborted and HydraError(ERR_TIMEOUT, "Timed out waiting ...") is
        raised -- the reference's per-op timeout (tcp/unbound_buffer.cc:60-85)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        check(_lib.lib().hydra_comm_wait(self._h, s, int(timeout_ms)))

    def run_plan_(self, ops, t, scratch_bytes: int, op: str = "sum",
                  dtype_code: int | None = None, flags: int = 0,
                  stream: int | None = None) -> None:
        """Executor test hook (hydra_comm_run_plan): run op dicts (as ring.plan returns) on t."""
        import torch

        from .reduce import _torch_dtype_code

        code = dtype_code if dtype_code is not None else _torch_dtype_code(t)
        arr = (_lib.PlanOp * max(1, len(ops)))()
        for i, o in enumerate(ops):
            for f, _ in _lib.PlanOp._fields_:
                setattr(arr[i], f, int(o[f]))
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        check(_lib.lib().hydra_comm_run_plan(self._h, arr, len(ops), OPS[op], code, flags,
                                             t.data_ptr(), t.numel() * t.element_size(),
                                             scratch_bytes, s))

    def close(self) -> None:
        """Destroy the communicator; raises if a teardown step reports a device error."""
        if self._h:
            h, self._h = self._h, ctypes.c_void_p()
            check(_lib.lib().hydra_comm_destroy(h))

    def __del__(self):
        # never call into HIP/RCCL while the interpreter is finalizing (the runtime may be gone);
        # `sys` is bound at import time: an import here fails during shutdown
        if _is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


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

    from . import synth

    rank, world = dist.get_rank(), dist.get_world_size()
    # a hung collective must fail the run, not stall it: hard exit (status 3) after `watchdog_s`,
    # printing the measured headline flagged when there is one (hydra_amd/watchdog.py)
    import os

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
            from .peer import PeerComm

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
        # 2) exactness at full size: integer-valued inputs whose sums are exact in fp32
        j = np.arange(n, dtype=np.int64)
        x0 = torch.from_numpy(((j % 1024) * (rank + 1)).astype(np.float32)).to(dev)
        x = x0.clone()
        full_exp = torch.from_numpy(((j % 1024) * (world * (world + 1) // 2))
                                    .astype(np.float32)).to(dev)
        def full_exact(a, ch=0):
            x.copy_(x0)
            run(a, x, ch)
            sync()
            good = bool(torch.equal(x, full_exp))
            return max_over_ranks(0.0 if good else 1.0, dev) == 0.0

        full_ok = {"direct": full_exact("direct")}
        def measure(a, ch):
            """The timed region (exactly `steps` allreduces, barrier + sync on both sides, max
            over ranks) and the per-iteration latency as the reference's benchmark reports it
            (runner.cc:693-697: wall time around each run(), p50/p99), outside the region."""
            def step():
                run(a, x, ch)

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
                {}, None, comm_seen)
        # 3) pick the algorithm: "auto" = the fastest bit-exact RCCL schedule on this node
        #    (DIRECT / A2A / RING), chosen on a few untimed steps; the peer-access kernel is
        #    checked and timed last (7) and replaces this headline only if it is faster
        chosen, chunk = algo, 0
        stall = float(os.environ.get("HYDRA_BENCH_STALL_AUTOTUNE", "0"))
        if stall > 0:  # test hook: an autotune candidate that hangs
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
                                 dict(peer_leg))

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
        stall = float(os.environ.get("HYDRA_BENCH_STALL_CONTEXT", "0"))
        if stall > 0:  # test hook: a context phase that hangs (tests the watchdog's report)
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
        if not getattr(args, "no_config5", False):
            n5 = int(getattr(args, "config5_elements", 256 << 20))  # a multiple of 1 Mi
            base = np.arange(1 << 20, dtype=np.int64) % 7 - 3
            xb = torch.from_numpy(synth.bf16_bits(base.astype(np.float32)).view(np.int16)) \
                .to(dev).repeat(n5 >> 20)

            c5_algo = chosen if chosen in ("direct", "a2a") else "direct"

            def bstep():
                run(c5_algo, xb, chunk if c5_algo == "direct" else 0,
                    dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)

            k5 = max(5, args.steps // 10)
            # full-size check first: every rank holds the same small integers, so one
            # allreduce must give exactly world x base in bf16 (|sum| <= 3P: exact in fp32 and
            # in bf16); the timed steps then keep folding in place
            err, good = None, False
            try:
                want = torch.from_numpy(synth.bf16_bits((base * world).astype(np.float32))
                                        .view(np.int16)).to(dev).repeat(n5 >> 20)
                bstep()
                bounded_wait()
                good = bool(torch.equal(xb, want))
                del want
            except HydraError as e:
                err = str(e)
            if any_rank(err):
                c5 = {"elements": n5, "algo": c5_algo, "error": err or "another rank failed"}
            else:
                full_ok["config5_bf16_acc32"] = max_over_ranks(0.0 if good else 1.0, dev) == 0.0
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
                          "busbw_GBps": round(b_alg * 2 * (world - 1) / world, 2)}
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
                           full_exp, tp, peer_leg)
            peer_leg["headline_ms"] = round(ms, 4)
            peer_leg["promoted"] = bool(pr is not None and pr[2] < ms)
            if peer_leg["promoted"]:  # bit-exact at full size and faster: the new headline
                others[chosen] = round(ms, 4)
                chosen, chunk, ms, lat_ms = pr
                full_ok[chosen] = True
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


def _peer_eligibility(args, comm_seen, world, dev) -> dict:
    """Whether the peer leg runs on this node, agreed over the ranks: --peer on / off, or (auto)
    every other rank's GPU reached from this one over xGMI with peer access
    (rccl_comm.links_from_device: hydra_device_link)."""
    mode = _peer_mode(args)
    if mode == "off":
        return {"enabled": False, "mode": mode, "reason": "disabled (--peer off)"}
    if mode == "on":
        return {"enabled": True, "mode": mode, "reason": "forced (--peer on)"}
    links = comm_seen.get("links_from_device")
    reason = None
    if world < 2:
        reason = "one rank: no peer to read from"
    elif not isinstance(links, list) or getattr(dev, "type", "") != "cuda":
        reason = "no GPU peer links visible to this process"
    else:
        mine = [lk for lk in links if lk.get("peer", -1) < world]
        if len(mine) < world - 1:
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


def _peer_leg(make_peer, pg, run, measure, sync, dev, rank, world, xs, exp, x, x0, full_exp, tp,
              leg):
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
        for a in ("peer2", "peer1"):
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
        if par.get("peer2") != "bit-exact":
            leg["error"] = "peer2 did not reproduce the reference bits; not timed"
            return None
        good = False
        try:
            x.copy_(x0)
            run("peer2", x)
            sync()
            good = bool(torch.equal(x, full_exp))
        except Exception as e:
            err = str(e)
        if not agreed(err) or not peer_ok():
            leg["error"] = f"full size: {err or 'a barrier expired or another rank failed'}"
            return None
        leg["full_size_exact"] = max_over_ranks(0.0 if good else 1.0, dev) == 0.0
        if not leg["full_size_exact"]:
            return None
        tune = {}
        # 0: derived from the bucket (one per slab, <= 256, one per CU).  With a GPU per rank,
        # 512 too: two per CU, still all resident at the fold's register count (peer_allreduce.cpp),
        # twice the remote loads in flight for xGMI's longer read latency.  Ranks sharing one GPU
        # (the rehearsal) are capped at 512 / world by run(), so 512 is not a candidate there.
        cands = (0, 128, 64) if leg.get("shared_gpu_workgroup_cap") else (0, 512, 128, 64)
        for wg in cands:
            tw = None
            try:
                def tstep(wg=wg):
                    run("peer2", x, wg)

                tw = max_over_ranks(timed_steps(tstep, 5, 2, sync, dist.barrier), dev) / 5
            except Exception as e:
                err = str(e)
            if not agreed(err) or not peer_ok():
                leg["error"] = f"autotune: {err or 'a barrier expired or another rank failed'}"
                return None
            tune[f"peer2/{wg}wg"] = round(tw * 1e3, 4)
        leg["autotune_ms"] = tune
        wg = int(min(tune, key=tune.get).split("/")[1][:-2])
        try:
            ms_p, lat_p = measure("peer2", wg)
        except Exception as e:
            err = str(e)
        if not agreed(err) or not peer_ok():
            leg["error"] = f"timed region: {err or 'a barrier expired or another rank failed'}"
            return None
        leg.update(algo="peer2", workgroups=wg, ms_per_step=round(ms_p, 4), latency_ms=lat_p)
        leg["phases"] = _peer_phases(run, sync, dev, x, wg, world)
        return "peer2", wg, ms_p, lat_p
    finally:
        p, pg["peer"] = pg["peer"], None
        if p is not None:
            try:
                p.close()
            except Exception as e:  # a teardown failure is reported, after every rank closed
                leg.setdefault("error", f"teardown: {e}")


def _peer_phases(run, sync, dev, x, wg, world) -> dict:
    """One event-timed peer allreduce (untimed otherwise): the kernel IS both phases -- it reads
    the peers' blocks over xGMI (link) and folds them as they arrive (fold) -- so the entry gives
    the one kernel's time against both rooflines: per-rank link bytes 2(P-1)/P x n x E (the
    owner block's P-1 remote reads + the P-1 finished blocks pulled back) over P-1 links, and
    the fused sum's algorithmic HBM bytes (P-1)/P x n x 3E."""
    import torch

    n, esize = x.numel(), x.element_size()
    local, err = -1.0, None
    try:
        if getattr(dev, "type", "") == "cuda":
            s = torch.cuda.current_stream(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            sync()
            e0.record(s)
            run("peer2", x, wg)
            e1.record(s)
            sync()
            local = e0.elapsed_time(e1)
        else:  # (the CPU rehearsal: wall time of one synchronous call)
            sync()
            t0 = time.perf_counter()
            run("peer2", x, wg)
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
    return {"calls": 1, "kernel_ms": round(ms, 4), "link_ms": round(ms, 4),
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
                  c5, comm_seen=None, cpu_base=None, phases=None, peer_leg=None) -> dict:
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
        "config5_bf16": (dict(c5, phases=(phases or {}).get("config5"))
                         if isinstance(c5, dict) else c5),
        "parity": {"fold_order_1M": parity, "full_size_exact": full_ok},
        "rccl_comm": comm_seen,
        "cpu_baseline": cpu_base,
        "peer_leg": peer_leg or {"enabled": False, "reason": "not reached"},
    }
