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
