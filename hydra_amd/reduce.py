"""Python face of the reduction plug-point (the Gloo ``ReductionFunction`` / ``Func`` surface).

Reference interfaces mirrored:
  * ``gloo::sum<T>(void* c, const void* a, const void* b, size_t n)``  gloo/gloo/math.h:15-23
    and product/max/min (math.h:30-73): element-wise, c may alias a (the ring's in-place form)
  * ``ReductionFunction<T>{type, fn}`` with ``.sum/.product/.min/.max`` gloo/gloo/algorithm.h:49-96
  * ``AllreduceOptions::Func = void(void*, const void*, const void*, size_t)`` allreduce.h:36

Device tensors go through ``hydra_reduce`` on torch's current stream; host (numpy) buffers go
through ``hydra_reduce_host`` (synchronous, staged).  Every call lands in libhydra_hip.so.
"""
from __future__ import annotations

import ctypes
import sys
import threading

import numpy as np

from . import _lib
from ._lib import HydraError, OPS, check

_is_finalizing = sys.is_finalizing

_TORCH_DTYPES = None


def _torch_dtype_code(t) -> int:
    global _TORCH_DTYPES
    import torch

    if _TORCH_DTYPES is None:
        _TORCH_DTYPES = {
            torch.int8: _lib.INT8, torch.uint8: _lib.UINT8, torch.int32: _lib.INT32,
            torch.int64: _lib.INT64, torch.float32: _lib.FLOAT32, torch.float64: _lib.FLOAT64,
            torch.float16: _lib.FLOAT16, torch.bfloat16: _lib.BFLOAT16,
        }
        for name, code in (("uint32", _lib.UINT32), ("uint64", _lib.UINT64)):
            if hasattr(torch, name):
                _TORCH_DTYPES[getattr(torch, name)] = code
    try:
        return _TORCH_DTYPES[t.dtype]
    except KeyError:
        raise HydraError(1, f"unsupported dtype {t.dtype}") from None


_NP_DTYPES = {np.dtype(np.int8): _lib.INT8, np.dtype(np.uint8): _lib.UINT8,
              np.dtype(np.int32): _lib.INT32, np.dtype(np.uint32): _lib.UINT32,
              np.dtype(np.int64): _lib.INT64, np.dtype(np.uint64): _lib.UINT64,
              np.dtype(np.float32): _lib.FLOAT32, np.dtype(np.float64): _lib.FLOAT64,
              np.dtype(np.float16): _lib.FLOAT16}


def _stream_ptr(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream


def reduce_(op: str, c, a, b, n: int | None = None, dtype_code: int | None = None,
            stream: int | None = None) -> None:
    """c[:n] = op(a[:n], b[:n]) on device tensors (asynchronous on the current stream).
    dtype_code overrides the tensor dtype (e.g. BFLOAT16/FLOAT16 data held in int16 tensors)."""
    if not (c.is_cuda and a.is_cuda and b.is_cuda):
        raise HydraError(1, "hydra reduce: device tensors required (use reduce_host for host)")
    code = dtype_code if dtype_code is not None else _torch_dtype_code(c)
    es = _lib.ESIZE[code]
    cap = min(t.numel() * t.element_size() for t in (c, a, b)) // es  # elements of `code`
    if n is None:
        n = (c.numel() * c.element_size()) // es
    if n > cap:
        raise HydraError(1, "n exceeds a tensor's length")
    if not (c.is_contiguous() and a.is_contiguous() and b.is_contiguous()):
        raise HydraError(1, "contiguous tensors required")
    s = stream if stream is not None else _stream_ptr(c.device)
    check(_lib.lib().hydra_reduce(OPS[op], code, c.data_ptr(), a.data_ptr(), b.data_ptr(), n, s))


def sum_(c, a, b, n: int | None = None, **kw) -> None:
    """gloo::sum<T>(c, a, b, n) on the GPU."""
    reduce_("sum", c, a, b, n, **kw)


def acc_bf16_f32_(acc, b_bf16, stream: int | None = None) -> None:
    """acc(fp32) += float(b_bf16): the fp32-accumulate form of a bf16 bucket (config 5)."""
    if b_bf16.numel() * b_bf16.element_size() < 2 * acc.numel() or acc.dtype.itemsize != 4:
        raise HydraError(1, "acc must be fp32 and b_bf16 hold at least acc.numel() bf16 values")
    s = stream if stream is not None else _stream_ptr(acc.device)
    check(_lib.lib().hydra_acc_bf16_f32(acc.data_ptr(), b_bf16.data_ptr(), acc.numel(), s))


def f32_to_bf16_(out_bf16, acc, stream: int | None = None) -> None:
    if out_bf16.numel() * out_bf16.element_size() < 2 * acc.numel() or acc.dtype.itemsize != 4:
        raise HydraError(1, "acc must be fp32 and out_bf16 hold at least acc.numel() values")
    s = stream if stream is not None else _stream_ptr(acc.device)
    check(_lib.lib().hydra_f32_to_bf16(out_bf16.data_ptr(), acc.data_ptr(), acc.numel(), s))


# --------------------------------------------------------------------------- host buffers
class HostContext:
    """One host-call context per calling thread (hydra_ctx_t): pinned staging, a stream, and the
    resident reducer that serves small synchronous calls without a launch."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check(_lib.lib().hydra_ctx_create(device, ctypes.byref(h)))
        self._h = h

    @property
    def handle(self) -> int:
        return self._h.value

    def set_option(self, key: int, value: int) -> None:
        """hydra_ctx_set_option: a per-context option (_lib.OPT_*, e.g. OPT_FORCE_STAGING)."""
        check(_lib.lib().hydra_ctx_set_option(self._h, key, int(value)))

    def stats(self) -> dict:
        """Calls the resident reducer served and instances launched (hydra_ctx_stats)."""
        calls, launches = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().hydra_ctx_stats(self._h, ctypes.byref(calls), ctypes.byref(launches)))
        return {"resident_calls": calls.value, "resident_launches": launches.value}

    def close(self) -> None:
        if self._h:
            _lib.lib().hydra_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        # never call into HIP/RCCL while the interpreter is finalizing (the runtime may be gone);
        # `sys` is bound at import time: an import here fails during shutdown
        if _is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def _thread_ctx(device: int) -> HostContext:
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        ctx = _tls.ctx = HostContext(device)
    return ctx


def reduce_host(op: str, c: np.ndarray, a: np.ndarray, b: np.ndarray, n: int | None = None,
                dtype_code: int | None = None, device: int = 0) -> None:
    """Synchronous host-buffer reduction through the GPU (H2D -> kernel -> D2H)."""
    code = dtype_code if dtype_code is not None else _NP_DTYPES[c.dtype]
    if n is None:
        n = c.size
    for x in (c, a, b):
        if not x.flags.c_contiguous:
            raise HydraError(1, "contiguous arrays required")
    check(_lib.lib().hydra_reduce_host(_thread_ctx(device).handle, OPS[op], code, c.ctypes.data,
                                       a.ctypes.data, b.ctypes.data, n))


class ReductionFunction:
    """gloo::ReductionFunction<T> (algorithm.h:59-96): a (type, fn) pair whose fn has the
    AllreduceOptions::Func shape fn(c, a, b, n).  Pointer form: integer device addresses."""

    SUM, PRODUCT, MAX, MIN = 1, 2, 3, 4  # ReductionType (algorithm.h:49-57)

    def __init__(self, op: str, dtype_code: int, stream: int | None = None):
        self.op = op
        self.dtype_code = dtype_code
        self.stream = stream
        self.type = {"sum": 1, "product": 2, "max": 3, "min": 4}[op]

    def __call__(self, c: int, a: int, b: int, n: int) -> None:
        """Func(void* c, const void* a, const void* b, size_t n) on device addresses."""
        check(_lib.lib().hydra_reduce(OPS[self.op], self.dtype_code, c, a, b, n,
                                      self.stream or 0))

    def call(self, x, y, n: int) -> None:
        """ReductionFunction<T>::call(T* x, const T* y, size_t n): x = op(x, y) (tensors)."""
        reduce_(self.op, x, x, y, n, dtype_code=self.dtype_code, stream=self.stream)
