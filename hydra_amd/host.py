"""ctypes face of libhydra_host.so (include/hydra_host.h): the C++ host runtime that mirrors
hydra/Gloo's new_allreduce_ring / bew_allreduce_a over loopback TCP, reducing each segment on
the MI355X through libhydra_hip.so."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib

LIB_PATH = os.path.join(_lib.HERE, "libhydra_host.so")
# OUT OF SCOPE, opt-in: the other Algorithm-API classes (include/hydra_host_extra.h)
EXTRA_LIB_PATH = os.path.join(_lib.HERE, "libhydra_host_extra.so")
REDUCER_GPU, REDUCER_FN = 0, 1
SPLIT_AA, SPLIT_AG = 0, 1
REDUCE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_size_t)
_h = None
_x = None


def lib():
    global _h
    if _h is None:
        _lib.lib()  # libhydra_hip.so first (binds to torch's HIP runtime when present)
        if not os.path.exists(LIB_PATH):
            raise _lib.HydraError(-1, f"{LIB_PATH} is not built")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.hydra_host_allreduce_threads.argtypes = [i, i, i, i, sz, vp, vp, sz, i, i, vp,
                                                   ctypes.c_long, ctypes.c_char_p, sz]
        L.hydra_host_apipe_threads.argtypes = [i, i, sz, vp, vp, i, i, vp, ctypes.c_char_p, sz]
        L.hydra_host_bench.argtypes = [i, i, sz, i, i, i, vp, vp, ctypes.c_char_p, sz]
        L.hydra_host_calculate_elements.argtypes = [i, i, sz, ctypes.POINTER(sz),
                                                    ctypes.POINTER(sz)]
        L.hydra_host_calculate_elements.restype = None
        L.hydra_host_timeout_probe.argtypes = [ctypes.c_long, ctypes.c_char_p, sz]
        L.hydra_host_allreduce_ring_old_threads.argtypes = [i, i, i, sz, vp, i, vp,
                                                            ctypes.c_char_p, sz]
        L.hydra_host_hip_ring_threads.argtypes = [i, i, i, sz, vp, i, i, ctypes.c_char_p, sz]
        L.hydra_host_hip_ring_chunked_threads.argtypes = L.hydra_host_hip_ring_threads.argtypes
        L.hydra_host_allreduce_ring_chunked_threads.argtypes = \
            L.hydra_host_allreduce_ring_old_threads.argtypes
        L.hydra_host_reduce_threads.argtypes = [i, i, i, sz, vp, vp, i, sz, i, vp,
                                                ctypes.c_long, ctypes.c_char_p, sz]
        L.hydra_host_reduce_timeout_probe.argtypes = [ctypes.c_long, ctypes.c_char_p, sz]
        L.hydra_host_slow_peer_probe.argtypes = [ctypes.c_long, ctypes.c_long, sz,
                                                 ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_int)]
        _h = L
    return _h


def extra_lib():
    """libhydra_host_extra.so: AllreduceHalvingDoubling / old-style AllreduceBcube /
    AllreduceLocal and their Hip* twins -- only the `extra` tests use it."""
    global _x
    if _x is None:
        lib()
        if not os.path.exists(EXTRA_LIB_PATH):
            raise _lib.HydraError(-1, f"{EXTRA_LIB_PATH} is not built")
        L = ctypes.CDLL(EXTRA_LIB_PATH)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        old = [i, i, i, sz, vp, i, vp, ctypes.c_char_p, sz]
        hip = [i, i, i, sz, vp, i, i, ctypes.c_char_p, sz]
        for nm in ("halving_doubling", "bcube_old", "local"):
            getattr(L, f"hydra_host_allreduce_{nm}_threads").argtypes = old
        for nm in ("halving_doubling", "local", "bcube"):
            getattr(L, f"hydra_host_hip_{nm}_threads").argtypes = hip
        _x = L
    return _x


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def _ptrs_int(addrs):
    return (ctypes.c_void_p * len(addrs))(*addrs)


def _fn(reducer_fn):
    """reducer_fn: None -> GPU; an int address of a C function with the Func signature."""
    if reducer_fn is None:
        return REDUCER_GPU, None
    return REDUCER_FN, ctypes.c_void_p(reducer_fn)


def allreduce_threads(outs, ins=None, dtype_code=None, op="sum", max_segment=0, reducer_fn=None,
                      timeout_ms=0, pinned_scratch=False, algorithm="ring"):
    """gloo::allreduce(RING) on len(outs) thread-ranks; outs/ins: [rank][ptr] numpy arrays.
    pinned_scratch (GPU reducer): the ring's receive slots come from pinned memory."""
    P, nptr = len(outs), len(outs[0])
    n = outs[0][0].size
    code = dtype_code if dtype_code is not None else _np_code(outs[0][0].dtype)
    red, fp = _fn(reducer_fn)
    if pinned_scratch:
        if reducer_fn is not None:
            raise _lib.HydraError(1, "pinned_scratch applies to the GPU reducer")
        red = 2
    err = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_allreduce_threads(
        P, nptr, _lib.OPS[op], code, n,
        ctypes.cast(_ptrs([a for r in ins for a in r]), ctypes.c_void_p) if ins else None,
        ctypes.cast(_ptrs([a for r in outs for a in r]), ctypes.c_void_p), max_segment,
        {"ring": 1, "bcube": 2}[algorithm], red, fp, timeout_ms, err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return outs


def reduce_threads(outs, ins=None, root=0, dtype_code=None, op="sum", max_segment=0,
                   reducer_fn=None, timeout_ms=0, pinned_scratch=False):
    """gloo::reduce (reduce.cc:21-262) to `root` on len(outs) thread-ranks; outs/ins: one numpy
    array per rank (ins None: in place).  Only outs[root] is the reduction."""
    P, n = len(outs), outs[0].size
    code = dtype_code if dtype_code is not None else _np_code(outs[0].dtype)
    red, fp = _fn(reducer_fn)
    if pinned_scratch:
        if reducer_fn is not None:
            raise _lib.HydraError(1, "pinned_scratch applies to the GPU reducer")
        red = 2
    err = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_reduce_threads(
        P, _lib.OPS[op], code, n,
        ctypes.cast(_ptrs(ins), ctypes.c_void_p) if ins is not None else None,
        ctypes.cast(_ptrs(outs), ctypes.c_void_p), root, max_segment, red, fp, timeout_ms,
        err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return outs


def slow_peer_probe(timeout_ms: int, delay_ms: int, n: int = 1 << 16):
    """(rc, message, intact): see hydra_host_slow_peer_probe (include/hydra_host.h)."""
    what = ctypes.create_string_buffer(512)
    intact = ctypes.c_int(0)
    rc = lib().hydra_host_slow_peer_probe(timeout_ms, delay_ms, n, what, 512,
                                          ctypes.byref(intact))
    return rc, what.value.decode(), bool(intact.value)


def reduce_timeout_probe(ms: int):
    what = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_reduce_timeout_probe(ms, what, 512)
    return rc, what.value.decode()


def apipe_threads(ins, outs, table=SPLIT_AA, reducer_fn=None, dtype_code=_lib.FLOAT32):
    P, n = len(ins), ins[0].size
    red, fp = _fn(reducer_fn)
    err = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_apipe_threads(P, dtype_code, n,
                                        ctypes.cast(_ptrs(ins), ctypes.c_void_p),
                                        ctypes.cast(_ptrs(outs), ctypes.c_void_p), table, red, fp,
                                        err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return outs


def allreduce_ring_old_threads(bufs, dtype_code=None, reducer_fn=None, chunked=False,
                               halving_doubling=False, bcube=False, local=False):
    """Old-style AllreduceRing<T>::run() on len(bufs) thread-ranks; bufs: [rank][ptr], in place.
    reducer_fn: None -> GPU sum; else address of a void(T* x, const T* y, size_t n).
    chunked: AllreduceRingChunked<T> instead; halving_doubling: AllreduceHalvingDoubling<T>."""
    P, nptr = len(bufs), len(bufs[0])
    n = bufs[0][0].size
    code = dtype_code if dtype_code is not None else _np_code(bufs[0][0].dtype)
    red, fp = _fn(reducer_fn)
    err = ctypes.create_string_buffer(512)
    f = (lib().hydra_host_allreduce_ring_chunked_threads if chunked
         else lib().hydra_host_allreduce_ring_old_threads)
    if halving_doubling:
        f = extra_lib().hydra_host_allreduce_halving_doubling_threads
    if bcube:
        f = extra_lib().hydra_host_allreduce_bcube_old_threads
    if local:
        f = extra_lib().hydra_host_allreduce_local_threads
    rc = f(
        P, nptr, code, n, ctypes.cast(_ptrs([b for r in bufs for b in r]), ctypes.c_void_p), red,
        fp, err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return bufs


def allreduce_halving_doubling_threads(bufs, dtype_code=None, reducer_fn=None):
    """hydra::AllreduceHalvingDoubling<T>::run() (allreduce_halving_doubling.h:37-358) on
    len(bufs) thread-ranks over loopback TCP; same arguments as allreduce_ring_old_threads."""
    return allreduce_ring_old_threads(bufs, dtype_code, reducer_fn, halving_doubling=True)


def allreduce_bcube_old_threads(bufs, dtype_code=None, reducer_fn=None):
    """Old-style hydra::AllreduceBcube<T>::run() (allreduce_bcube.h, base 2) on len(bufs)
    thread-ranks (a power of two); same arguments as allreduce_ring_old_threads."""
    return allreduce_ring_old_threads(bufs, dtype_code, reducer_fn, bcube=True)


def hip_ring_threads(tensors, workspace: str = "host", user_streams: bool = False,
                     dtype_code=None, chunked: bool = False, halving_doubling: bool = False,
                     local: bool = False, bcube: bool = False):
    """hydra::HipAllreduceRing<T, W>::run() (gloo::CudaAllreduceRing) on len(tensors)
    thread-ranks; tensors: [rank][ptr] contiguous device tensors, reduced in place.
    chunked: HipAllreduceRingChunked<T, W> (gloo::CudaAllreduceRingChunked) instead;
    halving_doubling: HipAllreduceHalvingDoubling<T, W> (gloo::CudaAllreduceHalvingDoubling)."""
    from .reduce import _torch_dtype_code

    P, nptr = len(tensors), len(tensors[0])
    n = tensors[0][0].numel()
    code = dtype_code if dtype_code is not None else _torch_dtype_code(tensors[0][0])
    for r in tensors:
        for t in r:
            if not (t.is_cuda and t.is_contiguous() and t.numel() == n):
                raise _lib.HydraError(1, "contiguous, equally sized device tensors required")
    ws = {"host": 0, "device": 1}[workspace]
    err = ctypes.create_string_buffer(512)
    fn = (lib().hydra_host_hip_ring_chunked_threads if chunked
          else lib().hydra_host_hip_ring_threads)
    if halving_doubling:
        fn = extra_lib().hydra_host_hip_halving_doubling_threads
    if local:  # HipAllreduceLocal<T> (gloo::CudaAllreduceLocal)
        fn = extra_lib().hydra_host_hip_local_threads
    if bcube:  # HipAllreduceBcube<T, W> (gloo::CudaAllreduceBcube)
        fn = extra_lib().hydra_host_hip_bcube_threads
    rc = fn(
        P, nptr, code, n, ctypes.cast(_ptrs_int([t.data_ptr() for r in tensors for t in r]),
                                      ctypes.c_void_p), ws, int(user_streams), err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return tensors


def bench(config: int, P: int, n: int, warmup: int, iters: int, reducer_fn=None,
          pinned: bool = False, gpu_rank0_only: bool = False) -> np.ndarray:
    """Per-iteration ns of rank 0.  pinned (GPU reducer only): pinned receive slots and a
    registered output, so each segment reduce is the zero-copy kernel.  gpu_rank0_only: rank 0
    reduces zero-copy on the GPU, the other ranks with reducer_fn (HYDRA_REDUCER_GPU_PINNED_RANK0:
    rank 0 has the box's one PCIe link to itself, as with one MI355X per rank)."""
    s = np.zeros(iters, np.float64)
    red, fp = _fn(reducer_fn)
    if gpu_rank0_only:
        if reducer_fn is None:
            raise _lib.HydraError(1, "gpu_rank0_only needs reducer_fn for the other ranks")
        red = 3
    elif pinned:
        if reducer_fn is not None:
            raise _lib.HydraError(1, "pinned applies to the GPU reducer")
        red = 2
    err = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_bench(config, P, n, warmup, iters, red, fp, s.ctypes.data, err, 512)
    if rc:
        raise _lib.HydraError(rc, err.value.decode())
    return s


def calculate_elements(table: int, P: int, n: int):
    e1, e2 = ctypes.c_size_t(), ctypes.c_size_t()
    lib().hydra_host_calculate_elements(table, P, n, ctypes.byref(e1), ctypes.byref(e2))
    return e1.value, e2.value


def timeout_probe(ms: int):
    buf = ctypes.create_string_buffer(512)
    rc = lib().hydra_host_timeout_probe(ms, buf, 512)
    return rc, buf.value.decode()


def _np_code(dt):
    return {np.dtype(np.float32): _lib.FLOAT32, np.dtype(np.int32): _lib.INT32,
            np.dtype(np.uint64): _lib.UINT64, np.dtype(np.int64): _lib.INT64,
            np.dtype(np.float64): _lib.FLOAT64, np.dtype(np.uint16): _lib.FLOAT16,
            np.dtype(np.int8): _lib.INT8, np.dtype(np.uint8): _lib.UINT8,
            np.dtype(np.uint32): _lib.UINT32}[np.dtype(dt)]
