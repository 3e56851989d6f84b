"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

numpy front-end for
  * ``liboracle.so``          our plain-C restatement of the hot path (oracle/hydra_oracle.c)
  * ``_ref/libgloo_ref.so``   the reference's own code compiled from /root/reference (Makefile)
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product (hydra_amd) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIBORACLE = os.path.join(HERE, "liboracle.so")
LIBREF = os.path.join(HERE, "_ref", "libgloo_ref.so")

DTYPES = {  # hydra_dtype_t numbering (include/hydra_hip.h)
    np.dtype(np.int8): 0, np.dtype(np.uint8): 1, np.dtype(np.int32): 2, np.dtype(np.uint32): 3,
    np.dtype(np.int64): 4, np.dtype(np.uint64): 5, np.dtype(np.float32): 6,
    np.dtype(np.float64): 7,
}
F16, BF16 = 8, 9
OPS = {"sum": 0, "product": 1, "max": 2, "min": 3}

_c = ctypes.c_size_t
_vp = ctypes.c_void_p


def build(force: bool = False) -> None:
    """Compile the C restatement (always possible) and, when the reference tree is present,
    the reference core.  Prebuilt files travel to the GPU box with the repo snapshot."""
    if force or not os.path.exists(LIBORACLE):
        subprocess.check_call(["make", "-s", "-C", HERE, "oracle"])
    if os.path.isdir("/root/reference/gloo"):
        if force or not os.path.exists(LIBREF):
            subprocess.check_call(["make", "-s", "-j8", "-C", HERE, "ref"])
        # the reference's two-rail split, compiled from its header text (split_ref.py)
        from oracle import split_ref

        if force or not os.path.exists(split_ref.OUT):
            split_ref.build()
        # the drop-in harness links libhydra_hip.so too: make rebuilds it when either changed
        if os.path.exists(os.path.join(os.path.dirname(HERE), "hydra_amd", "libhydra_hip.so")):
            subprocess.check_call(["make", "-s", "-C", HERE, "dropin"])


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run oracle.build())")
    return ctypes.CDLL(path)


_orc = None
_ref = None


def orc():
    global _orc
    if _orc is None:
        _orc = _load(LIBORACLE)
        _orc.orc_op.argtypes = [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _c]
        _orc.orc_allreduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       _c, _vp, _vp, _c]
        _orc.orc_ring_plan.argtypes = [ctypes.c_int, _c, _c, _c] + [ctypes.POINTER(_c)] * 3
        _orc.orc_split_aa.argtypes = [ctypes.c_int, _c, ctypes.POINTER(_c), ctypes.POINTER(_c)]
        _orc.orc_split_ag.argtypes = _orc.orc_split_aa.argtypes
        _orc.orc_f2h.argtypes = [ctypes.c_float]
        _orc.orc_f2h.restype = ctypes.c_uint16
        _orc.orc_h2f.argtypes = [ctypes.c_uint16]
        _orc.orc_h2f.restype = ctypes.c_float
        _orc.orc_acc_bf16_f32.argtypes = [_vp, _vp, _c]
        _orc.orc_allreduce_ring_old.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int, _c, _vp]
        _orc.orc_allreduce_ring_chunked.argtypes = _orc.orc_allreduce_ring_old.argtypes
        _orc.orc_allreduce_halving_doubling.argtypes = _orc.orc_allreduce_ring_old.argtypes
        _orc.orc_allreduce_bcube.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int, _c, _vp, _vp]
        _orc.orc_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c, _vp, _vp,
                                    ctypes.c_int, _c]
        _orc.orc_reduce_plan.argtypes = _orc.orc_ring_plan.argtypes
    return _orc


def ref_available() -> bool:
    return os.path.exists(LIBREF)


def ref():
    global _ref
    if _ref is None:
        _ref = _load(LIBREF)
        _ref.ref_op.argtypes = [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _c]
        _ref.ref_allreduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c,
                                       _vp, _vp, _c, ctypes.c_int, ctypes.c_long,
                                       ctypes.c_char_p, _c]
        _ref.ref_allreduce_timeout.argtypes = [ctypes.c_long, ctypes.c_char_p, _c]
        _ref.ref_time_op.argtypes = [ctypes.c_int, ctypes.c_int, _vp, _vp, _vp, _c,
                                     ctypes.c_int, ctypes.c_int]
        _ref.ref_time_op.restype = ctypes.c_double
        _ref.ref_bench_ring.argtypes = [ctypes.c_int, _c, ctypes.c_int, ctypes.c_int, _vp,
                                        ctypes.c_char_p, _c]
        _ref.ref_float2half.argtypes = [ctypes.c_float]
        _ref.ref_float2half.restype = ctypes.c_uint16
        _ref.ref_allreduce_ring_old.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c,
                                                _vp, ctypes.c_char_p, _c]
        _ref.ref_allreduce_ring_chunked.argtypes = _ref.ref_allreduce_ring_old.argtypes
        _ref.ref_allreduce_halving_doubling.argtypes = _ref.ref_allreduce_ring_old.argtypes
        _ref.ref_allreduce_bcube_old.argtypes = _ref.ref_allreduce_ring_old.argtypes
        _ref.ref_reduce.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c, _vp, _vp,
                                    ctypes.c_int, _c, ctypes.c_long, ctypes.c_char_p, _c]
        _ref.ref_reduce_timeout.argtypes = [ctypes.c_long, ctypes.c_char_p, _c]
    return _ref


_ESIZE = (1, 1, 4, 4, 8, 8, 4, 8, 2, 2)  # element size per hydra_dtype_t code


def _dt(arr: np.ndarray, dtype_code: int | None) -> int:
    if dtype_code is not None:
        # the C side walks arr.size elements of the code's size: they must be arr's own
        if not (0 <= dtype_code < len(_ESIZE)) or _ESIZE[dtype_code] != arr.itemsize:
            raise ValueError(f"dtype code {dtype_code} does not match a {arr.dtype} array")
        return dtype_code
    return DTYPES[arr.dtype]


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# ---------------------------------------------------------------- element-wise
def op(a: np.ndarray, b: np.ndarray, kind: str = "sum", dtype_code: int | None = None,
       lib: str = "oracle") -> np.ndarray:
    """c = op(a, b) via the C restatement (lib='oracle') or the reference (lib='ref').
    c starts as a copy of a: the in-place form the ring uses (allreduce.cc:301-305), which
    matters for float16, whose stores depend on the destination's old bits (types.h:112-130).
    fp16/bf16 operands are passed as uint16 bit patterns with dtype_code F16/BF16."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    c = a.copy()
    L = orc() if lib == "oracle" else ref()
    fn = L.orc_op if lib == "oracle" else L.ref_op
    rc = fn(OPS[kind], _dt(a, dtype_code), _ptr(c), _ptr(a), _ptr(b), a.size)
    if rc:
        raise ValueError(f"unsupported op/dtype rc={rc}")
    return c


def ring_plan(P: int, n: int, esize: int, max_segment: int = 1 << 20):
    ns, sb, S = _c(), _c(), _c()
    orc().orc_ring_plan(P, n, esize, max_segment, ctypes.byref(ns), ctypes.byref(sb),
                        ctypes.byref(S))
    return ns.value, sb.value, S.value


def _allreduce(fn_is_ref, P, outs, ins, kind, dtype_code, max_segment, algorithm=1):
    """outs/ins: list over ranks of list over pointers of arrays (modified in place)."""
    nptr = len(outs[0])
    n = outs[0][0].size
    code = _dt(outs[0][0], dtype_code)
    optrs = (_vp * (P * nptr))(*[_ptr(o) for r in outs for o in r])
    iptrs = (_vp * (P * nptr))(*[_ptr(i) for r in ins for i in r]) if ins is not None else None
    if fn_is_ref:
        err = ctypes.create_string_buffer(512)
        rc = ref().ref_allreduce(P, nptr, OPS[kind], code, n,
                                 ctypes.cast(iptrs, _vp) if iptrs is not None else None,
                                 ctypes.cast(optrs, _vp), max_segment, algorithm, 0, err, 512)
        if rc:
            raise RuntimeError(f"reference allreduce failed: {err.value.decode()}")
    elif algorithm == 2:  # BCUBE
        rc = orc().orc_allreduce_bcube(P, nptr, OPS[kind], code, n,
                                       ctypes.cast(iptrs, _vp) if iptrs is not None else None,
                                       ctypes.cast(optrs, _vp))
        if rc:
            raise RuntimeError("oracle bcube failed")
    else:
        rc = orc().orc_allreduce(P, nptr, OPS[kind], code, n,
                                 ctypes.cast(iptrs, _vp) if iptrs is not None else None,
                                 ctypes.cast(optrs, _vp), max_segment)
        if rc:
            raise RuntimeError("oracle allreduce failed")
    return outs


def allreduce(P, outs, ins=None, kind="sum", dtype_code=None, max_segment=1 << 20, algorithm=1):
    """C restatement of gloo::allreduce (1 RING, 2 BCUBE) over P ranks; returns outs (in place)."""
    return _allreduce(False, P, outs, ins, kind, dtype_code, max_segment, algorithm)


def bcube_result(xs: list[np.ndarray], kind: str = "sum",
                 dtype_code: int | None = None) -> np.ndarray:
    """Convenience: BCUBE-reduced bucket of in-place single-pointer ranks xs (not modified)."""
    outs = [[x.copy()] for x in xs]
    allreduce(len(xs), outs, None, kind, dtype_code, algorithm=2)
    return outs[0][0]


def ref_allreduce(P, outs, ins=None, kind="sum", dtype_code=None, max_segment=1 << 20,
                  algorithm=1):
    """The reference's own gloo::allreduce over P loopback thread-ranks."""
    return _allreduce(True, P, outs, ins, kind, dtype_code, max_segment, algorithm)


def ring_result(xs: list[np.ndarray], max_segment: int = 1 << 20, kind: str = "sum",
                dtype_code: int | None = None) -> np.ndarray:
    """Convenience: reduced bucket of in-place single-pointer ranks xs (not modified)."""
    outs = [[x.copy()] for x in xs]
    allreduce(len(xs), outs, None, kind, dtype_code, max_segment)
    return outs[0][0]


def _old_ring(fn_is_ref, bufs, kind, dtype_code, chunked=False, hd=False):
    """bufs: [rank][ptr] arrays, in place.  chunked: AllreduceRingChunked<T> instead;
    hd: AllreduceHalvingDoubling<T> instead."""
    P, nptr = len(bufs), len(bufs[0])
    n = bufs[0][0].size
    code = _dt(bufs[0][0], dtype_code)
    ptrs = (_vp * (P * nptr))(*[_ptr(b) for r in bufs for b in r])
    if fn_is_ref:
        err = ctypes.create_string_buffer(512)
        f = ref().ref_allreduce_ring_chunked if chunked else ref().ref_allreduce_ring_old
        f = ref().ref_allreduce_halving_doubling if hd else f
        rc = f(P, nptr, code, n, ctypes.cast(ptrs, _vp), err, 512)
        if rc:
            raise RuntimeError(f"reference AllreduceRing failed: {err.value.decode()}")
    else:
        f = orc().orc_allreduce_ring_chunked if chunked else orc().orc_allreduce_ring_old
        f = orc().orc_allreduce_halving_doubling if hd else f
        rc = f(P, nptr, OPS[kind], code, n, ctypes.cast(ptrs, _vp))
        if rc:
            raise RuntimeError(f"oracle AllreduceRing failed (rc {rc})")
    return bufs


def allreduce_ring_old(bufs, kind="sum", dtype_code=None):
    """C restatement of the old-style gloo::AllreduceRing<T>::run() over len(bufs) ranks."""
    return _old_ring(False, bufs, kind, dtype_code)


def ref_allreduce_ring_old(bufs, dtype_code=None):
    """The reference's own AllreduceRing<T> (ReductionFunction<T>::sum) on thread-ranks."""
    return _old_ring(True, bufs, "sum", dtype_code)


def allreduce_ring_chunked(bufs, kind="sum", dtype_code=None):
    """C restatement of gloo::AllreduceRingChunked<T>::run() over len(bufs) ranks."""
    return _old_ring(False, bufs, kind, dtype_code, chunked=True)


def ref_allreduce_ring_chunked(bufs, dtype_code=None):
    """The reference's own AllreduceRingChunked<T> (ReductionFunction<T>::sum) on thread-ranks."""
    return _old_ring(True, bufs, "sum", dtype_code, chunked=True)


def allreduce_halving_doubling(bufs, kind="sum", dtype_code=None):
    """C restatement of gloo::AllreduceHalvingDoubling<T>::run() over len(bufs) ranks
    (allreduce_halving_doubling.h:37-358)."""
    return _old_ring(False, bufs, kind, dtype_code, hd=True)


def ref_allreduce_halving_doubling(bufs, dtype_code=None):
    """The reference's own AllreduceHalvingDoubling<T> (ReductionFunction<T>::sum)."""
    return _old_ring(True, bufs, "sum", dtype_code, hd=True)


def ref_allreduce_bcube_old(bufs, dtype_code=None):
    """The reference's own old-style AllreduceBcube<T> (allreduce_bcube.h, context base 2) on
    thread-ranks, in place on bufs ([rank][ptr])."""
    P, nptr = len(bufs), len(bufs[0])
    ptrs = (_vp * (P * nptr))(*[_ptr(b) for r in bufs for b in r])
    err = ctypes.create_string_buffer(512)
    rc = ref().ref_allreduce_bcube_old(P, nptr, _dt(bufs[0][0], dtype_code), bufs[0][0].size,
                                      ctypes.cast(ptrs, _vp), err, 512)
    if rc:
        raise RuntimeError(f"reference AllreduceBcube failed: {err.value.decode()}")
    return bufs


def split_aa(P: int, n: int):
    e1, e2 = _c(), _c()
    orc().orc_split_aa(P, n, ctypes.byref(e1), ctypes.byref(e2))
    return e1.value, e2.value


def split_ag(P: int, n: int):
    e1, e2 = _c(), _c()
    orc().orc_split_ag(P, n, ctypes.byref(e1), ctypes.byref(e2))
    return e1.value, e2.value


def acc_bf16_f32(acc: np.ndarray, b_bits: np.ndarray) -> np.ndarray:
    acc = np.ascontiguousarray(acc, dtype=np.float32).copy()
    b_bits = np.ascontiguousarray(b_bits, dtype=np.uint16)
    orc().orc_acc_bf16_f32(_ptr(acc), _ptr(b_bits), acc.size)
    return acc


def f2h(x: float) -> int:
    return orc().orc_f2h(x)


def h2f(h: int) -> float:
    return orc().orc_h2f(h)


# ---------------------------------------------------------------- timing (cpu_baseline)
def ref_time_sum(dtype_code: int, c: np.ndarray, a: np.ndarray, b: np.ndarray, iters: int,
                 reps: int) -> float:
    """Seconds per call of the reference's gloo::sum<T> (single thread, best of reps)."""
    return ref().ref_time_op(0, dtype_code, _ptr(c), _ptr(a), _ptr(b), a.size, iters, reps)


def ref_bench_ring(P: int, n: int, warmup: int, iters: int) -> np.ndarray:
    s = np.zeros(iters, dtype=np.float64)
    err = ctypes.create_string_buffer(512)
    rc = ref().ref_bench_ring(P, n, warmup, iters, _ptr(s), err, 512)
    if rc:
        raise RuntimeError(err.value.decode())
    return s


# ---------------------------------------------------------------- gloo::reduce (reduce.cc)
def reduce_plan(P: int, n: int, esize: int, max_segment: int = 1 << 20):
    """(numSegments, segmentBytes, segments per rank) of gloo::reduce (reduce.cc:87-135)."""
    ns, sb, S = _c(), _c(), _c()
    orc().orc_reduce_plan(P, n, esize, max_segment, ctypes.byref(ns), ctypes.byref(sb),
                          ctypes.byref(S))
    return ns.value, sb.value, S.value


def _reduce(fn_is_ref, outs, ins, root, kind, dtype_code, max_segment, timeout_ms=0):
    P = len(outs)
    n = outs[0].size
    code = _dt(outs[0], dtype_code)
    optrs = (_vp * P)(*[_ptr(o) for o in outs])
    iptrs = (_vp * P)(*[_ptr(i) for i in ins]) if ins is not None else None
    ip = ctypes.cast(iptrs, _vp) if iptrs is not None else None
    if fn_is_ref:
        err = ctypes.create_string_buffer(512)
        rc = ref().ref_reduce(P, OPS[kind], code, n, ip, ctypes.cast(optrs, _vp), root,
                              max_segment, timeout_ms, err, 512)
        if rc:
            raise RuntimeError(f"reference reduce failed: {err.value.decode()}")
    else:
        rc = orc().orc_reduce(P, OPS[kind], code, n, ip, ctypes.cast(optrs, _vp), root,
                              max_segment)
        if rc:
            raise RuntimeError("oracle reduce failed")
    return outs


def reduce(outs, ins=None, root=0, kind="sum", dtype_code=None, max_segment=1 << 20):
    """C restatement of gloo::reduce: writes the root's output (outs[root]) only.  float16
    only in place (out of place, its stores depend on the output's old bits)."""
    return _reduce(False, outs, ins, root, kind, dtype_code, max_segment)


def ref_reduce(outs, ins=None, root=0, kind="sum", dtype_code=None, max_segment=1 << 20):
    """The reference's own gloo::reduce over len(outs) loopback thread-ranks; every rank's
    output is left as the reference leaves it."""
    return _reduce(True, outs, ins, root, kind, dtype_code, max_segment)


def ref_reduce_timeout(timeout_ms: int = 10) -> str:
    what = ctypes.create_string_buffer(512)
    if ref().ref_reduce_timeout(timeout_ms, what, 512):
        raise RuntimeError("reference reduce did not time out")
    return what.value.decode()
