"""ctypes binding of libhydra_hip.so (include/hydra_hip.h).

The library is built in-tree (hydra_amd/csrc/Makefile -> hydra_amd/libhydra_hip.so).  There is no
fallback: if the shared object is missing or fails to load, every entry point raises
HydraError -- the hot path never silently runs on the CPU.

measure_lib() loads libhydra_measure.so instead: the same library built with -DHYDRA_MEASURE,
which adds the A/B kernel variants and the peer kernel's phase clocks (include/hydra_measure.h).
Only scripts/ and the variant parity tests use it; select_measure() makes lib() return it for a
whole measurement process (so hydra_amd.peer / .ring / .reduce run on it).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libhydra_hip.so")
MEASURE_LIB_PATH = os.path.join(HERE, "libhydra_measure.so")
CSRC = os.path.join(HERE, "csrc")

# hydra_dtype_t / hydra_op_t
INT8, UINT8, INT32, UINT32, INT64, UINT64, FLOAT32, FLOAT64, FLOAT16, BFLOAT16 = range(10)
SUM, PRODUCT, MAX, MIN = range(4)
OPS = {"sum": SUM, "product": PRODUCT, "max": MAX, "min": MIN}
ESIZE = {INT8: 1, UINT8: 1, INT32: 4, UINT32: 4, INT64: 8, UINT64: 8, FLOAT32: 4, FLOAT64: 8,
         FLOAT16: 2, BFLOAT16: 2}

EXPORTS = [  # every symbol include/hydra_hip.h declares
    "hydra_abi_version", "hydra_last_error", "hydra_device_count", "hydra_device_arch",
    "hydra_device_check", "hydra_fault_report_enable", "hydra_fault_last", "hydra_fault_lookup",
    "hydra_event_create", "hydra_event_create_on", "hydra_event_record", "hydra_event_synchronize",
    "hydra_event_destroy",
    "hydra_reduce", "hydra_chunk_sum", "hydra_reduce_batch", "hydra_acc_bf16_f32", "hydra_f32_to_bf16",
    "hydra_set_option", "hydra_get_option", "hydra_ctx_set_option",
    "hydra_ctx_create", "hydra_ctx_destroy", "hydra_reduce_host",
    "hydra_chunk_sum_host", "hydra_host_register", "hydra_host_unregister",
    "hydra_page_interior", "hydra_host_mappings", "hydra_ctx_stats",
    "hydra_stream_create", "hydra_stream_destroy", "hydra_stream_synchronize", "hydra_malloc",
    "hydra_free", "hydra_memcpy", "hydra_ring_plan",
    "hydra_comm_get_unique_id", "hydra_comm_init", "hydra_comm_destroy", "hydra_comm_info", "hydra_allreduce",
    "hydra_plan", "hydra_allreduce_simulate", "hydra_fold", "hydra_memcpy_async",
    "hydra_malloc_host", "hydra_free_host", "hydra_cache_trim", "hydra_pointer_device", "hydra_split_elements",
    "hydra_apipe_allreduce", "hydra_apipe_allreduce_simulate", "hydra_comm_run_plan",
    "hydra_peer_create", "hydra_peer_connect", "hydra_peer_register", "hydra_peer_open",
    "hydra_peer_close", "hydra_peer_set_option", "hydra_peer_error", "hydra_peer_allreduce",
    "hydra_peer_detach", "hydra_peer_destroy", "hydra_comm_wait",
    "hydra_reduce_root", "hydra_reduce_root_plan", "hydra_reduce_root_simulate",
    "hydra_comm_profile", "hydra_comm_phases", "hydra_stream_wait_event", "hydra_device_peer_access",
    "hydra_host_trace", "hydra_host_trace_read", "hydra_device_link",
    "hydra_test_set", "hydra_test_get",
]
MEASURE_EXPORTS = ["hydra_set_variant", "hydra_measure_peer_stamps"]  # include/hydra_measure.h

# hydra_opt_t (include/hydra_hip.h): library options, no environment variables
(OPT_RESIDENT, OPT_STAGE_SPLIT, OPT_ROUND_MIN, OPT_STAGE_RESULT_MAX, OPT_STAGE_RESULT_REG_MAX,
 OPT_FORCE_STAGING, OPT_COPY_THREADS, OPT_RESIDENT_IDLE_US, OPT_RESIDENT_GRACE_US,
 OPT_RESIDENT_QUEUE, OPT_RESIDENT_BLOCKS, OPT_RESIDENT_BATCH, OPT_RESIDENT_SOLO,
 OPT_RESIDENT_TILES) = range(1, 15)
PEER_STAMPS = 6  # hydra_measure_peer_stamps: clocks per workgroup

(ALGO_AUTO, ALGO_RING, ALGO_DIRECT, ALGO_RCCL, ALGO_A2A, ALGO_RING_OLD, ALGO_RING_CHUNKED,
 ALGO_BCUBE, ALGO_HALVING_DOUBLING, ALGO_RCCL_RS_AG) = range(10)
ALGOS = {"auto": ALGO_AUTO, "ring": ALGO_RING, "direct": ALGO_DIRECT, "rccl": ALGO_RCCL,
         "a2a": ALGO_A2A, "ring_old": ALGO_RING_OLD,
         "ring_chunked": ALGO_RING_CHUNKED, "bcube": ALGO_BCUBE,
         "halving_doubling": ALGO_HALVING_DOUBLING, "rccl_rs_ag": ALGO_RCCL_RS_AG}
ACC_F32 = 1
ALLOW_CAPTURE = 2
ERR_UNSUPPORTED = 3
ERR_INVALID = 1
ERR_TIMEOUT = 5
UNIQUE_ID_BYTES = 128
# peer-access allreduce (hydra_peer_*)
PEER_HANDLE_BYTES = 128
PEER_ALGOS = {"peer": 0, "peer2": 1, "peer1": 2, "peer2w": 3}  # AUTO, TWO_SHOT, ONE_SHOT,
# TWO_SHOT_PUSH (the fold writes the result into every rank's bucket)
PEER_OPT_TIMEOUT_MS, PEER_OPT_BLOCKS, PEER_OPT_ONE_SHOT_MAX = 1, 2, 3


class PlanOp(ctypes.Structure):
    """hydra_plan_op_t (include/hydra_hip.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("peer", ctypes.c_int32), ("buf", ctypes.c_int32),
                ("nsrc", ctypes.c_int32), ("off", ctypes.c_int64), ("bytes", ctypes.c_int64),
                ("src_off", ctypes.c_int64), ("slot_stride", ctypes.c_int64),
                ("wait0", ctypes.c_int32), ("wait1", ctypes.c_int32)]


OP_SEND, OP_RECV, OP_GROUP, OP_REDUCE, OP_FOLD, OP_ALLTOALL, OP_ALLGATHER = 1, 2, 3, 4, 5, 6, 7


class Segment(ctypes.Structure):
    """hydra_segment_t (include/hydra_hip.h): one c = op(a, b) of a hydra_reduce_batch call."""
    _fields_ = [("c", ctypes.c_void_p), ("a", ctypes.c_void_p), ("b", ctypes.c_void_p),
                ("n", ctypes.c_size_t)]


class HostMapping(ctypes.Structure):
    """hydra_host_mapping_t (include/hydra_hip.h): one of hydra's live host mappings."""
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64), ("kind", ctypes.c_int32),
                ("owners", ctypes.c_int32), ("users", ctypes.c_int32),
                ("owner_lo", ctypes.c_uint64), ("owner_hi", ctypes.c_uint64)]


MAP_REGISTER, MAP_PIN, MAP_PINNED_BLOCK = 1, 2, 3


class HostCall(ctypes.Structure):
    """hydra_host_call_t (include/hydra_hip.h): one traced hydra_reduce_host call."""
    _fields_ = [("n", ctypes.c_uint64), ("elem_bytes", ctypes.c_uint64),
                ("intervals", ctypes.c_uint32), ("rounds", ctypes.c_uint32),
                ("resident", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("zero_copy_bytes", ctypes.c_uint64 * 3), ("staged_bytes", ctypes.c_uint64 * 3),
                ("total_us", ctypes.c_double), ("copy_in_us", ctypes.c_double),
                ("wait_us", ctypes.c_double), ("copy_out_us", ctypes.c_double)]


class CommPhases(ctypes.Structure):
    """hydra_comm_phases_t (include/hydra_hip.h): per-phase totals of profiled allreduces."""
    _fields_ = [("calls", ctypes.c_uint64), ("link_ops", ctypes.c_uint64),
                ("fold_ops", ctypes.c_uint64), ("link_ms", ctypes.c_double),
                ("fold_ms", ctypes.c_double), ("span_ms", ctypes.c_double),
                ("sent_bytes", ctypes.c_uint64), ("recv_bytes", ctypes.c_uint64),
                ("fold_hbm_bytes", ctypes.c_uint64), ("peers", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class HydraError(RuntimeError):
    """A non-zero hydra_status_t (or a missing library)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"hydra error {code}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None


def fault_lookup(addr: int) -> str:
    """Where `addr` lies: its /proc/self/maps line and every hydra block, registration or
    per-call pin whose pages hold it (hydra_fault_lookup; the fault report's body)."""
    buf = ctypes.create_string_buffer(8192)
    check(lib().hydra_fault_lookup(addr, buf, len(buf)))
    return buf.value.decode(errors="replace")


def fault_last():
    """(virtual address, reason mask, count) of the last GPU memory fault seen since
    hydra_fault_report_enable (count 0: none)."""
    va, reason, count = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint64()
    check(lib().hydra_fault_last(ctypes.byref(va), ctypes.byref(reason), ctypes.byref(count)))
    return va.value, reason.value, count.value


def build(force: bool = False) -> str:
    """Compile libhydra_hip.so for gfx950 (hipcc cross-compiles without a GPU)."""
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    # the peer kernels build as one translation unit per op: -j up to 8 runs them side by side
    jobs = max(1, min(8, os.cpu_count() or 1))
    subprocess.check_call(["make", "-s", f"-j{jobs}", "-C", CSRC])
    return LIB_PATH


def _declare(L) -> None:
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.hydra_abi_version.restype = i
    L.hydra_last_error.restype = ctypes.c_char_p
    L.hydra_device_count.argtypes = [ctypes.POINTER(i)]
    L.hydra_device_arch.argtypes = [i, ctypes.c_char_p, sz]
    L.hydra_device_check.argtypes = [i]
    L.hydra_fault_last.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                                   ctypes.POINTER(ctypes.c_uint64)]
    L.hydra_fault_lookup.argtypes = [ctypes.c_uint64, ctypes.c_char_p, sz]
    L.hydra_event_create.argtypes = [ctypes.POINTER(vp)]
    L.hydra_event_create_on.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.hydra_event_record.argtypes = [vp, vp]
    L.hydra_event_synchronize.argtypes = [vp]
    L.hydra_event_destroy.argtypes = [vp]
    L.hydra_reduce.argtypes = [i, i, vp, vp, vp, sz, vp]
    L.hydra_chunk_sum.argtypes = [i, vp, vp, vp, sz, vp]
    L.hydra_reduce_batch.argtypes = [i, i, vp, sz, vp]
    L.hydra_acc_bf16_f32.argtypes = [vp, vp, sz, vp]
    L.hydra_f32_to_bf16.argtypes = [vp, vp, sz, vp]
    L.hydra_set_option.argtypes = [i, ctypes.c_longlong]
    L.hydra_get_option.argtypes = [i, ctypes.POINTER(ctypes.c_longlong)]
    L.hydra_ctx_set_option.argtypes = [vp, i, ctypes.c_longlong]
    L.hydra_ctx_create.argtypes = [i, ctypes.POINTER(vp)]
    L.hydra_ctx_destroy.argtypes = [vp]
    L.hydra_reduce_host.argtypes = [vp, i, i, vp, vp, vp, sz]
    L.hydra_chunk_sum_host.argtypes = [vp, i, vp, vp, vp, sz]
    L.hydra_host_register.argtypes = [vp, sz]
    L.hydra_host_unregister.argtypes = [vp]
    L.hydra_ctx_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64),
                                  ctypes.POINTER(ctypes.c_uint64)]
    L.hydra_page_interior.argtypes = [ctypes.c_uint64, sz, ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
    L.hydra_page_interior.restype = None
    L.hydra_host_mappings.argtypes = [ctypes.POINTER(HostMapping), sz, ctypes.POINTER(sz),
                                      ctypes.POINTER(ctypes.c_uint64),
                                      ctypes.POINTER(ctypes.c_uint64)]
    L.hydra_stream_create.argtypes = [i, ctypes.POINTER(vp)]
    L.hydra_stream_destroy.argtypes = [vp]
    L.hydra_stream_synchronize.argtypes = [vp]
    L.hydra_malloc.argtypes = [i, sz, ctypes.POINTER(vp)]
    L.hydra_free.argtypes = [vp]
    L.hydra_memcpy.argtypes = [vp, vp, sz]
    L.hydra_memcpy_async.argtypes = [vp, vp, sz, vp]
    L.hydra_malloc_host.argtypes = [sz, ctypes.POINTER(vp)]
    L.hydra_free_host.argtypes = [vp]
    L.hydra_cache_trim.argtypes = []
    L.hydra_pointer_device.argtypes = [vp, ctypes.POINTER(i)]
    L.hydra_split_elements.argtypes = [i, i, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.hydra_split_elements.restype = None
    L.hydra_apipe_allreduce.argtypes = [vp, vp, i, i, i, i, i, vp, sz, sz, sz, vp]
    L.hydra_comm_run_plan.argtypes = [vp, ctypes.POINTER(PlanOp), sz, i, i, i, vp, sz, sz, vp]
    L.hydra_apipe_allreduce_simulate.argtypes = [i, i, i, i, i, i, ctypes.POINTER(vp), sz, sz,
                                                 sz]
    L.hydra_ring_plan.argtypes = [i, sz, sz, sz] + [ctypes.POINTER(sz)] * 3
    L.hydra_ring_plan.restype = None
    L.hydra_comm_get_unique_id.argtypes = [vp]
    L.hydra_comm_init.argtypes = [ctypes.POINTER(vp), i, i, vp, i]
    L.hydra_comm_destroy.argtypes = [vp]
    L.hydra_comm_info.argtypes = [vp, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)]
    L.hydra_allreduce.argtypes = [vp, i, i, i, i, vp, sz, sz, sz, vp]
    L.hydra_plan.argtypes = [i, i, i, sz, sz, sz, sz, ctypes.POINTER(PlanOp), sz,
                             ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.hydra_allreduce_simulate.argtypes = [i, i, i, i, i, ctypes.POINTER(vp), sz, sz, sz]
    L.hydra_reduce_root.argtypes = [vp, i, i, i, i, vp, sz, sz, sz, vp]
    L.hydra_reduce_root_plan.argtypes = L.hydra_plan.argtypes
    L.hydra_reduce_root_simulate.argtypes = L.hydra_allreduce_simulate.argtypes
    L.hydra_fold.argtypes = [i, i, i, vp, ctypes.POINTER(vp), i, sz, vp]
    L.hydra_peer_create.argtypes = [i, i, i, ctypes.POINTER(vp), vp]
    L.hydra_peer_connect.argtypes = [vp, vp]
    L.hydra_peer_register.argtypes = [vp, vp, sz, vp]
    L.hydra_peer_open.argtypes = [vp, vp, sz, vp]
    L.hydra_peer_close.argtypes = [vp, vp]
    L.hydra_peer_set_option.argtypes = [vp, i, ctypes.c_longlong]
    L.hydra_peer_error.argtypes = [vp, ctypes.POINTER(i)]
    L.hydra_peer_allreduce.argtypes = [vp, i, i, i, i, vp, sz, sz, vp]
    L.hydra_peer_detach.argtypes = [vp]
    L.hydra_peer_destroy.argtypes = [vp]
    L.hydra_comm_wait.argtypes = [vp, vp, ctypes.c_int64]
    L.hydra_stream_wait_event.argtypes = [vp, vp]
    L.hydra_host_trace.argtypes = [i]
    L.hydra_host_trace_read.argtypes = [vp, sz, ctypes.POINTER(sz)]
    L.hydra_device_peer_access.argtypes = [i, i, ctypes.POINTER(i)]
    L.hydra_device_link.argtypes = [i, i, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)]
    L.hydra_comm_profile.argtypes = [vp, i]
    L.hydra_comm_phases.argtypes = [vp, ctypes.POINTER(CommPhases)]
    L.hydra_test_set.argtypes = [i, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
    L.hydra_test_get.argtypes = [i, ctypes.POINTER(ctypes.c_int64)]


def _load(path):
    if not os.path.exists(path):
        raise HydraError(-1, f"{path} is not built (hydra_amd._lib.build())")
    try:
        import torch  # noqa: F401  (bind to torch's libamdhip64 when present)
    except ImportError:
        pass
    return ctypes.CDLL(path)


def lib():
    """Load (once) and return the ctypes handle.  torch must be imported first on a GPU box so
    that this library binds to the same HIP runtime as torch (same soname)."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                L = _load(LIB_PATH)
                _declare(L)
                _lib = L
    return _lib


_measure = None


def measure_lib():
    """libhydra_measure.so (measurement build: hydra_set_variant, hydra_measure_peer_stamps)."""
    global _measure
    if _measure is None:
        with _lock:
            if _measure is None:
                M = _load(MEASURE_LIB_PATH)
                _declare(M)
                M.hydra_set_variant.argtypes = [ctypes.c_int]
                M.hydra_measure_peer_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_size_t]
                _measure = M
    return _measure


def select_measure() -> None:
    """Measurement processes only (scripts/): lib() returns the measurement build from now on.
    Call before anything has loaded the product library."""
    global _lib
    if _lib is not None and _lib is not _measure:
        raise HydraError(-1, "select_measure: the product library is already loaded")
    _lib = measure_lib()


def check(rc: int) -> None:
    if rc != 0:
        raise HydraError(rc, lib().hydra_last_error().decode(errors="replace"))


def set_option(key: int, value: int) -> None:
    """hydra_set_option: a process-wide library option (hydra_opt_t)."""
    check(lib().hydra_set_option(key, int(value)))


def get_option(key: int) -> int:
    v = ctypes.c_longlong()
    check(lib().hydra_get_option(key, ctypes.byref(v)))
    return v.value


def ring_plan(P: int, n: int, esize: int, max_segment: int = 1 << 20):
    ns, sb, S = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    lib().hydra_ring_plan(P, n, esize, max_segment, ctypes.byref(ns), ctypes.byref(sb),
                          ctypes.byref(S))
    return ns.value, sb.value, S.value


def page_interior(ptr: int, nbytes: int):
    """The whole pages inside [ptr, ptr + nbytes): (lo, hi), lo == hi when there are none."""
    lo, hi = ctypes.c_uint64(), ctypes.c_uint64()
    lib().hydra_page_interior(ptr, nbytes, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def host_mappings():
    """(live mappings as dicts, hipHostRegister calls made, calls that covered a byte outside
    their caller range)."""
    cap = 256
    buf = (HostMapping * cap)()
    cnt, regs, out = ctypes.c_size_t(), ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().hydra_host_mappings(buf, cap, ctypes.byref(cnt), ctypes.byref(regs),
                                    ctypes.byref(out)))
    live = [{f: getattr(buf[i], f) for f, _ in HostMapping._fields_}
            for i in range(min(cnt.value, cap))]
    return live, regs.value, out.value


LINK_TYPES = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}


def device_links(device: int = 0) -> list:
    """hydra_device_link from `device` to every other visible device: link type, hops, peer
    access (an empty list on a one-GPU box)."""
    import torch

    out = []
    for q in range(torch.cuda.device_count()):
        if q == device:
            continue
        t, h, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().hydra_device_link(device, q, ctypes.byref(t), ctypes.byref(h),
                                      ctypes.byref(c)))
        out.append({"peer": q, "link": LINK_TYPES.get(t.value, t.value), "hops": h.value,
                    "peer_access": bool(c.value)})
    return out


def set_variant(v: int) -> int:
    """hydra_set_variant of the measurement build (measure_lib()); returns the previous value."""
    return measure_lib().hydra_set_variant(v)


# hydra_test_key_t (include/hydra_hip.h): test switches, 0 in production
TEST_LOCAL_STAGE, TEST_RESIDENT_GEN_STRIDE, TEST_RESIDENT_REGRESSIONS = 1, 2, 3


def test_set(key: int, value: int) -> int:
    """hydra_test_set: sets a test switch, returns its previous value."""
    prev = ctypes.c_int64()
    check(lib().hydra_test_set(key, value, ctypes.byref(prev)))
    return prev.value


def test_get(key: int) -> int:
    v = ctypes.c_int64()
    check(lib().hydra_test_get(key, ctypes.byref(v)))
    return v.value
