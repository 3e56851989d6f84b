"""The drop-in proven inside the reference itself (tests/cpp/dropin_gloo.cc): the REFERENCE's own
gloo::allreduce ring (allreduce.cc:147-422) and old-style gloo::AllreduceRing<T>
(allreduce_ring.h:20-125), compiled from its sources into oracle/_ref, run twice on identical
inputs -- once with gloo::sum<T> / ReductionFunction<T>::sum, once with libhydra_hip.so's gfx950
chunk-sum plugged into AllreduceOptions::setReduceFunction (allreduce.h:36,179-181) and into
AllreduceRing<T>'s ReductionFunction<T>* (algorithm.h:59-96) through include/hydra/gloo_reduce.h.
Bar: every byte of every rank identical (fp32 on fold-order-sensitive inputs, int32).

The new-style ring's scratch is the reference's own pageable `new uint8_t[]` (allreduce.cc:225),
so the plug-in is the host-buffer Func (hostSum: staged H2D -> kernel -> D2H); a device-buffer
Func (deviceSum) has no reference caller that hands it device memory -- the CUDA-workspace
classes that would are CUDA sources, unbuildable here."""
import json
import os
import subprocess

import pytest

from hydra_amd import _lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "dropin_gloo")


def dropin(mode, P, n, dt="f32", iters=0, ms=0, timeout=240, register=False, env_extra=None):
    assert os.path.exists(EXE), "built with the reference by oracle/Makefile (build())"
    args = [EXE, mode, str(P), str(n), dt, str(iters)] + ([str(ms)] if ms else [])
    env = dict(os.environ, HYDRA_DROPIN_REGISTER="1" if register else "0", **(env_extra or {}))
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


NEW_CASES = [(P, n, ms) for P in (2, 3, 4, 8) for (n, ms) in
             [(1, 0), (100, 128), (4099, 128), (262145, 0), (1 << 20, 0)]] + \
            [(2, 4 << 20, 0), (4, 4 << 20, 0), (8, 4 << 20, 0), (3, 3000001, 0)]


@pytest.mark.parametrize("P,n,ms", NEW_CASES)
def test_reference_allreduce_ring_with_hydra_func(gpu, P, n, ms):
    j = dropin("new_ring", P, n, ms=ms)
    assert j["mismatched_bytes"] == 0, j
    assert j["fnv_ref"] == j["fnv_hydra"]
    assert j["ref_ranks_equal"]  # the reference ring leaves every rank with the same bits


@pytest.mark.parametrize("P,n", [(2, 100003), (3, 1 << 20), (8, 262147)])
def test_reference_allreduce_ring_with_hydra_func_int32(gpu, P, n):
    j = dropin("new_ring", P, n, dt="i32")
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("P,n,dt", [(2, 1, "f32"), (3, 100, "f32"), (4, 4099, "f32"),
                                    (8, 1000, "f32"), (5, 1 << 20, "f32"), (3, 4099, "i32"),
                                    (8, 262147, "i32")])
def test_reference_allreduce_ring_old_with_hydra_reduction_function(gpu, P, n, dt):
    """old-style AllreduceRing<T>: every rank folds in its own order (ranks may differ in the
    last bits), so the bar is rank-by-rank identity with the reference's own run."""
    j = dropin("old_ring", P, n, dt=dt)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("P,n,ms", [(2, 1001, 128), (3, 262147, 0), (4, 1 << 20, 0)])
def test_reference_allreduce_two_pointers_with_hydra_func(gpu, P, n, ms):
    """Two local pointers per rank: the Func also pre-reduces the local inputs
    (genLocalReduceFunction, allreduce.cc:46-83) before the ring; both outputs of every rank."""
    j = dropin("new_ring2", P, n, ms=ms)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("P,n,ms,dt", [(2, 100, 128, "f32"), (3, 4099, 128, "f32"),
                                       (4, 1 << 20, 0, "f32"), (7, 262147, 0, "f32"),
                                       (3, 100003, 4096, "i32")])
def test_reference_reduce_with_hydra_func(gpu, P, n, ms, dt):
    """gloo::reduce to the last rank (reduce.cc:21-262), the Func's other new-style caller
    (reduce.cc:195, out of place): every rank's bytes, the non-roots' partial sums included."""
    j = dropin("new_reduce", P, n, dt=dt, ms=ms)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("P,n,dt", [(2, 1, "f32"), (3, 1000, "f32"), (5, 4099, "f32"),
                                    (8, 1 << 20, "f32"), (4, 100003, "i32")])
def test_reference_allreduce_ring_chunked_with_hydra_reduction_function(gpu, P, n, dt):
    """old-style AllreduceRingChunked<T> (allreduce_ring_chunked.h:20-248) with the hydra
    ReductionFunction<T>, incl. partial and empty chunks."""
    j = dropin("old_ring_chunked", P, n, dt=dt)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("n", [16 << 20, 64 << 20])
def test_config1_full_size_inside_the_reference(gpu, n):
    """BASELINE config 1 at its top sizes (new_allreduce_ring, fp32, 2 ranks, loopback TCP):
    the reference's ring with the hydra Func equals the reference's ring with gloo::sum<float>
    byte for byte at 16 Mi and 64 Mi elements (the published row is README.md:86)."""
    j = dropin("new_ring", 2, n, iters=1, timeout=600)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("result_path", ["default", "in_place", "staged"])
@pytest.mark.parametrize("mode,P,n", [("new_ring", 2, 1 << 20), ("new_ring", 3, 4099),
                                      ("new_ring2", 2, 262147), ("old_ring", 4, 100003),
                                      ("new_ring", 2, (4 << 20) + 3)])
def test_reference_with_hydra_func_registered_bucket(gpu, mode, P, n, result_path):
    """The bucket registered once (hydra_host_register): the kernel reads it in place over PCIe
    while only the reference's pageable scratch is staged, and writes its results either in place
    (registrations above 8 MiB -- the last case's 16 MiB bucket -- or always with the option
    HYDRA_OPT_STAGE_RESULT_REG_MAX = 0) or through the staging (smaller ones, or always): same
    bytes."""
    opt = {"default": "", "in_place": f"{_lib.OPT_STAGE_RESULT_REG_MAX}=0",
           "staged": f"{_lib.OPT_STAGE_RESULT_MAX}={1 << 30}"}[result_path]
    env = {"HYDRA_DROPIN_OPT": opt} if opt else {}
    j = dropin(mode, P, n, register=True, env_extra=env)
    assert j["mismatched_bytes"] == 0, j


@pytest.mark.parametrize("mode,P,n,ms", [("new_ring", 2, 100, 128), ("new_ring", 3, 4099, 0),
                                         ("new_ring", 8, 262147, 0), ("new_ring2", 3, 20011, 1024),
                                         ("new_reduce", 4, 30011, 4096),
                                         ("old_ring", 3, 4099, 0), ("old_ring", 5, 100003, 0),
                                         ("old_ring_chunked", 4, 20011, 0)])
def test_reference_float16_with_hydra(gpu, mode, P, n, ms):
    """gloo::float16 inside the reference: its sum<float16> stores through float16::operator=,
    whose `if (rhs != *this)` compares the new value with the OLD bits read as an integer
    (types.h:112-130) -- the store quirk.  The hydra plug-ins (hostReduce(SUM, FLOAT16) as the
    Func, gpuReductionFunctionAs<..., HYDRA_FLOAT16> as the ReductionFunction) reproduce it in
    every call site: in-place ring hops, the two-pointer local reduce, gloo::reduce's out-of-place
    form and the old-style rings."""
    j = dropin(mode, P, n, dt="f16", ms=ms)
    assert j["mismatched_bytes"] == 0, j


def test_shim_failures_are_gloos_own_exception_types(gpu):
    """include/hydra/gloo_errors.h: an invalid call inside the reference's gloo::allreduce (the
    hydra Func with an element type the library rejects, run by allreduce's local reduce,
    allreduce.cc:46-83, 129-133) leaves it as gloo::EnforceNotMet (common/logging.h:21,42) -- the
    type a reference caller already catches -- and a valid call on the same context then still
    sums; the timeout status maps to gloo::IoException (common/error.h:45)."""
    j = dropin("errors", 1, 1000)
    assert j["invalid_call"] == "gloo::EnforceNotMet", j
    assert "invalid dtype" in j["invalid_msg"], j
    assert j["valid_after"] == "none" and j["valid_sum_ok"], j
    assert j["timeout_status"] == "gloo::IoException", j
