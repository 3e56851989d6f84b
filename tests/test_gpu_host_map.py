"""GPU checks of which host pages hydra maps for the kernel (hydra_amd/csrc/host_map.h).

Round 3 caught the late device fault of rounds 1-2 with its address
(profiles/r03_fault_report.txt): a torch pageable H2D copy above 1 MiB -- the HIP runtime's
page-locking copy path -- faulted on heap pages that hydra had pinned per call (hipHostRegister /
hipHostUnregister) 47 s earlier, after the allocator had handed them out again.  hydra therefore
no longer registers host memory on its own.  These tests pin the rules that replace it:
  * pageable operands are never registered: the CPU copies them through pinned staging;
  * hydra_host_register covers whole pages strictly inside its range, the ragged edges staged;
  * a call holding a window on a registration keeps it mapped even when its owner unregisters
    meanwhile (round 2 advisor: one thread's operand inside another thread's mapping).
Only host memory from the session pool (tests/conftest.py host_buf) is ever registered here: its
pages never return to the allocator, so no pageable copy can land on them later.  (The fault
itself is not re-run: reproducing GPU faults is not allowed on this pool, and the evidence is
the report.)  All results are bit-exact against the oracle's gloo::sum<T> (math.h:15-23)."""
import ctypes
import os
import threading
import time

import numpy as np
import pytest

from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

PAGE = os.sysconf("SC_PAGESIZE")


def bits(x):
    return np.ascontiguousarray(x).view(f"u{x.itemsize}")


def f32_at(raw, off, n):
    """n fp32 at byte offset `off` of the uint8 array `raw`."""
    return raw[off:off + 4 * n].view(np.float32)


def live_registrations():
    live, regs, outside = _lib.host_mappings()
    assert outside == 0, "a registration covered bytes outside its range"
    return [m for m in live if m["kind"] in (_lib.MAP_REGISTER, _lib.MAP_PIN)], regs


@pytest.fixture
def ctx(gpu):
    c = HostContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("off,nelem", [(4, 1), (100, 1000), (4092, 1025), (8, 3 * 1024 + 5),
                                       (0, 4096), (2052, (1 << 18) + 3)])
def test_host_register_maps_only_interior_pages(ctx, O, off, nelem, host_buf):
    """hydra_host_register of a misaligned range registers the whole pages inside it, nothing
    else; the call that uses it reduces the interior zero-copy and stages the ragged edges --
    bits exact, every byte around the operands untouched."""
    L = _lib.lib()
    size = off + 4 * nelem + 2 * PAGE
    raw = host_buf(size, np.uint8, 0xA5)
    a = f32_at(raw, off, nelem)
    a[:] = synth.stress_f32(2, 0, nelem)
    b = host_buf(nelem, np.float32, synth.stress_f32(2, 1, nelem))
    exp = O.op(a.copy(), b.copy(), "sum", 6)
    p = raw.ctypes.data + off
    _lib.check(L.hydra_host_register(p, 4 * nelem))
    try:
        regs, _ = live_registrations()
        mine = [m for m in regs if m["owner_lo"] == p]
        lo, hi = _lib.page_interior(p, 4 * nelem)
        if lo == hi:
            assert not mine
        else:
            assert len(mine) == 1 and (mine[0]["lo"], mine[0]["hi"]) == (lo, hi), mine
            assert mine[0]["lo"] % PAGE == 0 and mine[0]["hi"] % PAGE == 0
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, p, p, b.ctypes.data, nelem))
        assert np.array_equal(bits(a), bits(exp))
        assert (raw[:off] == 0xA5).all() and (raw[off + 4 * nelem:] == 0xA5).all()
    finally:
        _lib.check(L.hydra_host_unregister(p))
    regs, _ = live_registrations()
    assert not [m for m in regs if m["owner_lo"] == p]


@pytest.mark.parametrize("n", [1, 1000, 1025, 262144 + 7, (3 << 20) + 11, (9 << 20) + 1])
@pytest.mark.parametrize("offs", [(0, 0, 0), (4, 8, 12), (4092, 2048, 100)])
def test_pageable_operands_are_never_registered(ctx, O, n, offs):
    """Pageable operands at odd offsets, in place and out of place, more than one staging round
    at the largest size: hydra makes no host registration at all (the registration counter does
    not move), and the result is bit-exact."""
    L = _lib.lib()
    live0, regs0 = live_registrations()
    bufs = [np.empty(n + o // 4 + 16, np.float32) for o in offs]
    c, a, b = (buf.view(np.uint8)[o:o + 4 * n].view(np.float32) for buf, o in zip(bufs, offs))
    x, y = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)
    exp = O.op(x, y, "sum", 6)
    a[:], b[:], c[:] = x, y, 7
    _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, c.ctypes.data, a.ctypes.data,
                                   b.ctypes.data, n))
    assert np.array_equal(bits(c), bits(exp))
    _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                   b.ctypes.data, n))
    assert np.array_equal(bits(a), bits(exp))
    live1, regs1 = live_registrations()
    assert regs1 == regs0 and len(live1) == len(live0), (regs0, regs1)


def test_window_outlives_an_unregister_by_its_owner(ctx, O, host_buf):
    """One thread keeps reducing segments of a registered 16 MiB bucket (zero-copy windows on the
    registration) while the owner unregisters it: calls in flight keep their window -- the pages
    stay registered until the last one ends -- and calls after that stage; every result exact,
    nothing left registered."""
    L = _lib.lib()
    n = 4 << 20
    bucket = host_buf(n, np.float32, synth.stress_f32(2, 0, n))
    orig = bucket.copy()
    m = 262144
    y = synth.stress_f32(2, 1, m)
    _lib.check(L.hydra_host_register(bucket.ctypes.data, bucket.nbytes))
    errors, done = [], []
    go = threading.Event()

    def worker():
        ctx2 = HostContext(0)
        try:
            go.set()
            for k in range(48):
                o = (k * 7919 * 64) % (n - m)
                out = np.empty(m, np.float32)
                rc = L.hydra_reduce_host(ctx2.handle, 0, 6, out.ctypes.data,
                                         bucket[o:].ctypes.data, y.ctypes.data, m)
                if rc:
                    errors.append(L.hydra_last_error())
                    return
                if not np.array_equal(bits(out), bits(O.op(orig[o:o + m], y, "sum", 6))):
                    errors.append(("mismatch", k))
                    return
                done.append(k)
        finally:
            ctx2.close()

    t = threading.Thread(target=worker)
    t.start()
    go.wait()
    while len(done) < 8 and t.is_alive():
        time.sleep(0.0002)
    _lib.check(L.hydra_host_unregister(bucket.ctypes.data))  # while calls are in flight
    t.join()
    assert not errors, errors
    assert len(done) == 48
    regs, _ = live_registrations()
    lo, hi = bucket.ctypes.data, bucket.ctypes.data + bucket.nbytes
    assert not [r for r in regs if lo <= r["lo"] < hi], regs


_STAGED_RESULT = r"""
import ctypes, json, sys, numpy as np
sys.path.insert(0, %r)
import torch
from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext
from oracle import oracle as O
L = _lib.lib()
c = HostContext(0)
for k, v in %r.items():
    c.set_option(k, v)
out = {}
n = 300007
buf = np.empty(n + 4096, np.float32)  # lives until exit: registered pages never go back
x = buf[1000:1000 + n]
_lib.check(L.hydra_host_register(x.ctypes.data, x.nbytes))
for mode, (cc, aa) in {"in_place": ("x", "x"), "out_of_place": ("y", "x")}.items():
    x[:] = synth.stress_f32(2, 0, n)
    b = synth.stress_f32(2, 1, n)
    exp = O.op(x.copy(), b, "sum", 6)
    y = np.zeros(n, np.float32) if cc == "y" else x
    _lib.check(L.hydra_host_trace(1))
    _lib.check(L.hydra_reduce_host(c.handle, 0, 6, y.ctypes.data, x.ctypes.data, b.ctypes.data, n))
    _lib.check(L.hydra_host_trace(0))
    rec = (_lib.HostCall * 4)()
    cnt = ctypes.c_size_t()
    _lib.check(L.hydra_host_trace_read(rec, 4, ctypes.byref(cnt)))
    out[mode] = {"exact": bool(np.array_equal(y.view(np.uint32), exp.view(np.uint32))),
                 "calls": cnt.value, "zero_copy_c": rec[0].zero_copy_bytes[0],
                 "zero_copy_a": rec[0].zero_copy_bytes[1], "staged_c": rec[0].staged_bytes[0]}
_lib.check(L.hydra_host_unregister(x.ctypes.data))
c.close()
print(json.dumps(out))
"""


@pytest.mark.parametrize("opts,staged", [
    ({}, True),  # default: a 1.2 MiB registration is below HYDRA_OPT_STAGE_RESULT_REG_MAX (8 MiB)
    ({_lib.OPT_STAGE_RESULT_REG_MAX: 0}, False),  # zero-copy result writes
    ({_lib.OPT_STAGE_RESULT_REG_MAX: 0, _lib.OPT_STAGE_RESULT_MAX: 1 << 30}, True),
])
def test_staged_result_path_choice(gpu, opts, staged):
    """Where a registered c's result goes: through the staging (the CPU copies it back, c stays
    in the CPU's cache) for a small registration -- the default -- or written in place over PCIe.
    The same bits either way, in place (c == a, the ring's call) and out of place; a's interior
    pages are read in place in every case."""
    import json
    import subprocess
    import sys

    p = subprocess.run([sys.executable, "-c", _STAGED_RESULT % (ROOT, opts)],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    for mode, v in r.items():
        assert v["exact"] and v["calls"] == 1, (mode, v)
        assert v["zero_copy_a"] > 0, (mode, v)  # the interior pages of a are read in place
    if staged:
        assert r["in_place"]["zero_copy_c"] == 0, r
        assert r["in_place"]["staged_c"] == 300007 * 4, r
    else:
        assert r["in_place"]["zero_copy_c"] > 0, r


def test_register_release_reuse_then_pageable_copies(gpu):
    """the sequence profiles/r03_fault_report.txt points at, made
    deterministic -- pages registered with hydra_host_register and used zero-copy by a kernel,
    unregistered, unmapped, then FRESH pages mapped at the very same virtual addresses
    (MAP_FIXED_NOREPLACE) and copied by the HIP runtime's pageable copy path (torch H2D of 8 MiB,
    which locks the caller's pages, and D2H back into them).  No fault, no stale data: round 4's
    probe ran 200 cycles clean (profiles/r04c2_register_reuse_probe.log), which refutes this
    sequence as a deterministic cause; this test keeps 40 cycles of it in the suite."""
    import json
    import subprocess
    import sys

    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "probe_register_reuse.py"),
                        "40", "8"], capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["cycles"] == 40 and r["n_mismatches"] == 0 and r["gpu_faults_seen"] == 0, r
