"""GPU checks of which host pages hydra maps for the kernel (hydra_amd/csrc/host_map.h).

Round 2's late device faults all surfaced in pageable copies above 1 MiB, the path on which the
HIP runtime locks the caller's pages page-rounded; hydra then registered sub-page operand ranges
per call (whose pages it shares with its neighbours).  These tests pin the replacement rules:
  * every registration hydra makes covers whole pages strictly inside its operand;
  * hydra's own registrations never overlap, and a call whose operand lies inside another call's
    pin references that pin, so the pin outlives both kernels;
  * the mechanism itself, run deterministically: register / pin sub-page ranges, release, free,
    reallocate at the same address, then torch's pageable >1 MiB copies (runtime locking path,
    tests/conftest.py no longer routes them through staging buffers) -- bytes exact, no fault.
All results are bit-exact against the oracle's restatement of gloo::sum<T> (math.h:15-23)."""
import ctypes
import os
import threading

import numpy as np
import pytest

from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext

pytestmark = pytest.mark.gpu

PAGE = os.sysconf("SC_PAGESIZE")
libc = ctypes.CDLL(None)
libc.malloc.restype = ctypes.c_void_p
libc.malloc.argtypes = [ctypes.c_size_t]
libc.free.argtypes = [ctypes.c_void_p]


def bits(x):
    return np.ascontiguousarray(x).view(f"u{x.itemsize}")


def f32_at(addr, n):
    return np.ctypeslib.as_array((ctypes.c_float * n).from_address(addr))


def inside_own_pages(m):
    """A registration (kind 1 / 2) covers whole pages inside the range it was made for."""
    return (m["lo"] % PAGE == 0 and m["hi"] % PAGE == 0 and m["owner_lo"] <= m["lo"]
            and m["hi"] <= m["owner_hi"])


def live_registrations():
    live, regs, outside = _lib.host_mappings()
    assert outside == 0, "a registration covered bytes outside its operand"
    return [m for m in live if m["kind"] in (_lib.MAP_REGISTER, _lib.MAP_PIN)], regs


@pytest.fixture
def ctx(gpu):
    c = HostContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("off,nelem", [(4, 1), (100, 1000), (4092, 1025), (8, 3 * 1024 + 5),
                                       (0, 4096), (2052, (1 << 18) + 3)])
def test_host_register_maps_only_interior_pages(ctx, O, off, nelem):
    """hydra_host_register of a misaligned range registers the whole pages inside it, nothing
    else; the call that uses it reduces the interior zero-copy and stages the ragged edges --
    bits exact, every byte around the operands untouched."""
    L = _lib.lib()
    registered = False
    size = off + 4 * nelem + 2 * PAGE
    base = libc.malloc(size)
    other = libc.malloc(4 * nelem + 64)
    try:
        raw = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(base))
        raw[:] = 0xA5
        a = f32_at(base + off, nelem)
        a[:] = synth.stress_f32(2, 0, nelem)
        b = f32_at(other, nelem)
        b[:] = synth.stress_f32(2, 1, nelem)
        exp = O.op(a.copy(), b.copy(), "sum", 6)
        _lib.check(L.hydra_host_register(base + off, 4 * nelem))
        registered = True
        regs, _ = live_registrations()
        mine = [m for m in regs if m["owner_lo"] == base + off]
        lo, hi = _lib.page_interior(base + off, 4 * nelem)
        if lo == hi:
            assert not mine
        else:
            assert len(mine) == 1 and (mine[0]["lo"], mine[0]["hi"]) == (lo, hi)
            assert inside_own_pages(mine[0])
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, base + off, base + off, other, nelem))
        assert np.array_equal(bits(a), bits(exp))
        assert (raw[:off] == 0xA5).all() and (raw[off + 4 * nelem:] == 0xA5).all()
        registered = False
        _lib.check(L.hydra_host_unregister(base + off))
        regs, _ = live_registrations()
        assert not [m for m in regs if m["owner_lo"] == base + off]
    finally:
        if registered:  # never free registered pages (a stale registration poisons the address)
            L.hydra_host_unregister(base + off)
        libc.free(other)
        libc.free(base)


@pytest.mark.parametrize("n", [1, 1000, 1025, 262144 + 7, (3 << 20) + 11])
@pytest.mark.parametrize("offs", [(0, 0, 0), (4, 8, 12), (4092, 2048, 100)])
def test_per_call_pins_stay_inside_operands(ctx, O, n, offs):
    """Pageable operands at odd offsets: each call pins only whole pages inside each operand,
    releases every pin before it returns, and the result is bit-exact (zero-copy interior, staged
    edges), in place and out of place."""
    L = _lib.lib()
    _, regs0 = live_registrations()
    bufs = [libc.malloc(4 * n + o + 64) for o in offs]
    try:
        c, a, b = (f32_at(p + o, n) for p, o in zip(bufs, offs))
        x, y = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)
        exp = O.op(x, y, "sum", 6)
        a[:], b[:], c[:] = x, y, 7
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, c.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        assert np.array_equal(bits(c), bits(exp))
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        assert np.array_equal(bits(a), bits(exp))
        regs, regs1 = live_registrations()
        assert not [m for m in regs if m["kind"] == _lib.MAP_PIN], "a per-call pin outlived its call"
        if 4 * n >= 3 * PAGE:
            assert regs1 > regs0, "pageable operands were not pinned"
    finally:
        for p in bufs:
            libc.free(p)


def test_operand_inside_another_calls_pin(ctx, O):
    """Two threads: one reduces a 48 MiB pageable operand (its interior pinned for the call, a
    ~10 ms kernel over PCIe), the other keeps reducing small operands that lie inside that pin.
    The second thread's calls reference the first one's pin instead of mapping the pages
    themselves, so no pin is released under a running kernel: every result exact, no fault, no
    pin left behind (round 2 advisor: mapped_device_range accepted another thread's pin)."""
    L = _lib.lib()
    n = 12 << 20
    big_b = synth.stress_f32(2, 1, n)
    big_a = synth.stress_f32(2, 0, n)
    exp_big = O.op(big_a, big_b, "sum", 6)
    m = 5000
    offs = [1, 40_000, 1 << 20, (7 << 20) + 3, n - m - 1]
    small_a = synth.stress_f32(3, 2, m)
    exp_small = {o: O.op(small_a, big_b[o:o + m], "sum", 6) for o in offs}
    errors = []
    stop = threading.Event()

    def big():
        ctx2 = HostContext(0)
        try:
            for _ in range(6):
                c = np.empty(n, np.float32)
                rc = L.hydra_reduce_host(ctx2.handle, 0, 6, c.ctypes.data, big_a.ctypes.data,
                                         big_b.ctypes.data, n)
                if rc:
                    errors.append(("big", L.hydra_last_error()))
                    return
                if not np.array_equal(bits(c), bits(exp_big)):
                    errors.append(("big", "mismatch"))
                    return
        finally:
            stop.set()
            ctx2.close()

    t = threading.Thread(target=big)
    t.start()
    k = 0
    while not stop.is_set() or k < len(offs):
        o = offs[k % len(offs)]
        c = np.empty(m, np.float32)
        rc = L.hydra_reduce_host(ctx.handle, 0, 6, c.ctypes.data, small_a.ctypes.data,
                                 big_b[o:].ctypes.data, m)
        if rc:
            errors.append(("small", L.hydra_last_error()))
            break
        if not np.array_equal(bits(c), bits(exp_small[o])):
            errors.append(("small", o))
            break
        k += 1
    t.join()
    assert not errors, errors
    regs, _ = live_registrations()
    assert not [r for r in regs if r["kind"] == _lib.MAP_PIN]


def test_release_free_realloc_then_pageable_copies(ctx, O, gpu):
    """The suspected mechanism, run deterministically once: sub-page registrations and per-call
    pins of operands inside a malloc'd block, released, the block freed (munmap: it is above the
    mmap threshold) and reallocated -- the allocator hands back the same address -- then torch's
    pageable copies of >1 MiB in both directions over those pages (the runtime's page-locking
    copy path).  Every byte round-trips, and the device stays healthy."""
    import torch

    L = _lib.lib()
    size = (6 << 20) + 123
    addrs = []
    for rnd in range(3):
        registered = False
        base = libc.malloc(size)
        addrs.append(base)
        try:
            raw = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(base))
            raw[:] = rnd
            # a registration of a sub-page-aligned range and per-call pins of odd operands
            _lib.check(L.hydra_host_register(base + 100, (1 << 20) + 10))
            registered = True
            n = 300_001
            a = f32_at(base + 4 + (2 << 20), n)
            b = f32_at(base + 40 + (4 << 20), n)
            a[:], b[:] = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)
            exp = O.op(a.copy(), b.copy(), "sum", 6)
            _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                           b.ctypes.data, n))
            assert np.array_equal(bits(a), bits(exp))
            registered = False
            _lib.check(L.hydra_host_unregister(base + 100))
            regs, _ = live_registrations()
            assert not [r for r in regs if base <= r["lo"] < base + size]
        finally:
            if registered:
                L.hydra_host_unregister(base + 100)
            libc.free(base)
        # reallocated (same address on glibc) and copied through torch's pageable path
        again = libc.malloc(size)
        try:
            view = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(again))
            pat = (np.arange(size, dtype=np.uint32) * 2654435761 >> 13).astype(np.uint8)
            view[:] = pat
            for lo, cnt in ((0, size), (77, (2 << 20) + 5), (4096 * 3 + 1, 3 << 20)):
                d = torch.from_numpy(view[lo:lo + cnt]).to(gpu)
                back = d.cpu().numpy()
                assert np.array_equal(back, pat[lo:lo + cnt])
                d.add_(1)
                view[lo:lo + cnt] = d.cpu().numpy()  # D2H into the reallocated pages
                assert np.array_equal(view[lo:lo + cnt], (pat[lo:lo + cnt] + 1).astype(np.uint8))
                view[lo:lo + cnt] = pat[lo:lo + cnt]
            torch.cuda.synchronize()
        finally:
            libc.free(again)
    _lib.check(L.hydra_device_check(0))
