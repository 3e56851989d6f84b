"""hydra's process-wide caches of streams, events, device and pinned blocks
(hydra_amd/csrc/resource_cache.cpp, include/hydra_hip.h): a release keeps the object for the
next request of the same kind, size class and device; hydra_cache_trim really releases
everything kept; a released block is never handed out while work enqueued before its release
may still use it."""
import ctypes

import numpy as np
import pytest

from hydra_amd import _lib

pytestmark = pytest.mark.gpu


def _malloc(L, nbytes):
    p = ctypes.c_void_p()
    _lib.check(L.hydra_malloc(0, nbytes, ctypes.byref(p)))
    return p


def test_blocks_streams_events_are_reused_and_trimmed(gpu):
    L = _lib.lib()
    _lib.check(L.hydra_cache_trim())
    a = _malloc(L, 3 << 20)
    _lib.check(L.hydra_free(a))
    b = _malloc(L, (3 << 20) - 100)  # same 64 KiB size class
    assert b.value == a.value
    c = _malloc(L, 5 << 20)  # another size class: a different block
    assert c.value != b.value
    for p in (b, c):
        _lib.check(L.hydra_free(p))

    h = ctypes.c_void_p()
    _lib.check(L.hydra_malloc_host(1 << 20, ctypes.byref(h)))
    _lib.check(L.hydra_free_host(h))
    h2 = ctypes.c_void_p()
    _lib.check(L.hydra_malloc_host(1 << 20, ctypes.byref(h2)))
    assert h2.value == h.value
    _lib.check(L.hydra_free_host(h2))

    s = ctypes.c_void_p()
    _lib.check(L.hydra_stream_create(0, ctypes.byref(s)))
    e = ctypes.c_void_p()
    _lib.check(L.hydra_event_create(ctypes.byref(e)))
    _lib.check(L.hydra_event_record(e, s))
    _lib.check(L.hydra_event_destroy(e))
    e2 = ctypes.c_void_p()
    _lib.check(L.hydra_event_create(ctypes.byref(e2)))
    assert e2.value == e.value
    _lib.check(L.hydra_event_destroy(e2))
    _lib.check(L.hydra_stream_destroy(s))
    s2 = ctypes.c_void_p()
    _lib.check(L.hydra_stream_create(0, ctypes.byref(s2)))
    assert s2.value == s.value
    _lib.check(L.hydra_stream_destroy(s2))

    _lib.check(L.hydra_cache_trim())
    _lib.check(L.hydra_device_check(0))


def test_released_block_waits_for_pending_work(gpu):
    """A block released while a long reduce still writes it comes back only after that reduce:
    the next owner's bytes are never overwritten by the previous owner's kernel."""
    import torch

    L = _lib.lib()
    n = 32 << 20
    nbytes = 4 * n
    p = _malloc(L, nbytes)
    s = ctypes.c_void_p()
    _lib.check(L.hydra_stream_create(0, ctypes.byref(s)))
    ones = torch.ones(n, dtype=torch.float32, device=gpu)
    torch.cuda.synchronize()
    for _ in range(8):  # queue a few hundred microseconds of writes into p on stream s
        _lib.check(L.hydra_reduce(0, 6, p, ones.data_ptr(), ones.data_ptr(), n, s))
    _lib.check(L.hydra_free(p))  # returns only once the device is drained
    q = _malloc(L, nbytes)
    assert q.value == p.value
    zero = np.zeros(n, np.float32)
    _lib.check(L.hydra_memcpy(q, zero.ctypes.data, nbytes))
    back = np.empty(n, np.float32)
    _lib.check(L.hydra_memcpy(back.ctypes.data, q, nbytes))
    assert not back.any()
    _lib.check(L.hydra_free(q))
    _lib.check(L.hydra_stream_destroy(s))


def test_double_release_is_refused(gpu):
    """Releasing a kept block / stream / event again fails (hipErrorInvalidValue) instead of
    freeing what the cache would hand out next; the cache stays consistent."""
    L = _lib.lib()
    p = _malloc(L, 1 << 20)
    _lib.check(L.hydra_free(p))
    assert L.hydra_free(p) != 0
    q = _malloc(L, 1 << 20)
    assert q.value == p.value  # still handed out once, and only once
    r = _malloc(L, 1 << 20)
    assert r.value != q.value
    for x in (q, r):
        _lib.check(L.hydra_free(x))
    s = ctypes.c_void_p()
    _lib.check(L.hydra_stream_create(0, ctypes.byref(s)))
    _lib.check(L.hydra_stream_destroy(s))
    assert L.hydra_stream_destroy(s) != 0
    e = ctypes.c_void_p()
    _lib.check(L.hydra_event_create(ctypes.byref(e)))
    _lib.check(L.hydra_event_destroy(e))
    assert L.hydra_event_destroy(e) != 0
    _lib.check(L.hydra_device_check(0))


def test_invalid_device_is_refused_and_current_device_kept(gpu):
    """hydra_malloc / hydra_stream_create on a device that does not exist fail (nothing is
    handed out on another device instead), and neither call changes the caller's current
    device."""
    import torch

    L = _lib.lib()
    before = torch.cuda.current_device()
    p = ctypes.c_void_p()
    assert L.hydra_malloc(99, 1 << 20, ctypes.byref(p)) != 0
    s = ctypes.c_void_p()
    assert L.hydra_stream_create(99, ctypes.byref(s)) != 0
    assert torch.cuda.current_device() == before
    L.hydra_device_check(0)  # collects the refused calls' (non-sticky) last error
    q = _malloc(L, 1 << 20)  # the device the caller is on still works
    _lib.check(L.hydra_free(q))
    assert torch.cuda.current_device() == before
    _lib.check(L.hydra_device_check(0))


def test_fault_ledger_names_blocks_and_registrations(gpu, host_buf):
    """The fault report's ledger (hydra_fault_lookup): a live cache block, a host range registered
    by hydra_host_register and, once released, the same range as RELEASED; a report for torch's
    own memory.  Nothing faults here: the report is read directly."""
    import torch

    L = _lib.lib()
    p = _malloc(L, 3 << 20)
    r = _lib.fault_lookup(p.value + 4096)
    assert "device block" in r and "LIVE" in r, r
    _lib.check(L.hydra_free(p))
    h = host_buf(1 << 20, np.float32, 0)
    _lib.check(L.hydra_host_register(h.ctypes.data, h.nbytes))
    lo, _ = _lib.page_interior(h.ctypes.data, h.nbytes)  # only whole pages inside are registered
    try:
        r = _lib.fault_lookup(lo + 100)
        assert "hydra_host_register" in r and "LIVE" in r, r
    finally:
        _lib.check(L.hydra_host_unregister(h.ctypes.data))
    r = _lib.fault_lookup(lo + 100)
    assert "hydra_host_register" in r and "RELEASED" in r, r
    t = torch.empty(1 << 20, device=gpu)
    r = _lib.fault_lookup(t.data_ptr())
    assert "mapped" in r, r  # a well-formed report for device memory too
    assert _lib.fault_last()[2] == 0  # no fault seen in this process


def test_host_register_is_reference_counted(gpu, host_buf):
    """Two owners of one buffer each register and unregister it: the registration lives until the
    last unregister (the fault ledger shows it LIVE, then RELEASED); a second register may not
    cover more bytes than the first; unregistering an unknown address is a no-op."""
    L = _lib.lib()
    h = host_buf(1 << 20, np.float32, 0)
    p = h.ctypes.data
    _lib.check(L.hydra_host_register(p, h.nbytes))
    _lib.check(L.hydra_host_register(p, h.nbytes // 2))  # a second owner, a shorter range: fine
    assert L.hydra_host_register(p, h.nbytes + 4096) == _lib.ERR_INVALID
    _lib.check(L.hydra_host_unregister(p))
    lo, _ = _lib.page_interior(p, h.nbytes)  # the registration: the whole pages inside h
    assert "LIVE" in _lib.fault_lookup(lo), _lib.fault_lookup(lo)  # the first owner still holds it
    # and it is still what hydra_reduce_host streams in place: same bits as the oracle
    from hydra_amd.reduce import HostContext

    b = np.ones(h.size, np.float32)
    ctx = HostContext(0)
    try:
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, p, p, b.ctypes.data, h.size))
    finally:
        ctx.close()
    assert (h == 1).all()
    _lib.check(L.hydra_host_unregister(p))
    assert "RELEASED" in _lib.fault_lookup(lo), _lib.fault_lookup(lo)
    _lib.check(L.hydra_host_unregister(p))  # nothing left to release: no-op
    x = np.zeros(16, np.float32)
    _lib.check(L.hydra_host_unregister(x.ctypes.data))
