"""The resident reducer (hydra_amd/csrc/resident.h): hydra_reduce_host's low-latency form for
the reference ring's synchronous per-segment Func (allreduce.cc:301-305) -- one persistent
launch per device per process, host contexts on leased slots.  Bit-exact against the
reference's own outputs (golden fixtures: every Gloo dtype x {sum, product, max, min}) and the
oracle, through every lifecycle edge: back-to-back calls on one instance, idle gaps long enough
for an instance to leave (the next call launches a new one), two contexts at once, more
contexts than slots, a context destroyed while the instance runs, calls of several staging
rounds, HYDRA_OPT_RESIDENT = 0 -- and the persistent grid never holds up another stream's work."""
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest

from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TYPES = [("i8", 0, np.int8), ("u8", 1, np.uint8), ("i32", 2, np.int32), ("u32", 3, np.uint32),
         ("i64", 4, np.int64), ("u64", 5, np.uint64), ("f32", 6, np.float32),
         ("f64", 7, np.float64), ("f16", 8, np.uint16)]
OPC = {"sum": 0, "product": 1, "max": 2, "min": 3}


def bits(x):
    return np.ascontiguousarray(x).view(f"u{x.itemsize}")


@pytest.fixture
def ctx(gpu):
    c = HostContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("name,code,dt", TYPES)
def test_resident_golden_ops(ctx, golden, name, code, dt):
    """The reference's own sum/product/max/min<T> outputs (tests/golden, incl. inf/NaN/-0/
    subnormal/overflow), in place c == a as the ring calls it, every one served resident."""
    L = _lib.lib()
    s0 = ctx.stats()
    for kind in OPC:
        if name == "i32" and kind == "product":
            a, b = golden[f"ops_{name}_pa"], golden[f"ops_{name}_pb"]
        else:
            a, b = golden[f"ops_{name}_a"], golden[f"ops_{name}_b"]
        exp = golden[f"ops_{name}_{kind}"]
        c = np.ascontiguousarray(a.copy())
        _lib.check(L.hydra_reduce_host(ctx.handle, OPC[kind], code, c.ctypes.data, c.ctypes.data,
                                       np.ascontiguousarray(b).ctypes.data, a.size))
        assert np.array_equal(bits(c), bits(exp)), (name, kind)
    s1 = ctx.stats()
    assert s1["resident_calls"] > s0["resident_calls"], (s0, s1)


def test_resident_back_to_back_and_idle_gaps(ctx, O):
    """200 synchronous calls of ragged sizes on pageable buffers, with gaps of 0, 1 and 6 ms
    (past the 2 ms idle limit: the instance leaves and the next call starts a new one) --
    every result bit-exact; more than one instance was launched, far fewer than calls."""
    L = _lib.lib()
    rng = np.random.default_rng(5)
    s0 = ctx.stats()
    for i in range(200):
        n = int(rng.integers(1, 70000))
        a = synth.stress_f32(2, 0, n, seed=i)
        b = synth.stress_f32(2, 1, n, seed=i)
        exp = O.op(a, b, "sum", 6)
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        assert np.array_equal(bits(a), bits(exp)), (i, n)
        if i % 50 == 49:
            time.sleep(0.006)
        elif i % 10 == 9:
            time.sleep(0.001)
    st = ctx.stats()
    # (a staged call of more than 256 KiB per operand is served as 2+ rounds: HYDRA_OPT_STAGE_SPLIT)
    assert 200 <= st["resident_calls"] - s0["resident_calls"] < 400, (s0, st)
    assert 2 <= st["resident_launches"] - s0["resident_launches"] < 60, (s0, st)


def test_resident_two_contexts_concurrently(gpu, O):
    """Two threads, one context (one slot of the device's resident reducer) each -- the two
    rails of bew_allreduce_a (pipeallreduce-a.cc:32-50) -- 300 calls each, every result exact."""
    L = _lib.lib()
    errs = []

    def rail(r):
        c = HostContext(0)
        try:
            for i in range(300):
                n = 1000 + 37 * i + r
                a = synth.stress_f32(3, r, n, seed=i)
                b = synth.stress_f32(3, r + 1, n, seed=i)
                exp = O.op(a, b, "sum", 6)
                rc = L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                         b.ctypes.data, n)
                if rc or not np.array_equal(bits(a), bits(exp)):
                    errs.append((r, i, rc))
                    return
        finally:
            c.close()

    ts = [threading.Thread(target=rail, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs


def test_resident_destroy_while_running(gpu, O):
    """A context destroyed right after a call (the instance still waiting for the next one)
    gives its slot back; a new context takes it at once and its calls are served."""
    L = _lib.lib()
    for k in range(5):
        c = HostContext(0)
        n = 4099 + k
        a, b = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)
        exp = O.op(a, b, "sum", 6)
        _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        c.close()
        assert np.array_equal(bits(a), bits(exp))
    _lib.check(L.hydra_device_check(0))


def _with_opts(code, opts):
    """`code` run after hydra_set_option(key, value) for each of `opts` (library options: the
    library reads no environment variable)."""
    pre = ("import sys; sys.path.insert(0, %r)\nimport torch\nfrom hydra_amd import _lib\n"
           "for _k, _v in %r.items():\n    _lib.set_option(_k, _v)\n" % (ROOT, opts))
    return pre + code


def test_resident_per_context_options(gpu, O):
    """hydra_ctx_set_option (round 6): one context turns the resident reducer off (its slot is
    returned; every round becomes one launch on its stream) and cuts staged calls into more
    rounds, while a second context keeps the process-wide defaults -- same bits on both; the
    option comes back on for the first and it is served resident again.  Invalid keys / values
    are refused."""
    L = _lib.lib()
    a_ctx, b_ctx = HostContext(0), HostContext(0)
    try:
        a_ctx.set_option(_lib.OPT_RESIDENT, 0)
        a_ctx.set_option(_lib.OPT_STAGE_SPLIT, 16)
        for k, (c, n) in enumerate(((a_ctx, 3000), (b_ctx, 3000), (a_ctx, 2_000_003),
                                    (b_ctx, 2_000_003))):
            s0 = c.stats()
            x, y = synth.stress_f32(2, 0, n, seed=k), synth.stress_f32(2, 1, n, seed=k)
            e = O.op(x, y, "sum", 6)
            _lib.check(L.hydra_reduce_host(c.handle, 0, 6, x.ctypes.data, x.ctypes.data,
                                           y.ctypes.data, n))
            assert np.array_equal(bits(x), bits(e)), (k, n)
            served = c.stats()["resident_calls"] - s0["resident_calls"]
            assert (served == 0) if c is a_ctx else (served > 0), (k, served)
        a_ctx.set_option(_lib.OPT_RESIDENT, 1)  # leases a slot again
        s0 = a_ctx.stats()
        x, y = synth.stress_f32(2, 0, 5000), synth.stress_f32(2, 1, 5000)
        _lib.check(L.hydra_reduce_host(a_ctx.handle, 0, 6, x.ctypes.data, x.ctypes.data,
                                       y.ctypes.data, 5000))
        assert a_ctx.stats()["resident_calls"] > s0["resident_calls"]
        with pytest.raises(_lib.HydraError):
            a_ctx.set_option(_lib.OPT_COPY_THREADS, 2)  # process-wide only
        with pytest.raises(_lib.HydraError):
            a_ctx.set_option(_lib.OPT_STAGE_SPLIT, 0)
    finally:
        a_ctx.close()
        b_ctx.close()


def test_resident_off_by_option(gpu):
    """HYDRA_OPT_RESIDENT = 0 (process-wide): every call is one batched launch on the context's
    stream; same bits."""
    code = (
        "import sys, numpy as np; sys.path.insert(0, %r)\n"
        "import torch\n"
        "from hydra_amd import _lib, synth\n"
        "from hydra_amd.reduce import HostContext\n"
        "from oracle import oracle as O\n"
        "c = HostContext(0); L = _lib.lib()\n"
        "for n in (1, 1000, 262145):\n"
        "    a, b = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)\n"
        "    e = O.op(a, b, 'sum', 6)\n"
        "    _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,"
        " b.ctypes.data, n))\n"
        "    assert np.array_equal(a.view(np.uint32), e.view(np.uint32)), n\n"
        "assert c.stats()['resident_calls'] == 0, c.stats()\n"
        "c.close(); print('ok')\n" % ROOT)
    p = subprocess.run([sys.executable, "-c", _with_opts(code, {_lib.OPT_RESIDENT: 0})],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "ok" in p.stdout, (p.stdout, p.stderr[-2000:])


def test_resident_solo_and_spread_calls_across_instances(ctx, O, host_buf):
    """Small calls (<= 4 tiles: workgroup 0 alone, nothing published to the others) and larger
    ones (every workgroup) interleaved across instance restarts (idle gaps): a worker of a new
    instance must never take the publication an earlier instance left behind for a new call
    -- it would redo that old call on its old pointers.  The old call's output buffer is
    registered (kept mapped) and refilled with a canary afterwards: it must stay untouched."""
    L = _lib.lib()
    big = 40000  # 10 tiles: every workgroup
    old_c = host_buf(big, np.float32, 0)
    _lib.check(L.hydra_host_register(old_c.ctypes.data, old_c.nbytes))
    try:
        a0, b0 = synth.stress_f32(2, 0, big), synth.stress_f32(2, 1, big)
        _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, old_c.ctypes.data, a0.ctypes.data,
                                       b0.ctypes.data, big))
        assert np.array_equal(bits(old_c), bits(O.op(a0, b0, "sum", 6)))
        old_c[:] = np.float32(-7.0)  # canary
        for rnd in range(4):
            time.sleep(0.006)  # past the idle limit: the next call starts a new instance
            for i, n in enumerate((100, 3000, 4096, 50000, 17, 70001)):
                a = synth.stress_f32(2, 0, n, seed=rnd * 10 + i)
                b = synth.stress_f32(2, 1, n, seed=rnd * 10 + i)
                exp = O.op(a, b, "sum", 6)
                _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                               b.ctypes.data, n))
                assert np.array_equal(bits(a), bits(exp)), (rnd, n)
        _lib.check(L.hydra_device_check(0))
        assert (old_c == np.float32(-7.0)).all(), "an old call was redone on its old output"
    finally:
        _lib.check(L.hydra_host_unregister(old_c.ctypes.data))


_BLOCKING_PROBE = r"""
import json, sys, time, numpy as np
sys.path.insert(0, %r)
import torch
from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext
L = _lib.lib()
x = torch.zeros(1024, device="cuda")
streams = [torch.cuda.Stream() for _ in range(24)]  # more than the hardware queues per process
if len(sys.argv) > 1:  # (probe only) torch's high-priority pool as well
    streams += [torch.cuda.Stream(priority=-1) for _ in range(int(sys.argv[1]))]
torch.cuda.synchronize()
c = HostContext(0)
a, b = synth.stress_f32(2, 0, 5000), synth.stress_f32(2, 1, 5000)
_lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data, b.ctypes.data, 5000))
t_call = time.perf_counter()  # the instance now waits up to 1 s for the next call
lat = []
for s in streams:
    with torch.cuda.stream(s):
        t0 = time.perf_counter()
        x.add_(1)
        s.synchronize()
        lat.append(time.perf_counter() - t0)
t0 = time.perf_counter()
x.add_(1)  # the default (legacy null) stream
torch.cuda.default_stream().synchronize()
lat.append(time.perf_counter() - t0)
alive = time.perf_counter() - t_call
# (hipDeviceSynchronize waits for every grid on the device, the instance's too: not timed here)
print(json.dumps({"max_s": max(lat), "lat_ms": [round(v * 1e3, 3) for v in lat],
                  "elapsed_s": alive, "launches": c.stats()["resident_launches"]}))
c.close()
"""


def test_resident_instance_never_blocks_other_streams(gpu):
    """The persistent grid runs on a hardware queue of its own: with an instance alive (idle
    limit 1 s), a kernel on each of 24 fresh torch streams and on the default stream completes
    in milliseconds -- on a shared queue it would wait for the instance to leave."""
    import json

    p = subprocess.run([sys.executable, "-c",
                        _with_opts(_BLOCKING_PROBE % ROOT, {_lib.OPT_RESIDENT_IDLE_US: 1000000})],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["launches"] == 1, json.dumps(r)  # one instance stayed alive through the probe
    assert r["elapsed_s"] < 0.9, json.dumps(r)
    assert r["max_s"] < 0.1, json.dumps(r)


def test_resident_more_contexts_than_slots(gpu, O):
    """40 contexts on one device (the reducer has 32 slots, some perhaps held by other live
    contexts of this process): those beyond the free slots launch; every context's calls are
    exact, and a slot is free again once the contexts close."""
    L = _lib.lib()
    ctxs = [HostContext(0) for _ in range(40)]
    try:
        for k, c in enumerate(ctxs):
            n = 3000 + 517 * k
            a, b = synth.stress_f32(2, 0, n, seed=k), synth.stress_f32(2, 1, n, seed=k)
            exp = O.op(a, b, "sum", 6)
            _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                           b.ctypes.data, n))
            assert np.array_equal(bits(a), bits(exp)), k
        served = [c.stats()["resident_calls"] for c in ctxs]
        leased = sum(1 for v in served if v == 1)
        assert set(served) <= {0, 1} and 1 <= leased <= 32 and served.count(0) >= 8, served
        assert served == sorted(served, reverse=True), served  # the first ones got the slots
    finally:
        for c in ctxs:
            c.close()
    c = HostContext(0)
    try:
        a, b = synth.stress_f32(2, 0, 9000), synth.stress_f32(2, 1, 9000)
        exp = O.op(a, b, "sum", 6)
        _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, 9000))
        assert np.array_equal(bits(a), bits(exp))
        assert c.stats()["resident_calls"] == 1
    finally:
        c.close()


@pytest.mark.parametrize("n", [(4 << 20) // 4 + 1, 5 << 20, (17 << 20) // 4 + 3])
def test_resident_multi_round_calls(ctx, O, n):
    """Calls staging more than one round (4 MiB per operand): every round through the reducer,
    the CPU filling round r + 1 while round r runs; c == a and c distinct from a and b."""
    L = _lib.lib()
    a, b = synth.stress_f32(2, 0, n), synth.stress_f32(2, 1, n)
    exp = O.op(a, b, "sum", 6)
    s0 = ctx.stats()
    c = np.empty_like(a)
    _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, c.ctypes.data, a.ctypes.data,
                                   b.ctypes.data, n))
    assert np.array_equal(bits(c), bits(exp))
    _lib.check(L.hydra_reduce_host(ctx.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                   b.ctypes.data, n))
    assert np.array_equal(bits(a), bits(exp))
    rounds = ctx.stats()["resident_calls"] - s0["resident_calls"]
    assert rounds >= 2 * (-(-n * 4 // (4 << 20))), rounds


_SOLO_STREAM = r"""
import json, sys, time, numpy as np
sys.path.insert(0, %r)
import torch
from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext
from oracle import oracle as O
L = _lib.lib()
c = HostContext(0)
def call(n, seed):
    a, b = synth.stress_f32(2, 0, n, seed=seed), synth.stress_f32(2, 1, n, seed=seed)
    e = O.op(a, b, "sum", 6)
    _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data, b.ctypes.data, n))
    assert np.array_equal(a.view(np.uint32), e.view(np.uint32)), n
call(50000, 0)  # a published job: every worker has seen one
t0, k = time.perf_counter(), 0
while time.perf_counter() - t0 < 0.4:  # solo calls only (<= 4 tiles), well past idle + grace
    call(1000 + k %% 3000, k)
    k += 1
for i in range(3):  # then published jobs again: the workers must still be there
    call(50000 + 4097 * i, 100 + i)
st = c.stats()
c.close()
print(json.dumps({"solo_calls": k, "launches": st["resident_launches"]}))
"""


def test_resident_solo_calls_past_the_grace_period(gpu):
    """a steady stream of solo calls (workgroup 0 alone, nothing published)
    longer than idle + grace must not make the waiting workers give up -- they follow workgroup
    0's heartbeat -- and a large call afterwards is served by the same instance, exactly.
    Grace shortened to 20 ms and the idle limit to 50 ms (HYDRA_OPT_RESIDENT_GRACE_US / _IDLE_US):
    0.4 s of solo calls crosses idle + grace more than 5 times, and a scheduling hiccup shorter
    than 50 ms between two calls cannot end the instance."""
    import json

    p = subprocess.run([sys.executable, "-c",
                        _with_opts(_SOLO_STREAM % ROOT, {_lib.OPT_RESIDENT_GRACE_US: 20000,
                                                         _lib.OPT_RESIDENT_IDLE_US: 50000})],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout[-1000:], p.stderr[-3000:])
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["solo_calls"] > 100, r
    assert r["launches"] == 1, r  # one instance served everything: nobody left on an error


def test_resident_device_drains_are_bounded(gpu, O):
    """while another thread keeps the resident reducer busy with host calls,
    the library's own device-wide drains -- freeing a pinned block, trimming the caches,
    destroying a context, hydra_device_check -- stop the instance first instead of waiting for
    the calls to stop.  Each returns within 50 ms; every concurrent call stays bit-exact."""
    L = _lib.lib()
    stop = threading.Event()
    errs, calls = [], [0]

    def loop():
        c = HostContext(0)
        try:
            i = 0
            while not stop.is_set():
                n = (3000, 40000, 70001)[i % 3]
                a, b = synth.stress_f32(2, 0, n, seed=i), synth.stress_f32(2, 1, n, seed=i)
                exp = O.op(a, b, "sum", 6)
                rc = L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                         b.ctypes.data, n)
                if rc or not np.array_equal(bits(a), bits(exp)):
                    errs.append((i, rc, L.hydra_last_error()))
                    return
                i += 1
                calls[0] = i
        finally:
            c.close()

    import ctypes

    # (what earlier tests left in the caches is really freed first: unpinning gigabytes takes
    # time of its own, which is not a drain)
    _lib.check(L.hydra_cache_trim())
    th = threading.Thread(target=loop)
    th.start()
    times = {}
    try:
        time.sleep(0.2)
        for rep in range(3):
            p = ctypes.c_void_p()
            _lib.check(L.hydra_malloc_host(1 << 20, ctypes.byref(p)))
            t0 = time.perf_counter()
            _lib.check(L.hydra_free_host(p))
            times[f"free_pinned_{rep}"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            _lib.check(L.hydra_device_check(0))
            times[f"device_check_{rep}"] = time.perf_counter() - t0
            c2 = HostContext(0)
            t0 = time.perf_counter()
            c2.close()
            times[f"ctx_destroy_{rep}"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            _lib.check(L.hydra_cache_trim())
            times[f"cache_trim_{rep}"] = time.perf_counter() - t0
            time.sleep(0.05)
        n0 = calls[0]
        time.sleep(0.1)
        still_serving = calls[0] > n0
    finally:
        stop.set()
        th.join(timeout=60)
    assert not errs, errs
    assert still_serving and calls[0] > 50, calls
    slow = {k: round(v * 1e3, 2) for k, v in times.items() if v > 0.05}
    assert not slow, (slow, {k: round(v * 1e3, 2) for k, v in times.items()})


_GEN_WRAP = r"""
import ctypes, json, sys, time, numpy as np
sys.path.insert(0, %r)
import torch
from hydra_amd import _lib, synth
from hydra_amd.reduce import HostContext
from oracle import oracle as O
L = _lib.lib()
# every launch advances the generation by 2^16: the job word's 16-bit tag is the same for every
# instance, so only the zeroed device record keeps an old job word from a new instance's workers
_lib.test_set(_lib.TEST_RESIDENT_GEN_STRIDE, 65536)
blocks = []
def pinned(n, fill):
    p = ctypes.c_void_p()
    _lib.check(L.hydra_malloc_host(n * 4, ctypes.byref(p)))
    blocks.append(p)
    x = np.frombuffer((ctypes.c_char * (n * 4)).from_address(p.value), np.float32)
    x[:] = fill
    return x
c = HostContext(0)
big, G = 40000, 4096  # 10 tiles: a published job; guard elements on both sides
buf = pinned(big + 2 * G, np.float32(3.25))
guard = np.float32(3.25)
a0 = pinned(big, 0); a0[:] = synth.stress_f32(2, 0, big)
b0 = pinned(big, 0); b0[:] = synth.stress_f32(2, 1, big)
out0 = buf[G:G + big]
_lib.check(L.hydra_reduce_host(c.handle, 0, 6, out0.ctypes.data, a0.ctypes.data, b0.ctypes.data, big))
assert np.array_equal(out0.view(np.uint32), O.op(a0, b0, "sum", 6).view(np.uint32))
out0[:] = np.float32(-7.0)  # canary: a replay of the first job would rewrite it
l0 = c.stats()["resident_launches"]
calls = 0
for rnd in range(12):
    time.sleep(0.004)  # past the 300 us idle limit: the next call launches a new instance
    for i, n in enumerate((100, 3000, 50000, 17, 4096, 70001)):
        a = synth.stress_f32(2, 0, n, seed=rnd * 10 + i)
        b = synth.stress_f32(2, 1, n, seed=rnd * 10 + i)
        e = O.op(a, b, "sum", 6)
        _lib.check(L.hydra_reduce_host(c.handle, 0, 6, a.ctypes.data, a.ctypes.data,
                                       b.ctypes.data, n))
        assert np.array_equal(a.view(np.uint32), e.view(np.uint32)), (rnd, n)
        calls += 1
_lib.check(L.hydra_device_check(0))
res = {"calls": calls, "launches": c.stats()["resident_launches"] - l0,
       "canary_intact": bool((out0 == np.float32(-7.0)).all()),
       "guards_intact": bool((buf[:G] == guard).all() and (buf[G + big:] == guard).all()),
       "done_regressions": _lib.test_get(_lib.TEST_RESIDENT_REGRESSIONS),
       "gen_stride": _lib.test_get(_lib.TEST_RESIDENT_GEN_STRIDE)}
c.close()
for p in blocks:
    _lib.check(L.hydra_free_host(p))
print(json.dumps(res))
"""


def test_resident_generation_tag_wrap(gpu):
    """VERDICT r04 next #1 / ADVICE r04 (high): the job word carries 16 bits of the instance's
    generation.  With the test switch HYDRA_TEST_RESIDENT_GEN_STRIDE = 65536 every instance has
    the same tag, so a new instance's workers would take the job word the previous one published
    and replay its descriptor -- unless the device record is zeroed before every launch.  A
    published job, then 12 idle-outs, each followed by solo and spread calls on a new instance:
    every result bit-exact, the first job's output (pinned, still mapped) and the guard elements
    around it untouched, and no slot's completion word ever seen moving backwards."""
    import json

    p = subprocess.run([sys.executable, "-c",
                        _with_opts(_GEN_WRAP % ROOT, {_lib.OPT_RESIDENT_IDLE_US: 300})],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, (p.stdout[-1000:], p.stderr[-3000:])
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["gen_stride"] == 65536 and r["calls"] == 72, r
    assert r["launches"] >= 12, r  # every round ran on a fresh instance with the same tag
    assert r["canary_intact"] and r["guards_intact"], r
    assert r["done_regressions"] == 0, r
