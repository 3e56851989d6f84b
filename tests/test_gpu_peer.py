"""Peer-access allreduce (hydra_peer_*): P real processes, each mapping the others' buckets by
hipIpc handles, one kernel per allreduce reading the peers' data directly.  On the one-GPU box
all ranks share cuda:0 (IPC across processes on one device: the same handles, signal flags,
system-scope fences and per-workgroup barriers the xGMI node uses).  Bar: bit-exact vs the
reference ring (oracle) for every Gloo element type (fp32 and fp64 on fold-order-sensitive
inputs, full-range integers that wrap, float16 with its store quirk) and hydra's bf16; bf16 with
fp32 accumulation bit-exact vs the reference ring's fp32 fold + one rounding on config 5's
order-sensitive values (plus a tolerance check on plain uniform values)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from hydra_amd import _lib, synth
from peer_worker import inputs

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "peer_worker.py")


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(tmp_path, P, cases, blocks=64, timeout=150, arena_bytes=64 << 20):
    cpath = tmp_path / "cases.json"
    cpath.write_text(json.dumps(cases))
    port = free_port()
    procs = []
    for r in range(P):
        cmd = [sys.executable, "-u", WORKER, "--rank", str(r), "--world", str(P), "--port",
               str(port), "--out", str(tmp_path), "--cases", str(cpath), "--blocks", str(blocks),
               "--arena-bytes", str(arena_bytes)]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      start_new_session=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append(out.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, 9)
                p.wait()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} rc={p.returncode}\n{o[-3000:]}"
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(P)]
    st = [json.loads((tmp_path / f"status{r}.json").read_text()) for r in range(P)]
    return res, st


def f16_inputs(P, n):
    rng = [np.random.default_rng(1000 + r) for r in range(P)]
    return [g.uniform(-4, 4, n).astype(np.float16).view(np.uint16).copy() for g in rng]


def expected(O, c, P):
    n = c["n"]
    if c["data"] == "stress_f32":
        xs = [synth.stress_f32(P, r, n) for r in range(P)]
        return O.ring_result(xs, c.get("ms") or (1 << 20), kind=c.get("op", "sum")).view(np.uint8)
    if c["data"] == "int32":
        xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        return O.ring_result(xs, c.get("ms") or (1 << 20), kind=c.get("op", "sum")).view(np.uint8)
    if c["data"] == "f16":
        return O.ring_result(f16_inputs(P, n), c.get("ms") or (1 << 20),
                             dtype_code=_lib.FLOAT16).view(np.uint8)
    if c["data"] in ("typed", "bf16_native"):  # the worker's own generator, the oracle's ring
        code = c["dtype"] if c["data"] == "bf16_native" else None
        xs = [inputs(c, P, r) for r in range(P)]
        return O.ring_result(xs, c.get("ms") or (1 << 20), kind=c.get("op", "sum"),
                             dtype_code=code).view(np.uint8)
    if c["data"] == "bf16_cancel":  # the reference ring's fp32 fold on the widened values,
        # bf16 block geometry, one RNE rounding (tests/fold_expect.py, pinned in test_oracle.py)
        from fold_expect import bf16_acc32_expected

        exp, _, _ = bf16_acc32_expected(O, P, n, np.arange(n, dtype=np.int64),
                                        c.get("ms") or (1 << 20))
        return exp.view(np.uint8)
    raise ValueError(c["data"])


def cases_for(P):
    F32, I32, F16, BF16 = _lib.FLOAT32, _lib.INT32, _lib.FLOAT16, _lib.BFLOAT16
    cs = []
    for algo in ("peer2", "peer2w", "peer1"):
        for n, ms, off in ((1, 0, 0), (7, 0, 4), (1000, 128, 0), (4099, 128, 12),
                           (262145, 0, 0), (1 << 20, 0, 4), (3000001, 0, 0)):
            if algo == "peer1" and n > (1 << 20):
                continue
            cs.append(dict(name=f"{algo}_f32_{n}_{ms}_{off}", algo=algo, data="stress_f32",
                           dtype=F32, n=n, ms=ms, offset_bytes=off))
    cs.append(dict(name="peer2_i32", algo="peer2", data="int32", dtype=I32, n=100003, ms=4096,
                   offset_bytes=8))
    cs.append(dict(name="peer2w_i32", algo="peer2w", data="int32", dtype=I32, n=100003, ms=4096,
                   offset_bytes=8))
    cs.append(dict(name="peer2w_f16", algo="peer2w", data="f16", dtype=F16, n=20011, ms=1024,
                   offset_bytes=2))
    cs.append(dict(name="peer1_i32", algo="peer1", data="int32", dtype=I32, n=100003, ms=4096))
    cs.append(dict(name="peer2_f16", algo="peer2", data="f16", dtype=F16, n=20011, ms=1024,
                   offset_bytes=2))
    cs.append(dict(name="peer1_f16", algo="peer1", data="f16", dtype=F16, n=20011, ms=1024))
    for op in ("max", "min", "product"):
        for algo in ("peer2", "peer2w"):
            cs.append(dict(name=f"{algo}_{op}", algo=algo, data="stress_f32", dtype=F32,
                           n=70001, ms=4096, op=op))
    cs.append(dict(name="auto_small", algo="peer", data="stress_f32", dtype=F32, n=5000))
    cs.append(dict(name="repeat", algo="peer2", data="stress_f32", dtype=F32, n=262147,
                   repeat=25))
    cs.append(dict(name="graph2", algo="peer2", data="stress_f32", dtype=F32, n=300007,
                   graph=True))
    cs.append(dict(name="graph2w", algo="peer2w", data="stress_f32", dtype=F32, n=300007,
                   graph=True))
    # buckets at different addresses mod 16 on different ranks: the push cannot store at the
    # local alignment everywhere, so every rank runs the pull schedule instead (same bits)
    cs.append(dict(name="peer2w_rank_shift", algo="peer2w", data="stress_f32", dtype=F32,
                   n=262147, rank_shift=4))
    cs.append(dict(name="auto_rank_shift", algo="peer", data="stress_f32", dtype=F32,
                   n=(1 << 20) + 1, rank_shift=8))
    cs.append(dict(name="repeat2w", algo="peer2w", data="stress_f32", dtype=F32, n=262147,
                   repeat=25))
    cs.append(dict(name="graph1", algo="peer1", data="int32", dtype=I32, n=30011, ms=4096,
                   graph=True))
    cs.append(dict(name="stress2", algo="peer2", data="stress", dtype=F32, n=200003, iters=40,
                   offset_bytes=4))
    cs.append(dict(name="stress1", algo="peer1", data="stress", dtype=F32, n=50021, iters=40))
    cs.append(dict(name="stress2w", algo="peer2w", data="stress", dtype=F32, n=200003, iters=40,
                   offset_bytes=4))
    # calls on two streams with no ordering between them: serialized by the library
    cs.append(dict(name="streams2", algo="peer2", data="streams", dtype=F32, n=100003, iters=8))
    cs.append(dict(name="streams1", algo="peer1", data="streams", dtype=F32, n=30011, iters=8))
    cs.append(dict(name="streams2w", algo="peer2w", data="streams", dtype=F32, n=100003,
                   iters=8))
    cs.append(dict(name="bf16_acc32", algo="peer2", data="bf16", dtype=BF16, n=1 << 20,
                   flags=_lib.ACC_F32))
    # config 5's arithmetic bit-exact: fold-order-sensitive bf16 values, fp32 accumulation in
    # the reference order, one rounding (both schedules; 2P-misaligned sizes, small segments)
    for algo, n, ms, off in (("peer2", (1 << 20) + 3, 0, 2), ("peer2", 100003, 4096, 0),
                             ("peer2w", (1 << 20) + 3, 0, 2), ("peer1", 30011, 1024, 6)):
        cs.append(dict(name=f"{algo}_bf16_acc32_cancel_{n}", algo=algo, data="bf16_cancel",
                       dtype=BF16, n=n, ms=ms, offset_bytes=off, flags=_lib.ACC_F32))
    # every other element type the kernels instantiate, both schedules
    for nm, npt, code in (("i8", "int8", _lib.INT8), ("u8", "uint8", _lib.UINT8),
                          ("i64", "int64", _lib.INT64), ("u64", "uint64", _lib.UINT64),
                          ("f64", "float64", _lib.FLOAT64)):
        for algo, n, ms, off in (("peer2", 65543, 4096, 8), ("peer2w", 65543, 4096, 8),
                                 ("peer1", 4099, 128, 0)):
            cs.append(dict(name=f"{algo}_{nm}_{n}", algo=algo, data="typed", np=npt, dtype=code,
                           n=n, ms=ms, offset_bytes=off))
    cs.append(dict(name="peer2_i8_max", algo="peer2", data="typed", np="int8", dtype=_lib.INT8,
                   n=70001, ms=4096, op="max"))
    cs.append(dict(name="peer2_u64_min", algo="peer2", data="typed", np="uint64",
                   dtype=_lib.UINT64, n=30011, ms=4096, op="min"))
    cs.append(dict(name="peer2_f64_product", algo="peer2", data="typed", np="float64",
                   dtype=_lib.FLOAT64, n=30011, ms=4096, op="product"))
    cs.append(dict(name="peer2_bf16_native", algo="peer2", data="bf16_native", dtype=BF16,
                   n=100003, ms=4096, offset_bytes=2))
    cs.append(dict(name="peer2w_bf16_native", algo="peer2w", data="bf16_native", dtype=BF16,
                   n=100003, ms=4096, offset_bytes=2))
    cs.append(dict(name="peer1_bf16_native", algo="peer1", data="bf16_native", dtype=BF16,
                   n=20011, ms=1024))
    cs.append(dict(name="reregister", algo="peer2", data="reregister", dtype=F32,
                   n=(1 << 20) + 3, iters=12))
    return cs


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_peer_allreduce_bit_exact(gpu, O, tmp_path, P):
    cases = cases_for(P)
    res, st = run_ranks(tmp_path, P, cases)
    for c in cases:
        name = c["name"]
        assert all(s[name] == 0 for s in st), (name, st)
        if c["data"] in ("stress", "reregister", "streams"):  # checked word by word in every rank
            continue
        if c["data"] == "bf16":
            n = c["n"]
            xs = [synth.bf16_bits(synth.uniform_f32(n, 100 + r) * 4) for r in range(P)]
            vals = np.stack([synth.bf16_to_f32(x).astype(np.float64) for x in xs])
            exact = vals.sum(0)
            tol = np.abs(exact) * 2.0 ** -8 + P * 2.0 ** -24 * np.abs(vals).sum(0) + 1e-30
            got = synth.bf16_to_f32(res[0][name].view(np.uint16)).astype(np.float64)
            assert np.all(np.abs(got - exact) <= tol), name
            assert all(np.array_equal(r[name], res[0][name]) for r in res), name
            continue
        exp = expected(O, c, P)
        for r in range(P):
            assert np.array_equal(res[r][name], exp), (name, r)


def test_peer_default_grid(gpu, O, tmp_path):
    """The derived grid (one workgroup per 64 KiB slab, up to 256 per rank) at P = 2."""
    P = 2
    cases = [dict(name="big", algo="peer2", data="stress_f32", dtype=_lib.FLOAT32,
                  n=(8 << 20) + 5, ms=0, offset_bytes=4)]
    res, st = run_ranks(tmp_path, P, cases, blocks=0)
    exp = expected(O, cases[0], P)
    assert all(np.array_equal(r["big"], exp) for r in res)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_peer_config4_full_size_order_sensitive(gpu, O, tmp_path, P):
    """BASELINE config 4 at its full size through the peer-access kernel --
    P ranks x 64 Mi fp32 of fold-order-sensitive values (synth.stress_at, generated on the GPU),
    every rank's whole bucket (sha256 of its bytes) equal to the C restatement of the reference
    ring (O.ring_result), for both two-shot schedules (pull and push: the ones the N>1 line may
    promote) and the one-shot one.  Reference geometry at this size: 256 segments of 1 MiB, S = 256/P per rank
    (allreduce.cc:212-221, 253-258): S = 128 / 64 / 32 at P = 2 / 4 / 8.  The ranks share the
    one GPU, so each rank's grid is 512 / P workgroups (all of them resident at once)."""
    import hashlib

    import torch

    from fold_expect import device_bucket

    n = 64 << 20
    ns, sb, S = O.ring_plan(P, n, 4)
    assert (ns, sb, S) == (256, 1 << 20, 256 // P)
    F32 = _lib.FLOAT32
    cases = [dict(name=f"{a}_full", algo=a, data="full_stress", dtype=F32, n=n)
             for a in ("peer2", "peer2w", "peer1")]
    res, st = run_ranks(tmp_path, P, cases, blocks=512 // P, timeout=240,
                        arena_bytes=4 * n)
    xs = [device_bucket(synth.stress_at, P, r, n, gpu, torch.float32).cpu().numpy()
          for r in range(P)]
    want = O.ring_result(xs)
    if P > 2:  # the data can tell fold orders apart: a plain left fold differs on many
        # elements (at P = 2 every order is the one commutative sum x_0 + x_1)
        left = xs[0].copy()
        for x in xs[1:]:
            left += x
        assert float(np.mean(left.view(np.uint32) != want.view(np.uint32))) > 0.1
        del left
    digest = hashlib.sha256(want.tobytes()).hexdigest()
    del xs, want
    for c in cases:
        for r in range(P):
            assert st[r][c["name"]] == 0, (c["name"], r, st[r])
            assert st[r][c["name"] + "#sha256"] == digest, (c["name"], r)


def test_peer_config5_full_size_sampled(gpu, O, tmp_path):
    """BASELINE config 5 at its full size through the peer-access kernel --
    8 ranks x 256 Mi bf16 with fp32 accumulation (HYDRA_ACC_F32) on synth.stress_cancel_at
    (+-2^k pivots that cancel, so the one bf16 rounding does not hide the fp32 fold order), both
    two-shot schedules (pull, push); >= 1 Mi sampled elements of every rank (every segment boundary, random ones) equal
    the C restatement's fold on the widened values with the bf16 geometry (512 segments of 1 MiB,
    S = 64 per rank), rounded once."""
    from fold_expect import bf16_acc32_expected, sample_indices

    P, n = 8, 256 << 20
    ns, sb, S = O.ring_plan(P, n, 2)
    assert (ns, sb, S) == (512, 1 << 20, 64)
    idx = sample_indices(n, ns, sb // 2)
    ipath = tmp_path / "idx.npy"
    np.save(ipath, idx)
    cases = [dict(name=f"{a}_bf16_full", algo=a, data="full_cancel_bf16",
                  dtype=_lib.BFLOAT16, n=n, flags=_lib.ACC_F32, idx_file=str(ipath))
             for a in ("peer2", "peer2w")]
    res, st = run_ranks(tmp_path, P, cases, blocks=512 // P, timeout=240, arena_bytes=2 * n)
    exp, vals, _ = bf16_acc32_expected(O, P, n, idx)
    left = synth.bf16_to_f32(vals[0]).astype(np.float32)
    for v in vals[1:]:
        left = O.acc_bf16_f32(left, v)
    assert float(np.mean(synth.bf16_bits(left) != exp)) > 0.3  # the check sees fold orders
    for c in cases:
        for r in range(P):
            assert st[r][c["name"]] == 0, (r, st[r])
            got = res[r][c["name"]]
            bad = np.flatnonzero(got != exp)
            assert bad.size == 0, (c["name"], r, bad.size, idx[bad[:5]].tolist())


@pytest.mark.parametrize("P", [4, 8])
def test_peer_colocated_grid_rule(gpu, O, tmp_path, P):
    """ranks of one group on the same GPU (every rank here shares cuda:0)
    must all have their grids resident at once.  The library knows which ranks share a GPU (the
    PCI identity travels in the signal handle) and enforces it: an explicit grid of 512
    workgroups at P = 4 / 8 is refused at once (HYDRA_ERR_INVALID, no barrier timeout), one that
    fits (512 / P) is accepted, and the derived grid (blocks = 0: up to 256 per rank with a GPU
    each) shrinks to fit -- an 8 Mi+5 bucket, which round 5's r05e session saw time out at P = 4,
    completes bit-exact."""
    cases = [dict(name="too_many", data="set_blocks", blocks=512),
             dict(name="fits", data="set_blocks", blocks=512 // P),
             dict(name="derived", algo="peer2", data="stress_f32", dtype=_lib.FLOAT32,
                  n=(8 << 20) + 5, ms=0, offset_bytes=4)]
    res, st = run_ranks(tmp_path, P, cases, blocks=0, timeout=120)
    for r in range(P):
        msg = st[r]["too_many"]
        assert msg.startswith("refused in ") and "resident capacity" in msg, msg
        assert float(msg.split()[2]) < 1.0, msg  # immediately, not after a barrier timeout
        assert st[r]["fits"] == "accepted", st[r]
        assert st[r]["derived"] == 0, st[r]
    exp = expected(O, cases[2], P)
    assert all(np.array_equal(r["derived"], exp) for r in res)


def test_peer_timeout_reports_and_poisons(gpu, tmp_path):
    """A rank that never arrives: the kernel leaves after the timeout (every wave drains), the
    error word is set, and the group refuses further allreduces."""
    cases = [dict(name="lonely", algo="peer2", data="stress_f32", dtype=_lib.FLOAT32, n=4096,
                  skip_rank=1, timeout_ms=300)]
    _, st = run_ranks(tmp_path, 2, cases)
    assert st[0]["lonely"] != 0
    assert "timed out" in st[0]["lonely/next"]


@pytest.mark.parametrize("P,n", [(2, 1000003), (3, 4099)])
def test_peer_from_c(gpu, P, n):
    """The C-ABI alone (tests/cpp/peer_capi.c: fork, pipes for the handle blobs, hydra_malloc /
    hydra_peer_* / hydra_stream_*), as a C caller such as the reference's benchmark wires it."""
    exe = os.path.join(ROOT, "tests", "cpp", "peer_capi")
    assert os.path.exists(exe), "built by hydra_amd/csrc/Makefile (hydra_amd._lib.build())"
    r = subprocess.run([exe, str(P), str(n)], capture_output=True, timeout=120)
    out = r.stdout.decode() + r.stderr.decode()
    assert r.returncode == 0, out
    assert f"peer_capi P={P} n={n}: ok" in out


@pytest.mark.parametrize("P,n", [(2, 1000003), (4, 262147)])
def test_peer_algorithm_class_cpp(gpu, tmp_path, P, n):
    """hydra::PeerAllreduce<T> (include/hydra/peer_allreduce.h) from C++ over the host runtime's
    FileStore + TCP rendezvous (tests/cpp/peer_algo.cc): fp32 and int32, changing inputs every
    run, every word exact on every rank."""
    exe = os.path.join(ROOT, "tests", "cpp", "peer_algo")
    assert os.path.exists(exe), "built by hydra_amd/csrc/Makefile (hydra_amd._lib.build())"
    r = subprocess.run([exe, str(P), str(n), str(tmp_path)], capture_output=True, timeout=150)
    out = r.stdout.decode() + r.stderr.decode()
    assert r.returncode == 0, out
    assert f"peer_algo P={P} n={n}: ok" in out


def test_register_refuses_a_changed_allocation(gpu):
    """Register once: a peer group refuses to export an address whose allocation
    changed since it was exported (freed and reallocated without hydra_peer_close), and accepts
    it again once the old registration is closed.  A 1-rank group in this process; the check
    needs a NEW allocation at the freed address: hydra_free keeps the block in hydra's cache
    (the same allocation comes back, which is safe), so the cache is trimmed first and a
    same-size hipMalloc then hands the address back."""
    import ctypes

    L = _lib.lib()
    h = ctypes.c_void_p()
    sig = ctypes.create_string_buffer(_lib.PEER_HANDLE_BYTES)
    _lib.check(L.hydra_peer_create(1, 0, 0, ctypes.byref(h), sig))
    try:
        _lib.check(L.hydra_peer_connect(h, sig))
        nbytes = 64 << 20
        _lib.check(L.hydra_cache_trim())  # nothing else kept: a's address is the one freed below
        a = ctypes.c_void_p()
        _lib.check(L.hydra_malloc(0, nbytes, ctypes.byref(a)))
        blob = ctypes.create_string_buffer(_lib.PEER_HANDLE_BYTES)
        _lib.check(L.hydra_peer_register(h, a, nbytes, blob))
        _lib.check(L.hydra_peer_open(h, a, nbytes, blob))
        _lib.check(L.hydra_peer_register(h, a, nbytes, blob))  # same allocation again: fine
        _lib.check(L.hydra_free(a))
        _lib.check(L.hydra_cache_trim())  # really free it
        b = ctypes.c_void_p()
        _lib.check(L.hydra_malloc(0, nbytes, ctypes.byref(b)))
        reused = b.value == a.value
        rc = L.hydra_peer_register(h, b, nbytes, blob)
        if reused:
            assert rc == _lib.ERR_INVALID, "a changed allocation at a registered address"
            assert b"changed" in L.hydra_last_error()
        _lib.check(L.hydra_peer_close(h, a))  # the old registration released ...
        _lib.check(L.hydra_peer_register(h, b, nbytes, blob))  # ... the new one is accepted
        _lib.check(L.hydra_free(b))
        if not reused:
            pytest.skip("allocator did not reuse the address; refusal not exercised")
    finally:
        L.hydra_peer_detach(h)
        L.hydra_peer_destroy(h)
