"""The multi-GPU allreduce on one MI355X: hydra_allreduce_simulate runs every rank's plan with
the real HIP kernels and the real cross-stream event edges, device copies standing in for xGMI.
Bar: bit-exact vs the reference ring (oracle) for fp32/int32/f16; bf16 with fp32 accumulation
bit-exact vs the reference's own fp32 ring on the widened values + one RNE rounding (fixtures),
and within one bf16 rounding of the fp64 sum."""
import numpy as np
import pytest

from hydra_amd import _lib, ring, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm1(gpu):
    """One 1-rank RCCL communicator shared by the executor tests that leave it usable (a
    communicator per test would re-create RCCL's own buffers, streams and proxy thread each
    time).  Tests that abort a communicator or capture one build their own."""
    c = ring.XgmiComm(0, 1, gpu.index or 0, ring._rccl_unique_id())
    yield c
    c.close()


def dev_bufs(gpu, xs, view=None):
    import torch

    return [torch.from_numpy(x.view(view) if view else x.copy()).to(gpu) for x in xs]


@pytest.mark.parametrize("algo", ["ring", "direct"])
@pytest.mark.parametrize("P,n,ms,ch", [(2, 1, 0, 0), (2, 1000, 128, 256), (3, 4099, 128, 1024),
                                       (4, 262145, 0, 0), (5, 1 << 20, 0, 1 << 18),
                                       (8, 3000001, 0, 0), (8, 5003, 64, 128)])
def test_simulated_allreduce_f32(gpu, O, algo, P, n, ms, ch):
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate(bufs, algo=algo, max_segment=ms, chunk_bytes=ch)
    exp = O.ring_result(xs, ms or (1 << 20))
    for r in range(P):
        got = bufs[r].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (algo, P, n, r)


@pytest.mark.parametrize("algo", ["ring", "direct"])
def test_simulated_int32_f16(gpu, O, algo):
    import torch

    P, n = 4, 100003
    xs = [synth.int32_bucket(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate(bufs, algo=algo, max_segment=4096, chunk_bytes=8192)
    exp = O.ring_result(xs, 4096)
    assert all(np.array_equal(b.cpu().numpy(), exp) for b in bufs)
    rng = np.random.default_rng(4)
    hs = [np.array([O.f2h(float(v)) for v in rng.uniform(-4, 4, 20011)], np.uint16)
          for _ in range(P)]
    bufs = [torch.from_numpy(h.view(np.int16).copy()).to(gpu) for h in hs]
    ring.simulate(bufs, algo=algo, dtype_code=_lib.FLOAT16, max_segment=1024, chunk_bytes=2048)
    exp = O.ring_result(hs, 1024, dtype_code=8)
    assert all(np.array_equal(b.cpu().numpy().view(np.uint16), exp) for b in bufs)


def test_simulated_bf16_fp32_accumulate(gpu):
    """BASELINE config 5 building block: bf16 bucket, fp32 accumulation in the reference fold
    order, ONE rounding to bf16.  Tolerance: half a bf16 ulp of the fp64 sum plus the fp32
    accumulation error (P * 2^-24 * sum|x|)."""
    import torch

    P, n = 8, 1 << 20
    xs = [synth.bf16_bits(synth.uniform_f32(n, 100 + r) * 4) for r in range(P)]
    bufs = [torch.from_numpy(x.view(np.int16).copy()).to(gpu) for x in xs]
    ring.simulate(bufs, algo="direct", dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    vals = np.stack([synth.bf16_to_f32(x).astype(np.float64) for x in xs])
    exact = vals.sum(0)
    tol = np.abs(exact) * 2.0 ** -8 + P * 2.0 ** -24 * np.abs(vals).sum(0) + 1e-30
    for b in bufs:
        got = synth.bf16_to_f32(b.cpu().numpy().view(np.uint16)).astype(np.float64)
        assert np.all(np.abs(got - exact) <= tol)
    # and every rank holds the same bits
    ref0 = bufs[0].cpu().numpy()
    assert all(np.array_equal(b.cpu().numpy(), ref0) for b in bufs)


@pytest.fixture(scope="module")
def golden_bf16():
    import json
    import os

    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(g, "golden_bf16.json")) as f:
        meta = json.load(f)
    return np.load(os.path.join(g, "golden_bf16.npz"), allow_pickle=False), meta["cases"]


@pytest.mark.parametrize("algo", ["direct", "a2a"])
def test_simulated_bf16_acc32_vs_reference_ring(gpu, golden_bf16, algo):
    """Config 5's arithmetic pinned to the reference: the bf16 bucket folded with fp32
    accumulation (k_fold<bf16, ACC32>, DIRECT / A2A plans) equals, bit for bit, the reference's
    own gloo::allreduce RING run on the same values widened to fp32, rounded once (RNE) to bf16
    (tests/golden/golden_bf16.*, oracle/gen_golden.py --bf16): P = 2, 3, 4, 8."""
    import hashlib

    import torch

    npz, cases = golden_bf16
    for c in cases:
        P, n = c["P"], c["n"]
        xs = [synth.bf16_bits(synth.stress_f32(P, r, n)) for r in range(P)]
        assert hashlib.sha256(np.stack(xs).tobytes()).hexdigest() == c["inputs_sha256"]
        bufs = [torch.from_numpy(x.view(np.int16).copy()).to(gpu) for x in xs]
        ring.simulate(bufs, algo=algo, dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
        exp = npz[c["key"]]
        for r, b in enumerate(bufs):
            assert np.array_equal(b.cpu().numpy().view(np.uint16), exp), (algo, P, n, r)


def test_acc_f32_rejected_on_ring(gpu):
    import torch

    bufs = [torch.zeros(64, dtype=torch.int16, device=gpu) for _ in range(2)]
    with pytest.raises(_lib.HydraError):
        ring.simulate(bufs, algo="ring", dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)


def test_single_rank_comm(gpu):
    """RCCL loads inside libhydra_hip.so next to torch's, a 1-rank communicator initialises, and
    the P = 1 allreduce short-circuits (allreduce.cc:129-133)."""
    import torch

    uid = ring._rccl_unique_id()
    comm = ring.XgmiComm(0, 1, gpu.index or 0, uid)
    try:
        t = torch.arange(1000, dtype=torch.float32, device=gpu)
        comm.allreduce_(t)
        comm.allreduce_(t, algo="rccl")
        torch.cuda.synchronize()
        assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=gpu))
    finally:
        comm.close()


@pytest.mark.parametrize("op", ["sum", "product", "max", "min"])
@pytest.mark.parametrize("name,code,dt", [("i8", 0, np.int8), ("u64", 5, np.uint64),
                                          ("f64", 7, np.float64), ("f32", 6, np.float32)])
def test_simulated_ops_dtypes(gpu, O, op, name, code, dt):
    """Every op through both plans: the fold kernel and the ring hop keep the reference's
    c = op(local, received) order for product/max/min too."""
    import torch

    P, n = 3, 30011
    rng = np.random.default_rng(code * 7 + len(op))
    if np.issubdtype(dt, np.integer):
        xs = [rng.integers(-5 if dt == np.int8 else 0, 6, n).astype(dt) for _ in range(P)]
    else:
        xs = [rng.uniform(0.5, 1.5, n).astype(dt) for _ in range(P)]
    for algo in ("ring", "direct"):
        bufs = [torch.from_numpy(x.copy().view(np.uint8)).to(gpu) for x in xs]
        ring.simulate(bufs, algo=algo, op=op, dtype_code=code, max_segment=2048,
                      chunk_bytes=4096)
        outs = [[x.copy()] for x in xs]
        O.allreduce(P, outs, None, kind=op, dtype_code=code, max_segment=2048)
        for b in bufs:
            got = b.cpu().numpy().view(dt)
            assert np.array_equal(got.view(f"u{got.itemsize}"),
                                  outs[0][0].view(f"u{got.itemsize}")), (algo, op, name)


def test_allreduce_argument_checks(gpu, comm1):
    import torch

    t = torch.zeros(16, device=gpu)
    with pytest.raises(_lib.HydraError):
        comm1.allreduce_(t, dtype_code=42)
    with pytest.raises(_lib.HydraError):
        comm1.allreduce_(t, dtype_code=_lib.FLOAT32, flags=_lib.ACC_F32)


@pytest.mark.parametrize("P,n", [(2, 1 << 20), (4, 1 << 22), (8, 1 << 23), (8, 1 << 16)])
def test_simulated_a2a(gpu, O, P, n):
    """A2A (all-to-all + rank-ordered fold + all-gather) is bit-exact with the reference ring."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate(bufs, algo="a2a")
    exp = O.ring_result(xs)
    for r in range(P):
        assert np.array_equal(bufs[r].cpu().numpy().view(np.uint32), exp.view(np.uint32))


def test_simulated_a2a_bf16_acc32_matches_direct(gpu):
    """Same fold order => A2A and DIRECT give identical bits for the bf16/fp32-acc bucket."""
    import torch

    P, n = 8, 1 << 21
    xs = [synth.bf16_bits(synth.uniform_f32(n, 300 + r) * 3) for r in range(P)]
    a = [torch.from_numpy(x.view(np.int16).copy()).to(gpu) for x in xs]
    d = [torch.from_numpy(x.view(np.int16).copy()).to(gpu) for x in xs]
    ring.simulate(a, algo="a2a", dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    ring.simulate(d, algo="direct", dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    for r in range(P):
        assert torch.equal(a[r], d[r])


def test_a2a_rejects_unequal_blocks(gpu):
    import torch

    bufs = [torch.zeros(1001, device=gpu) for _ in range(3)]
    with pytest.raises(_lib.HydraError):
        ring.simulate(bufs, algo="a2a")


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("P", [1, 2, 5, 8, 16])
def test_fold_abi_reference_order(gpu, O, P, variant):
    """hydra_fold == the owner's P-1 in-place ring hops, every fold variant, ragged sizes and
    misaligned sources."""
    import ctypes

    import torch

    for n in (1, 13, 4099, 1 << 18):
        xs = [synth.stress_f32(P, r, n) for r in range(P)]
        bufs = [torch.from_numpy(np.concatenate([np.zeros(r % 4, np.float32), x])).to(gpu)
                for r, x in enumerate(xs)]
        ptrs = (ctypes.c_void_p * P)(*[b.data_ptr() + 4 * (r % 4) for r, b in enumerate(bufs)])
        dst = torch.zeros(n + 3, dtype=torch.float32, device=gpu)
        if variant:  # the fold variants live in the measurement build
            L = _lib.measure_lib()
            prev = L.hydra_set_variant(variant)
            try:
                _lib.check(L.hydra_fold(0, 6, 0, dst.data_ptr() + 4, ptrs, P, n, None))
            finally:
                L.hydra_set_variant(prev)
        else:  # the shipped fold, product library
            _lib.check(_lib.lib().hydra_fold(0, 6, 0, dst.data_ptr() + 4, ptrs, P, n, None))
        torch.cuda.synchronize()
        acc = xs[P - 1].copy()
        for j in range(P - 2, -1, -1):
            acc = O.op(xs[j], acc, "sum", 6)
        assert np.array_equal(dst.cpu().numpy()[1:n + 1].view(np.uint32), acc.view(np.uint32))


def test_simulated_ring_old_vs_reference_fixtures(gpu, golden, golden_meta):
    """Device RING_OLD plan == the reference's own old-style AllreduceRing<T> outputs
    (tests/golden old_ring fixtures, built from allreduce_ring.h), every rank, f32/i32/f16.
    Several pointers per rank: the local pre-reduce ptrs[0] op= ptrs[i] and the closing
    broadcast (allreduce_ring.h:60-66,108-112) are hydra_reduce + copies around the plan."""
    import torch

    from hydra_amd import reduce as R

    views = {_lib.FLOAT32: np.uint32, _lib.INT32: np.int32, _lib.FLOAT16: np.int16}
    for row in golden_meta["old_ring"]:
        key, P, k, code = row["key"], row["P"], row["nptr"], row["dtype"]
        ins = golden[key + "_in"]
        exp = golden[key + "_out"]
        v = views[code]
        bufs = [[torch.from_numpy(ins[r, i].view(v).copy()).to(gpu) for i in range(k)]
                for r in range(P)]
        for r in range(P):
            for i in range(1, k):
                R.reduce_("sum", bufs[r][0], bufs[r][0], bufs[r][i], dtype_code=code)
        ring.simulate([b[0] for b in bufs], algo="ring_old", dtype_code=code, chunk_bytes=1024)
        for r in range(P):
            for i in range(1, k):
                bufs[r][i].copy_(bufs[r][0])
        torch.cuda.synchronize()
        for r in range(P):
            for i in range(k):
                got = bufs[r][i].cpu().numpy()
                assert np.array_equal(got, exp[r, i].view(v)), (key, r, i)


@pytest.mark.parametrize("P,n", [(2, 1 << 20), (8, 3000001)])
def test_simulated_ring_old_large(gpu, O, P, n):
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate(bufs, algo="ring_old")
    olds = [[x.copy()] for x in xs]
    O.allreduce_ring_old(olds)
    for r in range(P):
        assert np.array_equal(bufs[r].cpu().numpy().view(np.uint32), olds[r][0].view(np.uint32))


def test_simulated_ring_chunked_vs_reference_fixtures(gpu, golden, golden_meta):
    """Device RING_CHUNKED plan == the reference's own AllreduceRingChunked<T> on every rank
    (tests/golden chunked_ring, f32/i32/f16, 1-2 pointers per rank)."""
    import torch

    from hydra_amd import reduce as R

    views = {_lib.FLOAT32: np.uint32, _lib.INT32: np.int32, _lib.FLOAT16: np.int16}
    for row in golden_meta["chunked_ring"]:
        key, P, k, code = row["key"], row["P"], row["nptr"], row["dtype"]
        ins = golden[key + "_in"]
        v = views[code]
        exp = golden[key + "_out"].view(v)
        bufs = [[torch.from_numpy(ins[r, i].view(v).copy()).to(gpu) for i in range(k)]
                for r in range(P)]
        for r in range(P):
            for i in range(1, k):
                R.reduce_("sum", bufs[r][0], bufs[r][0], bufs[r][i], dtype_code=code)
        ring.simulate([b[0] for b in bufs], algo="ring_chunked", dtype_code=code)
        for r in range(P):
            for i in range(1, k):
                bufs[r][i].copy_(bufs[r][0])
        torch.cuda.synchronize()
        for r in range(P):
            for i in range(k):
                assert np.array_equal(bufs[r][i].cpu().numpy(), exp), (key, r, i)


@pytest.mark.parametrize("P,n", [(2, 1 << 20), (8, 3000001)])
def test_simulated_ring_chunked_large(gpu, O, P, n):
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate(bufs, algo="ring_chunked")
    exp = [[x.copy()] for x in xs]
    O.allreduce_ring_chunked(exp)
    for r in range(P):
        assert np.array_equal(bufs[r].cpu().numpy().view(np.uint32), exp[r][0].view(np.uint32))


@pytest.mark.parametrize("table", [0, 1])
@pytest.mark.parametrize("algo", ["direct", "ring", "ring_chunked"])
@pytest.mark.parametrize("P,n", [(2, 1000), (2, 1500000), (3, 600000), (4, 1048577),
                                 (6, 2000000), (8, 200000)])
def test_simulated_apipe(gpu, O, table, algo, P, n):
    """bew_allreduce_a on device: the split of calculateElements_AA/_AG, then each rail's part is
    exactly the reference ring (or AllreduceRingChunked) on that slice, as apipe_allreduce
    runs gloo::allreduce per rail (pipeallreduce-a.cc:27-61)."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate_apipe(bufs, table=table, algo=algo)
    e1, e2 = ring.split_elements(table, P, n)
    assert e1 + e2 == n
    exp = np.empty(n, np.float32)
    for lo, hi in ((0, e1), (e1, n)):
        if hi > lo:
            part = [x[lo:hi].copy() for x in xs]
            if algo == "ring_chunked":
                b = [[p] for p in part]
                O.allreduce_ring_chunked(b)
                exp[lo:hi] = b[0][0]
            else:
                exp[lo:hi] = O.ring_result(part)
    for r in range(P):
        assert np.array_equal(bufs[r].cpu().numpy().view(np.uint32), exp.view(np.uint32)), r


def test_apipe_single_rank_rails(gpu):
    """Two 1-rank communicators as rails: argument checks and the P = 1 short circuit."""
    import torch

    r1 = ring.XgmiComm(0, 1, gpu.index or 0, ring._rccl_unique_id())
    r2 = ring.XgmiComm(0, 1, gpu.index or 0, ring._rccl_unique_id())
    try:
        t = torch.arange(1 << 20, dtype=torch.float32, device=gpu)
        r1.apipe_allreduce_(r2, t)
        r1.apipe_allreduce_(r2, t, table=1, algo="rccl")
        torch.cuda.synchronize()
        assert torch.equal(t, torch.arange(1 << 20, dtype=torch.float32, device=gpu))
        with pytest.raises(_lib.HydraError):
            r1.apipe_allreduce_(r1, t)  # the two rails must be distinct communicators
        with pytest.raises(_lib.HydraError):
            r1.apipe_allreduce_(r2, t, table=7)
    finally:
        r1.close()
        r2.close()


def test_simulated_bcube_vs_reference_fixtures(gpu, golden, golden_meta):
    """Device BCUBE plan == the reference's own BCUBE allreduce (tests/golden bcube: P up to 12,
    fp32 stress / int32 / f16)."""
    import hashlib

    import torch

    views = {6: np.uint32, 2: np.int32, 8: np.int16}
    for row in golden_meta["bcube"]:
        P, n, key, code = row["P"], row["n"], row["key"], row["dtype"]
        if row.get("stored_inputs"):
            xs = list(golden[key + "_in"])
        elif code == 2:
            xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        else:
            xs = [synth.stress_f32(P, r, n) for r in range(P)]
        v = views[code]
        bufs = [torch.from_numpy(x.view(v).copy()).to(gpu) for x in xs]
        ring.simulate(bufs, algo="bcube", dtype_code=code)
        for r in range(P):
            got = bufs[r].cpu().numpy()
            if key in golden:
                assert np.array_equal(got, golden[key].view(v)), (key, r)
            else:
                assert hashlib.sha256(got.tobytes()).hexdigest() == row["output_sha256"], key


@pytest.mark.extra
def test_simulated_halving_doubling_vs_reference_fixtures(gpu, golden_algo):
    """Device HALVING_DOUBLING plan == the reference's own AllreduceHalvingDoubling<T> on every
    rank (tests/golden/golden_algo: P = 1..12, one to three binary blocks, fp32 stress / int32 /
    f16, single-pointer cases)."""
    import torch

    golden, meta = golden_algo
    views = {6: np.uint32, 2: np.int32, 8: np.int16}
    for row in meta["halving_doubling"]:
        if row["nptr"] != 1:
            continue
        P, key, code = row["P"], row["key"], row["dtype"]
        v = views[code]
        ins = golden[key + "_in"]
        bufs = [torch.from_numpy(ins[r, 0].view(v).copy()).to(gpu) for r in range(P)]
        ring.simulate(bufs, algo="halving_doubling", dtype_code=code)
        exp = golden[key + "_out"].view(v)
        for r in range(P):
            assert np.array_equal(bufs[r].cpu().numpy(), exp), (key, r)


@pytest.mark.extra
@pytest.mark.parametrize("P,n", [(8, 1 << 22), (6, 3000017), (7, 1 << 20)])
def test_simulated_halving_doubling_large(gpu, O, P, n):
    """Multi-MiB buckets through the simulator: bit-exact vs the oracle on every rank."""
    import torch

    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = [torch.from_numpy(x.copy()).to(gpu) for x in xs]
    ring.simulate(bufs, algo="halving_doubling")
    exp = [[x.copy()] for x in xs]
    O.allreduce_halving_doubling(exp)
    for r in range(P):
        assert np.array_equal(bufs[r].cpu().numpy().view(np.uint32), exp[r][0].view(np.uint32)), r


@pytest.mark.parametrize("algo,P,n,ch", [("ring", 2, 1 << 20, 1 << 18), ("ring", 4, 1 << 20, 0),
                                         ("direct", 4, 1 << 20, 1 << 18),
                                         ("direct", 8, 1 << 21, 1 << 19),
                                         ("ring_old", 3, 300000, 1 << 18),
                                         ("ring_chunked", 4, 1 << 20, 0),
                                         ("bcube", 8, 1 << 20, 0), ("bcube", 6, 6 << 12, 0),
                                         pytest.param("halving_doubling", 8, 1 << 20, 0, marks=pytest.mark.extra),
                                         ("a2a", 2, 1 << 20, 0), ("a2a", 8, 1 << 20, 0)])
def test_rccl_executor_self_loop(gpu, O, comm1, algo, P, n, ch):
    """The real RCCL executor on one GPU: rank 0's plan with every peer remapped to itself runs
    on a 1-rank communicator (RCCL send/recv-to-self), through the same groups, streams and
    event edges as on 8 GPUs (A2A: ncclAllToAll / ncclAllGather on the 1-rank communicator).
    Expected bytes: the numpy interpreter on the same remapped plan."""
    import torch

    from plan_interp import RECV, SEND, run_plan_numpy

    ops, scr = ring.plan(algo, P, 0, n, 4, 0, ch)
    for o in ops:
        if o["kind"] in (SEND, RECV):
            o["peer"] = 0
    x = synth.stress_f32(P, 0, n)
    exp = run_plan_numpy(O, algo, [x], 0, ch, plans=[ops], scr=scr)[0]
    t = torch.from_numpy(x.copy()).to(gpu)
    comm1.run_plan_(ops, t, scr)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy().view(np.uint32), exp.view(np.uint32))
    # a plan reaching outside the buffers is refused before anything is launched
    bad = [dict(o) for o in ops]
    bad[0]["off"] = 4 * n
    with pytest.raises(_lib.HydraError):
        comm1.run_plan_(bad, t, scr)


def test_executor_graph_replay(gpu, O):
    """The executor's stream fork/join, events, scratch reset and kernels capture into a
    hipGraph and replay: a compute-only plan (REDUCE then FOLD on the compute stream, waiting
    on each other and joined into the caller's stream; op = max against the zeroed scratch,
    i.e. max(x, 0)) plus RCCL's own collective (HYDRA_ALGO_RCCL) on a 1-rank communicator,
    captured once and replayed three times.  (RCCL send/recv-to-self and ncclAllToAll on a
    1-rank communicator crash inside RCCL under capture -- scripts/probe_graph.py -- so p2p
    plans are not captured here)"""
    import torch

    n = 1 << 18
    B = n * 4
    x = synth.stress_f32(4, 1, n)
    ops = [dict(kind=4, peer=0, buf=0, nsrc=0, off=0, bytes=B, src_off=0, slot_stride=0,
                wait0=-1, wait1=-1),
           dict(kind=5, peer=-1, buf=0, nsrc=2, off=0, bytes=B, src_off=B, slot_stride=B,
                wait0=0, wait1=-1)]
    zero = np.zeros(n, np.float32)
    exp = O.op(O.op(x, zero, "max", 6), zero, "max", 6)
    comm = ring.XgmiComm(0, 1, gpu.index or 0, ring._rccl_unique_id())
    try:
        xin = torch.from_numpy(x).to(gpu)
        t = xin.clone()
        u = xin.clone()
        comm.run_plan_(ops, t, 2 * B, op="max")  # warm-up outside capture (scratch, events)
        comm.allreduce_(u, algo="rccl")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            comm.run_plan_(ops, t, 2 * B, op="max")
            comm.allreduce_(u, algo="rccl")  # 1 rank: a captured identity collective
        for _ in range(3):
            t.copy_(xin)
            u.copy_(xin)
            g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(t.cpu().numpy().view(np.uint32), exp.view(np.uint32))
        assert np.array_equal(u.cpu().numpy().view(np.uint32), x.view(np.uint32))
        # eager calls after the captured one, on two different streams (the executor orders
        # its scratch across calls only after eager calls: a captured ev_ks is a graph node)
        for k, st in enumerate((torch.cuda.Stream(gpu), torch.cuda.Stream(gpu))):
            t.copy_(xin)
            torch.cuda.synchronize()
            comm.run_plan_(ops, t, 2 * B, op="max", stream=st.cuda_stream)
            st.synchronize()
            assert np.array_equal(t.cpu().numpy().view(np.uint32), exp.view(np.uint32)), k
    finally:
        comm.close()


def test_comm_wait_timeout_aborts(gpu):
    """hydra_comm_wait: the reference's per-op timeout for the asynchronous device path.  Work
    that finishes in time returns; a stream held by a long spin kernel times out with
    "Timed out waiting ...", the communicator is aborted and refuses further allreduces."""
    import torch

    comm = ring.XgmiComm(0, 1, gpu.index or 0, ring._rccl_unique_id())
    try:
        t = torch.ones(1 << 16, device=gpu)
        comm.allreduce_(t, algo="rccl")
        comm.wait(5000)
        torch.cuda._sleep(500_000_000)  # 0.2-5 s of spinning (GPU clock or 100 MHz)
        with pytest.raises(_lib.HydraError, match="Timed out waiting 50ms") as e:
            comm.wait(50)
        assert e.value.code == _lib.ERR_TIMEOUT
        with pytest.raises(_lib.HydraError, match="aborted"):
            comm.allreduce_(t, algo="direct")
        torch.cuda.synchronize()
    finally:
        comm.close()


@pytest.mark.parametrize("algo", ["direct", "ring", "a2a"])
def test_simulated_config4_full_size(gpu, algo):
    """BASELINE config 4 at its full size (8 ranks x 64 Mi fp32) through a size-independent
    property: integer-valued inputs whose sums are exact in fp32 in any order, so every rank
    must hold exactly sum_r x_r -- the full-size companion of the bit-exact fold-order tests."""
    import torch

    P, n = 8, 64 << 20
    j = torch.arange(n, device=gpu, dtype=torch.int64) % 1024
    bufs = [(j * (r + 1)).to(torch.float32) for r in range(P)]
    exp = (j * (P * (P + 1) // 2)).to(torch.float32)
    del j
    ring.simulate(bufs, algo=algo)
    for r, b in enumerate(bufs):
        assert torch.equal(b, exp), (algo, r)


def test_simulated_config5_full_size(gpu):
    """BASELINE config 5 at its full size (8 ranks x 256 Mi bf16, fp32 accumulation): small
    integer inputs make every partial sum exact, so the one final rounding to bf16 is exact
    and every rank must hold sum_r x_r bit for bit."""
    import torch

    P, n = 8, 256 << 20
    base = (torch.arange(n, device=gpu, dtype=torch.int32) % 7 - 3)
    m = [1, 2, -1, 3, -2, 1, 0, 2]  # |partial sums| <= 88: exact in fp32 and in bf16
    bufs = [(base * m[r] + r % 3).to(torch.bfloat16).view(torch.int16) for r in range(P)]
    exp = sum(base * m[r] + r % 3 for r in range(P)).to(torch.bfloat16)
    del base
    ring.simulate(bufs, algo="direct", dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    for r, b in enumerate(bufs):
        assert torch.equal(b.view(torch.bfloat16), exp), r


@pytest.fixture(scope="module")
def config4_full(gpu, O):
    """BASELINE config 4 at its full size with fold-order-sensitive values: 8 ranks x 64 Mi fp32
    of synth.stress_at (stress_f32's distribution, scales 2^0 .. 2^21 across ranks, generated on
    the GPU), and the C restatement's ring result (O.ring_result, pinned to the reference) on the
    same values: at this size the reference geometry is 256 segments of 1 MiB, S = 32 per rank
    (allreduce.cc:199-221), so every one of the 8 blocks is 32 segments long."""
    import torch

    P, n = 8, 64 << 20
    idx = torch.arange(n, device=gpu, dtype=torch.int64)
    xs = [synth.stress_at(P, r, idx) for r in range(P)]
    del idx
    host = [x.cpu().numpy() for x in xs]
    exp = torch.from_numpy(O.ring_result(host)).to(gpu)
    # the values are order-sensitive: a plain left fold x_0 + x_1 + ... differs from the
    # reference's per-block order on a large share of the elements
    left = host[0].copy()
    for h in host[1:]:
        left += h
    differ = float(np.mean(left.view(np.uint32) != exp.cpu().numpy().view(np.uint32)))
    del host, left
    yield xs, exp, differ
    del xs, exp


@pytest.mark.parametrize("algo", ["direct", "ring", "a2a"])
def test_simulated_config4_full_size_order_sensitive(gpu, config4_full, algo):
    """config 4 (8 x 64 Mi fp32) bit-exact at its BASELINE size on values
    whose sums depend on the fold order -- every rank of RING, DIRECT and A2A equals the C
    restatement of the reference ring (block ownership and chunking at S = 32)."""
    import torch

    xs, exp, differ = config4_full
    assert differ > 0.2, differ  # the check can tell fold orders apart
    bufs = [x.clone() for x in xs]
    ring.simulate(bufs, algo=algo)
    for r, b in enumerate(bufs):
        assert torch.equal(b.view(torch.int32), exp.view(torch.int32)), (algo, r)


@pytest.mark.parametrize("algo", ["direct", "a2a"])
def test_simulated_config5_full_size_sampled(gpu, O, algo):
    """config 5 (8 x 256 Mi bf16, fp32 accumulation) at its BASELINE size on
    order-sensitive values (synth.stress_cancel_at: +-2^k pivots that cancel, so the one bf16
    rounding does not hide the fp32 fold order): >= 1 Mi sampled elements -- every owner block's and every segment's
    first two and last two elements, plus random ones spread over the bucket -- on every rank
    equal the C restatement's fold on the widened values with the bf16 geometry (512 segments
    of 1 MiB, S = 64 per rank)."""
    import torch

    P, n = 8, 256 << 20
    idx_t = torch.arange(n, device=gpu, dtype=torch.int64)
    bufs = []
    for r in range(P):
        bufs.append(synth.stress_cancel_at(P, r, idx_t).to(torch.bfloat16).view(torch.int16))
    del idx_t
    ns, sb, S = O.ring_plan(P, n, 2)
    seg = sb // 2
    edges = np.concatenate([np.arange(ns + 1, dtype=np.int64) * seg + d for d in (-2, -1, 0, 1)])
    rnd = np.random.default_rng(55).integers(0, n, 1 << 20, dtype=np.int64)
    idx = np.unique(np.concatenate([edges, rnd, [0, 1, n - 2, n - 1]]))
    idx = idx[(idx >= 0) & (idx < n)]
    from fold_expect import bf16_acc32_expected

    exp, vals, geom = bf16_acc32_expected(O, P, n, idx)
    assert geom == (512, 1 << 20, 64) and idx.size > (1 << 20) - 4096, (geom, idx.size)
    # the check can tell fold orders apart: a plain left fold differs on many samples
    left = synth.bf16_to_f32(vals[0]).astype(np.float32)
    for v in vals[1:]:
        left = O.acc_bf16_f32(left, v)
    assert float(np.mean(synth.bf16_bits(left) != exp)) > 0.3
    ring.simulate(bufs, algo=algo, dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    it = torch.from_numpy(idx).to(gpu)
    for r, b in enumerate(bufs):
        got = b[it].cpu().numpy().view(np.uint16)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, (algo, r, bad.size, idx[bad[:5]].tolist())


@pytest.mark.parametrize("P,n,ms,ch", [(2, 1, 0, 0), (2, 1000, 128, 256), (3, 4099, 128, 1024),
                                       (4, 262145, 0, 0), (5, 1 << 20, 0, 1 << 18),
                                       (8, 3000001, 0, 0), (8, 5003, 64, 128)])
def test_simulated_reduce_root_f32(gpu, O, P, n, ms, ch):
    """hydra_reduce_root (gloo::reduce to a root on device): with the real HIP fold kernel and
    event edges, the root's bucket equals the reference's root output bit for bit."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    for root in sorted({0, P - 1, P // 2}):
        bufs = dev_bufs(gpu, xs)
        ring.simulate_reduce(bufs, root, max_segment=ms, chunk_bytes=ch)
        exp = [x.copy() for x in xs]
        O.reduce(exp, None, root, max_segment=ms or (1 << 20))
        got = bufs[root].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), exp[root].view(np.uint32)), (P, n, root)


def test_simulated_reduce_root_int32_bf16(gpu, O):
    import torch

    P, n = 4, 100003
    xs = [synth.int32_bucket(P, r, n) for r in range(P)]
    bufs = dev_bufs(gpu, xs)
    ring.simulate_reduce(bufs, 2, max_segment=4096, chunk_bytes=8192)
    exp = [x.copy() for x in xs]
    O.reduce(exp, None, 2, max_segment=4096)
    assert np.array_equal(bufs[2].cpu().numpy(), exp[2])
    # bf16 bucket, fp32 accumulation (config 5's arithmetic), integer-valued: exact
    base = torch.arange(n, device=gpu, dtype=torch.int32) % 7 - 3
    m = [1, 2, -1, 3]
    bb = [(base * m[r] + r).to(torch.bfloat16).view(torch.int16) for r in range(P)]
    ring.simulate_reduce(bb, 1, dtype_code=_lib.BFLOAT16, flags=_lib.ACC_F32)
    want = sum(base * m[r] + r for r in range(P)).to(torch.bfloat16)
    assert torch.equal(bb[1].view(torch.bfloat16), want)


def test_reduce_root_public_entry(gpu, comm1):
    """hydra_reduce_root through a live 1-rank RCCL communicator: P = 1 is the identity
    (reduce.cc:52-58), and bad roots are refused before anything is enqueued.  (A remapped
    self-loop of the multi-rank plan, as for the allreduces, cannot run: the gather half only
    sends on non-roots and only receives on the root.)"""
    import torch

    x = synth.stress_f32(2, 0, 100003)
    y = torch.from_numpy(x.copy()).to(gpu)
    comm1.reduce_(y, 0)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy().view(np.uint32), x.view(np.uint32))
    for bad in (-1, 1):
        with pytest.raises(_lib.HydraError):
            comm1.reduce_(y, bad)
