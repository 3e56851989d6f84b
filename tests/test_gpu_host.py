"""Host-resident path on the GPU: the C++ host runtime's ring and two-rail split with every
segment reduced on the MI355X (hydra_reduce_host: H2D -> gfx950 kernel -> D2H), bit-exact vs
the reference ring."""
import numpy as np
import pytest

from hydra_amd import host, synth

pytestmark = pytest.mark.gpu


def assert_bits(got, exp, ctx):
    """Bit-exact, and on a mismatch say how many elements differ and where (a stale chunk, a
    torn tail and a single bad element read differently)."""
    g, e = got.view(np.uint32), exp.view(np.uint32)
    if np.array_equal(g, e):
        return
    bad = np.flatnonzero(g != e)
    runs = np.split(bad, np.flatnonzero(np.diff(bad) != 1) + 1)
    spans = [(int(r[0]), int(r[-1]) + 1) for r in runs[:8]]
    raise AssertionError(f"{ctx}: {bad.size} of {g.size} elements differ; spans {spans}"
                         f"{' ...' if len(runs) > 8 else ''}; got[:4] at first "
                         f"{g[bad[0]:bad[0] + 4].tolist()} exp {e[bad[0]:bad[0] + 4].tolist()}")


@pytest.mark.parametrize("P,n,ms", [(2, 100, 0), (2, 262145, 0), (3, 100003, 4096),
                                    (4, 1 << 20, 0)])
def test_host_ring_gpu_reducer(gpu, O, P, n, ms):
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [[x.copy()] for x in xs]
    host.allreduce_threads(outs, None, max_segment=ms)  # GPU reducer
    exp = O.ring_result(xs, ms or (1 << 20))
    for r in range(P):
        assert np.array_equal(outs[r][0].view(np.uint32), exp.view(np.uint32))


def test_host_ring_gpu_reducer_multi_input(gpu, O):
    """2 inputs per rank out of place: local pre-reduction also runs on the GPU."""
    P, n = 2, 50001
    ins = [[synth.stress_f32(P, r, n, seed=7 + i) for i in range(2)] for r in range(P)]
    outs = [[np.zeros(n, np.float32) for _ in range(2)] for _ in range(P)]
    host.allreduce_threads(outs, ins, max_segment=8192)
    o2 = [[np.zeros(n, np.float32) for _ in range(2)] for _ in range(P)]
    O.allreduce(P, o2, ins, max_segment=8192)
    for r in range(P):
        for i in range(2):
            assert np.array_equal(outs[r][i].view(np.uint32), o2[r][i].view(np.uint32))


@pytest.mark.parametrize("n", [1000, 1500001])
def test_apipe_gpu_reducer(gpu, O, n):
    """bew_allreduce_a with both rails reducing concurrently on one GPU (one staging context
    per rail thread)."""
    P = 2
    ins = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [np.zeros(n, np.float32) for _ in range(P)]
    host.apipe_threads(ins, outs)
    e1, e2 = O.split_aa(P, n)
    exp = np.empty(n, np.float32)
    if e1:
        exp[:e1] = O.ring_result([x[:e1].copy() for x in ins])
    if e2:
        exp[e1:] = O.ring_result([x[e1:].copy() for x in ins])
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp.view(np.uint32))


def test_old_style_allreduce_ring_gpu_reducer_vs_reference(gpu, golden, golden_meta):
    """hydra::AllreduceRing<T> with the GPU in-place sum (gpuReductionFunction) reproduces the
    reference's own old-style AllreduceRing<T> outputs (tests/golden old_ring) for f32/i32;
    f16 is exercised by the CPU test with the custom reducer."""
    for row in golden_meta["old_ring"]:
        if row["dtype"] not in (6, 2):  # FLOAT32, INT32
            continue
        key = row["key"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(row["nptr"])] for r in range(row["P"])]
        host.allreduce_ring_old_threads(bufs, dtype_code=row["dtype"])
        got = np.stack([np.stack(b) for b in bufs])
        exp = golden[key + "_out"]
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), key


def test_chunked_allreduce_ring_gpu_reducer_vs_reference(gpu, golden, golden_meta):
    """hydra::AllreduceRingChunked<T> with the GPU in-place sum == the reference's own
    AllreduceRingChunked<T> outputs (f32/i32), every rank and pointer."""
    for row in golden_meta["chunked_ring"]:
        if row["dtype"] not in (6, 2):
            continue
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_ring_old_threads(bufs, dtype_code=row["dtype"], chunked=True)
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                assert np.array_equal(bufs[r][i].view(np.uint32), exp.view(np.uint32)), key


@pytest.mark.extra
def test_halving_doubling_gpu_reducer_vs_reference(gpu, golden_algo):
    """hydra::AllreduceHalvingDoubling<T> with the GPU in-place sum (gpuReductionFunction) ==
    the reference's own AllreduceHalvingDoubling<T> outputs (f32/i32), every rank and pointer,
    P = 1..12 (one to three binary blocks)."""
    golden, meta = golden_algo
    for row in meta["halving_doubling"]:
        if row["dtype"] not in (6, 2):
            continue
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_halving_doubling_threads(bufs, dtype_code=row["dtype"])
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                assert np.array_equal(bufs[r][i].view(np.uint32), exp.view(np.uint32)), (key, r)


@pytest.mark.extra
def test_bcube_old_gpu_reducer_vs_reference(gpu, golden_algo):
    """Old-style hydra::AllreduceBcube<T> with the GPU in-place sum == the reference's own
    AllreduceBcube<T> outputs (f32/i32), every rank and pointer."""
    golden, meta = golden_algo
    for row in meta["bcube_old"]:
        if row["dtype"] not in (6, 2):
            continue
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_bcube_old_threads(bufs, dtype_code=row["dtype"])
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                assert np.array_equal(bufs[r][i].view(np.uint32), exp.view(np.uint32)), (key, r)


def _local(O, xs, code, left_fold):
    """The CUDA algorithms' local reduce: cudaHostReduce's left fold in pointer order
    (host workspace below kOnDeviceThreshold = 256 KiB, algorithm.cc:16) or the pairwise tree."""
    if not left_fold:
        return _tree(O, xs, code)
    acc = xs[0].copy()
    for x in xs[1:]:
        acc = O.op(acc, x, "sum", code)
    return acc


def _tree(O, xs, code):
    """CudaLocalNativeReduce's pairwise tree in pointer order (cuda_collectives_native.h:93-122)."""
    xs = [x.copy() for x in xs]
    sz = 1
    while sz < len(xs):
        for j in range(0, len(xs) - sz, 2 * sz):
            xs[j] = O.op(xs[j], xs[j + sz], "sum", code)
        sz *= 2
    return xs[0]


@pytest.mark.parametrize("workspace", ["host", "device"])
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 1, 1000, "f32"), (2, 1, 262145, "f32"),
                                         (3, 2, 100003, "f32"), (4, 4, 4099, "f32"),
                                         (5, 3, 7, "f32"), (3, 2, 70001, "i32"),
                                         (2, 1, 0, "f32")])
def test_hip_allreduce_ring(gpu, O, workspace, P, nptr, n, dt, monkeypatch, stage=False):
    """hydra::HipAllreduceRing<T, W> (gloo::CudaAllreduceRing<T, W>): rank r ends with its own
    left fold x_r + x_{r-1} + ... of the locally reduced values (the AllreduceRing result,
    pinned to the reference by the old_ring fixtures); host workspace pre-reduces pointers as a
    left fold, device workspace as the pairwise tree; every pointer gets the result."""
    import torch

    code = {"f32": 6, "i32": 2}[dt]
    if dt == "f32":
        xs = [[synth.stress_f32(P, r, n, seed=40 + i) for i in range(nptr)] for r in range(P)]
    else:
        xs = [[synth.int32_bucket(P, r, n, seed=40 + i) for i in range(nptr)] for r in range(P)]
    local = []
    for r in range(P):
        if workspace == "device":
            local.append(_tree(O, xs[r], code))
        else:
            acc = xs[r][0].copy()
            for i in range(1, nptr):
                acc = O.op(acc, xs[r][i], "sum", code)
            local.append(acc)
    exp = [[v.copy()] for v in local]
    O.allreduce_ring_old(exp, dtype_code=code)
    for user_streams in (False, True):
        ts = [[torch.from_numpy(x.copy()).to(gpu) for x in xs[r]] for r in range(P)]
        host.hip_ring_threads(ts, workspace=workspace, user_streams=user_streams)
        for r in range(P):
            for i in range(nptr):
                got = ts[r][i].cpu().numpy()
                assert_bits(got, exp[r][0], (r, i, user_streams))


def test_hip_allreduce_ring_rejects_host_pointers(gpu):
    """CudaDevicePointer<T>::create needs device memory; so does the HIP ring's constructor."""
    import ctypes

    x = np.zeros(10, np.float32)
    ptrs = (ctypes.c_void_p * 1)(x.ctypes.data)
    err = ctypes.create_string_buffer(512)
    rc = host.lib().hydra_host_hip_ring_threads(1, 1, 6, 10, ctypes.cast(ptrs, ctypes.c_void_p),
                                                0, 0, err, 512)
    assert rc != 0 and b"device memory" in err.value


@pytest.mark.parametrize("config", [1, 3])
def test_host_bench_pinned_zero_copy(gpu, O, config):
    """Config 1 / 3 with pinned receive slots + registered output (zero-copy reduces) runs."""
    s = host.bench(config, 2, 1 << 18, 1, 3, pinned=True)
    assert s.shape == (3,) and np.all(s > 0)
    # one GPU per rank, approximated on the one-GPU box: rank 0 zero-copy, rank 1 a CPU sum
    import ctypes

    fn = ctypes.cast(O.orc().orc_sum_f32, ctypes.c_void_p).value
    s = host.bench(config, 2, 1 << 18, 1, 3, reducer_fn=fn, gpu_rank0_only=True)
    assert s.shape == (3,) and np.all(s > 0)


def test_host_ring_pinned_scratch_zero_copy(gpu, O, host_buf):
    """The ring over pinned receive slots and a registered output (zero-copy GPU reduces) is
    bit-exact vs the reference ring: the default GPU reducer path picks zero-copy by itself."""
    import ctypes

    from hydra_amd import _lib

    L = _lib.lib()
    P, n = 3, 100003
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [[host_buf(n, np.float32, x)] for x in xs]
    for o in outs:
        _lib.check(L.hydra_host_register(o[0].ctypes.data, o[0].nbytes))
    try:
        host.allreduce_threads(outs, None, max_segment=4096, pinned_scratch=True)
    finally:
        for o in outs:
            L.hydra_host_unregister(o[0].ctypes.data)
    exp = O.ring_result(xs, 4096)
    for r in range(P):
        assert np.array_equal(outs[r][0].view(np.uint32), exp.view(np.uint32)), r


def test_reduce_gpu_reducer_vs_golden(gpu, golden, golden_meta):
    """gloo::reduce (reduce.cc:21-262) with every segment reduced on the MI355X (out of place:
    reduce(out + off, in + off, tmp)) against the reference's own outputs on every rank."""
    for row in golden_meta["reduce"]:
        if "dtype" in row and row["dtype"] != 2:
            continue  # the GPU sum covers int32/fp32 here (float16: tests/test_gpu_reduce.py)
        if "dtype" in row:
            xs = list(golden[row["key"] + "_inputs"])
            outs = [x.copy() for x in xs]
            host.reduce_threads(outs, None, row["root"], dtype_code=2,
                                max_segment=row["max_segment"])
            assert np.array_equal(np.stack(outs), golden[row["key"]]), row["key"]
            continue
        P, n = row["P"], row["n"]
        xs = [synth.stress_f32(P, r, n) for r in range(P)]
        if row["inplace"]:
            outs, ins = [x.copy() for x in xs], None
        else:
            outs, ins = [np.zeros(n, np.float32) for _ in xs], [x.copy() for x in xs]
        host.reduce_threads(outs, ins, row["root"], max_segment=row["max_segment"])
        if row["key"] in golden.files:
            assert np.array_equal(np.stack(outs).view(np.uint32),
                                  golden[row["key"]].view(np.uint32)), row["key"]
        else:
            assert np.array_equal(outs[row["root"]].view(np.uint32),
                                  golden[row["key"] + "_root"].view(np.uint32)), row["key"]


@pytest.mark.parametrize("pinned", [False, True])
def test_reduce_gpu_reducer_large(gpu, O, pinned):
    """Past the 1 MiB segment cap, out of place, GPU reducer (staged, or zero-copy from pinned
    receive slots): the root equals the C restatement bit for bit."""
    P, n, root = 4, 3_000_001, 1
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [np.zeros(n, np.float32) for _ in range(P)]
    host.reduce_threads(outs, [x.copy() for x in xs], root, pinned_scratch=pinned)
    exp = [np.zeros(n, np.float32) for _ in range(P)]
    O.reduce(exp, [x.copy() for x in xs], root)
    assert np.array_equal(outs[root].view(np.uint32), exp[root].view(np.uint32))


@pytest.mark.parametrize("workspace", ["host", "device"])
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 1, 1000, "f32"), (2, 1, 262145, "f32"),
                                         (3, 2, 100003, "f32"), (4, 4, 4099, "f32"),
                                         (5, 3, 7, "f32"), (3, 2, 70001, "i32"),
                                         (2, 1, 0, "f32")])
def test_hip_allreduce_ring_chunked(gpu, O, workspace, P, nptr, n, dt, monkeypatch=None,
                                    stage=False):
    """hydra::HipAllreduceRingChunked<T, W> (gloo::CudaAllreduceRingChunked<T, W>): every rank
    ends with AllreduceRingChunked's result (pinned to the reference by the chunked_ring
    fixtures) over the locally reduced values -- CudaLocalNativeReduce's pairwise tree for both
    workspaces (cuda_collectives_device.h:29-56); every pointer gets the result."""
    import torch

    code = {"f32": 6, "i32": 2}[dt]
    if dt == "f32":
        xs = [[synth.stress_f32(P, r, n, seed=50 + i) for i in range(nptr)] for r in range(P)]
    else:
        xs = [[synth.int32_bucket(P, r, n, seed=50 + i) for i in range(nptr)] for r in range(P)]
    exp = [[_tree(O, xs[r], code)] for r in range(P)]
    if n:
        O.allreduce_ring_chunked(exp, dtype_code=code)
    for user_streams in (False, True):
        ts = [[torch.from_numpy(x.copy()).to(gpu) for x in xs[r]] for r in range(P)]
        host.hip_ring_threads(ts, workspace=workspace, user_streams=user_streams, chunked=True)
        for r in range(P):
            for i in range(nptr):
                got = ts[r][i].cpu().numpy()
                assert_bits(got, exp[r][0], (r, i, user_streams))


@pytest.mark.parametrize("workspace", ["host", "device"])
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 3, 1000, "f32"), (3, 2, 100003, "f32"),
                                         (4, 4, 4099, "f32"), (3, 2, 70001, "i32")])
def test_hip_rings_local_reduce_staged(gpu, O, workspace, P, nptr, n, dt, monkeypatch):
    """The rings over several GPUs of one process: a local-reduce step whose two
    pointers sit on devices without peer access copies the source to a buffer on the
    destination's device first, ordered by events.  The test switch HYDRA_TEST_LOCAL_STAGE (hydra_test_set) takes that branch
    for every step on the one GPU: the same bits as the reference semantics."""
    from hydra_amd import _lib

    prev = _lib.test_set(_lib.TEST_LOCAL_STAGE, 1)  # every local-reduce step staged
    try:
        test_hip_allreduce_ring(gpu, O, workspace, P, nptr, n, dt, monkeypatch, stage=True)
        test_hip_allreduce_ring_chunked(gpu, O, workspace, P, nptr, n, dt, monkeypatch,
                                        stage=True)
    finally:
        _lib.test_set(_lib.TEST_LOCAL_STAGE, prev)


@pytest.mark.extra
@pytest.mark.parametrize("workspace", ["host", "device"])
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 2, 1000, "f32"), (2, 1, 262145, "f32"),
                                         (3, 2, 100003, "f32"), (4, 4, 4099, "f32"),
                                         (5, 3, 7, "f32"), (6, 1, 300001, "f32"),
                                         (7, 2, 70001, "i32"), (2, 1, 0, "f32")])
def test_hip_allreduce_halving_doubling(gpu, O, workspace, P, nptr, n, dt):
    """hydra::HipAllreduceHalvingDoubling<T, W> (gloo::CudaAllreduceHalvingDoubling<T, W>):
    every rank ends with AllreduceHalvingDoubling's result (pinned to the reference by the
    golden_algo fixtures) over the pairwise-tree local values, both workspaces, caller or own
    streams; every pointer gets the result."""
    import torch

    code = {"f32": 6, "i32": 2}[dt]
    if dt == "f32":
        xs = [[synth.stress_f32(P, r, n, seed=60 + i) for i in range(nptr)] for r in range(P)]
    else:
        xs = [[synth.int32_bucket(P, r, n, seed=60 + i) for i in range(nptr)] for r in range(P)]
    exp = [[_local(O, xs[r], code, workspace == "host" and n * 4 < 256 * 1024)]
           for r in range(P)]
    if n:
        O.allreduce_halving_doubling(exp, dtype_code=code)
    for user_streams in (False, True):
        ts = [[torch.from_numpy(x.copy()).to(gpu) for x in xs[r]] for r in range(P)]
        host.hip_ring_threads(ts, workspace=workspace, user_streams=user_streams,
                              halving_doubling=True)
        for r in range(P):
            for i in range(nptr):
                got = ts[r][i].cpu().numpy()
                assert_bits(got, exp[r][0], (r, i, user_streams))


@pytest.mark.extra
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 1, 1000, "f32"), (1, 2, 262145, "f32"),
                                         (2, 3, 100003, "f32"), (1, 5, 4099, "i32"),
                                         (1, 8, 7, "f32"), (1, 2, 0, "f32")])
def test_hip_allreduce_local(gpu, O, P, nptr, n, dt):
    """hydra::HipAllreduceLocal<T> (gloo::CudaAllreduceLocal<T>): every pointer of a rank ends
    with the pairwise tree of cudaDeviceReduce (cuda_collectives_device.h:29-56) over that
    rank's pointers, on the gfx950 kernel; caller or own streams."""
    import torch

    code = {"f32": 6, "i32": 2}[dt]
    if dt == "f32":
        xs = [[synth.stress_f32(nptr, i, n, seed=70 + r) for i in range(nptr)] for r in range(P)]
    else:
        xs = [[synth.int32_bucket(nptr, i, n, seed=70 + r) for i in range(nptr)] for r in range(P)]
    exp = [_tree(O, xs[r], code) for r in range(P)]
    for user_streams in (False, True):
        ts = [[torch.from_numpy(x.copy()).to(gpu) for x in xs[r]] for r in range(P)]
        host.hip_ring_threads(ts, user_streams=user_streams, local=True)
        for r in range(P):
            for i in range(nptr):
                got = ts[r][i].cpu().numpy()
                assert_bits(got, exp[r], (r, i, user_streams))


@pytest.mark.extra
@pytest.mark.parametrize("workspace", ["host", "device"])
@pytest.mark.parametrize("P,nptr,n,dt", [(1, 2, 1000, "f32"), (2, 1, 262145, "f32"),
                                         (4, 3, 1000, "f32"), (4, 3, 100003, "f32"),
                                         (8, 2, 4099, "f32"), (2, 2, 70001, "i32"),
                                         (2, 1, 0, "f32")])
def test_hip_allreduce_bcube(gpu, O, workspace, P, nptr, n, dt):
    """hydra::HipAllreduceBcube<T, W> (gloo::CudaAllreduceBcube<T, W>): the local reduce
    (host workspace below 256 KiB: left fold in pointer order, cudaHostReduce; otherwise the
    pairwise tree) then the old-style AllreduceBcube result (= the BCUBE bits for P = 2^k,
    pinned by the golden_algo fixtures); every pointer gets it, caller or own streams."""
    import torch

    code = {"f32": 6, "i32": 2}[dt]
    if dt == "f32":
        xs = [[synth.stress_f32(P, r, n, seed=40 + i) for i in range(nptr)] for r in range(P)]
    else:
        xs = [[synth.int32_bucket(P, r, n, seed=40 + i) for i in range(nptr)] for r in range(P)]
    left = workspace == "host" and n * 4 < 256 * 1024
    loc = [_local(O, xs[r], code, left) for r in range(P)]
    exp = O.bcube_result(loc, dtype_code=code) if n and P > 1 else None
    for user_streams in (False, True):
        ts = [[torch.from_numpy(x.copy()).to(gpu) for x in xs[r]] for r in range(P)]
        host.hip_ring_threads(ts, workspace=workspace, user_streams=user_streams, bcube=True)
        for r in range(P):
            want = exp if exp is not None else loc[r]
            for i in range(nptr):
                got = ts[r][i].cpu().numpy()
                assert_bits(got, want, (r, i, user_streams))


@pytest.mark.parametrize("n", [16 << 20, 64 << 20])
def test_configs_1_and_3_full_size_gpu_reducer(gpu, O, n):
    """BASELINE configs 1 and 3 at their top sizes, 2 ranks on loopback TCP with every segment
    reduced on the MI355X: the host runtime's ring (new_allreduce_ring) and two-rail split
    (bew_allreduce_a, calculateElements_AA) are bit-exact vs the oracle ring, full output.
    (runner.cc:338-362 sweeps up to 2^26; the published rows are README.md:86,123.)"""
    P = 2
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    exp = O.ring_result(xs)
    outs = [[x.copy()] for x in xs]
    host.allreduce_threads(outs, None)  # config 1
    for r in range(P):
        assert np.array_equal(outs[r][0].view(np.uint32), exp.view(np.uint32)), r
    del outs
    aout = [np.zeros(n, np.float32) for _ in range(P)]
    host.apipe_threads(xs, aout)  # config 3
    e1, e2 = O.split_aa(P, n)
    exp3 = np.empty(n, np.float32)
    if e1:
        exp3[:e1] = O.ring_result([x[:e1].copy() for x in xs])
    if e2:
        exp3[e1:] = O.ring_result([x[e1:].copy() for x in xs])
    for r in range(P):
        assert np.array_equal(aout[r].view(np.uint32), exp3.view(np.uint32)), r
