"""The C++ host runtime (libhydra_host.so) on the CPU: thread-per-rank over loopback TCP, as the
reference's own tests run (gloo/gloo/test/base_test.h:116-156).  The reducer is the oracle here
(the GPU reducer is exercised by tests/test_gpu_host.py); what is tested is the ring schedule,
the segment geometry, local reduce/broadcast, the transport, timeouts and the rail split."""
import ctypes

import numpy as np
import pytest

from hydra_amd import host, synth
from hydra_amd._lib import HydraError


def fnptr(O, name):
    return ctypes.cast(getattr(O.orc(), name), ctypes.c_void_p).value


@pytest.mark.parametrize("algorithm", ["ring", "bcube"])
@pytest.mark.parametrize("P", [1, 2, 4, 7])
@pytest.mark.parametrize("nptr", [1, 2, 3])
@pytest.mark.parametrize("inplace", [True, False])
def test_allreduce_new_test_default(O, P, nptr, inplace, algorithm):
    """AllreduceNewTest.Default (test/allreduce_test.cc:302-362): uint64, maxSegmentSize=128;
    the reference test is parametrized over RING and BCUBE (allreduce_test.cc:355-362)."""
    for n in (1, 10, 100, 1000):
        stride = P * nptr
        vals = [[np.arange(n, dtype=np.uint64) * stride + r * nptr + i for i in range(nptr)]
                for r in range(P)]
        if inplace:
            outs, ins = [[v.copy() for v in vr] for vr in vals], None
        else:
            outs = [[np.zeros(n, np.uint64) for _ in range(nptr)] for _ in range(P)]
            ins = vals
        host.allreduce_threads(outs, ins, max_segment=128, reducer_fn=fnptr(O, "orc_sum_u64"),
                               algorithm=algorithm)
        exp = np.arange(n, dtype=np.uint64) * stride * stride + np.uint64(stride * (stride - 1) // 2)
        for r in range(P):
            for i in range(nptr):
                assert np.array_equal(outs[r][i], exp), (P, nptr, n, inplace)


@pytest.mark.parametrize("P,n,ms", [(2, 100, 0), (3, 1001, 128), (4, 262145, 0),
                                    (5, 10007, 4096), (8, 40009, 1024)])
def test_fold_order_bit_exact(O, P, n, ms):
    """fp32 stress inputs: the host ring equals the reference ring bit for bit."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [[x.copy()] for x in xs]
    host.allreduce_threads(outs, None, max_segment=ms, reducer_fn=fnptr(O, "orc_sum_f32"))
    exp = O.ring_result(xs, ms or (1 << 20))
    for r in range(P):
        assert np.array_equal(outs[r][0].view(np.uint32), exp.view(np.uint32))


def test_float16_quirk_through_ring(O):
    P, n = 3, 5000
    rng = np.random.default_rng(8)
    hs = [np.array([O.f2h(float(v)) for v in rng.integers(0, 5, n)], np.uint16) for _ in range(P)]
    outs = [[h.copy()] for h in hs]
    host.allreduce_threads(outs, None, dtype_code=8, max_segment=256,
                           reducer_fn=fnptr(O, "orc_sum_f16"))
    exp = O.ring_result(hs, 256, dtype_code=8)
    assert all(np.array_equal(o[0], exp) for o in outs)


@pytest.mark.parametrize("table", [host.SPLIT_AA, host.SPLIT_AG])
@pytest.mark.parametrize("P", [2, 3, 4, 6, 8])
def test_split_tables_match_restatement(O, table, P):
    fn = O.split_aa if table == host.SPLIT_AA else O.split_ag
    ns = [1, 1000, 6144, 6145, 65535, 65536, 65537, 131071, 131072, 262144, 262145, 524288,
          524289, 828343, 828344, 1048576, 1048577, 1500000, 1500001, 2097152, 2097153, 4194304,
          4194305, 8388608, 16777216, 16777217, 33554432, 33554433, 67108864, 67108865]
    for n in ns:
        assert host.calculate_elements(table, P, n) == fn(P, n), (P, n)


@pytest.mark.parametrize("P,n", [(2, 1000), (2, 65536), (2, 1500001), (3, 200003),
                                 (4, 1 << 20)])
def test_apipe_two_rails(O, P, n):
    """bew_allreduce_a: split by calculateElements_AA, two concurrent rings on two rails
    (pipeallreduce-a.cc:27-61); each part equals an independent reference ring on its slice."""
    ins = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [np.zeros(n, np.float32) for _ in range(P)]
    host.apipe_threads(ins, outs, reducer_fn=fnptr(O, "orc_sum_f32"))
    e1, e2 = O.split_aa(P, n)
    exp = np.empty(n, np.float32)
    if e1:
        exp[:e1] = O.ring_result([x[:e1].copy() for x in ins])
    if e2:
        exp[e1:] = O.ring_result([x[e1:].copy() for x in ins])
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp.view(np.uint32))


def test_timeout_raises_io_exception():
    """AllreduceNewTest.TestTimeout (allreduce_test.cc:381-397)."""
    rc, what = host.timeout_probe(10)
    assert rc == 0 and "Timed out" in what


def test_bench_bodies_run(O):
    s = host.bench(1, 2, 1 << 16, 1, 3, reducer_fn=fnptr(O, "orc_sum_f32"))
    assert s.shape == (3,) and np.all(s > 0)
    s = host.bench(3, 2, 1 << 16, 1, 3, reducer_fn=fnptr(O, "orc_sum_f32"))
    assert np.all(s > 0)
    with pytest.raises(HydraError):  # the other ranks' reducer is required
        host.bench(3, 2, 1 << 16, 1, 3, gpu_rank0_only=True)


def test_old_style_allreduce_ring_vs_golden(O, golden, golden_meta):
    """hydra::AllreduceRing<T> (old Algorithm API, allreduce_ring.h:20-125) reproduces the
    reference's per-rank results -- the oracle's in-place reduction stands in for the GPU."""
    names = {6: "orc_isum_f32", 2: "orc_isum_i32", 8: "orc_isum_f16"}
    for row in golden_meta["old_ring"]:
        key = row["key"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(row["nptr"])] for r in range(row["P"])]
        host.allreduce_ring_old_threads(bufs, dtype_code=row["dtype"],
                                        reducer_fn=fnptr(O, names[row["dtype"]]))
        got = np.stack([np.stack(b) for b in bufs])
        exp = golden[key + "_out"]
        assert np.array_equal(got.view(f"u{got.itemsize}"), exp.view(f"u{exp.itemsize}")), key


def test_chunked_allreduce_ring_vs_golden(O, golden, golden_meta):
    """hydra::AllreduceRingChunked<T> (allreduce_ring_chunked.h:20-248) reproduces the
    reference's result on every rank and pointer (oracle in-place sum as the reducer)."""
    names = {6: "orc_isum_f32", 2: "orc_isum_i32", 8: "orc_isum_f16"}
    for row in golden_meta["chunked_ring"]:
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_ring_old_threads(bufs, dtype_code=row["dtype"],
                                        reducer_fn=fnptr(O, names[row["dtype"]]), chunked=True)
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                got = bufs[r][i]
                assert np.array_equal(got.view(f"u{got.itemsize}"),
                                      exp.view(f"u{exp.itemsize}")), (key, r, i)


def test_chunked_allreduce_ring_large(O):
    """Many chunks in flight per pair: 2P chunks of ~n/2P, P = 4, n = 1 Mi + 7 (ragged tail)."""
    P, n = 4, (1 << 20) + 7
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = [[x.copy()] for x in xs]
    host.allreduce_ring_old_threads(bufs, reducer_fn=fnptr(O, "orc_isum_f32"), chunked=True)
    exp = [[x.copy()] for x in xs]
    O.allreduce_ring_chunked(exp)
    for r in range(P):
        assert np.array_equal(bufs[r][0].view(np.uint32), exp[r][0].view(np.uint32))


def test_bcube_vs_golden(O, golden, golden_meta):
    """BCUBE (allreduce.cc:423-700) on the host runtime == the reference's own BCUBE output
    (fixtures: P in 1,2,3,4,6,8,12, ragged n, fp32 stress / int32 / f16)."""
    import hashlib

    names = {6: "orc_sum_f32", 2: "orc_sum_i32", 8: "orc_sum_f16"}
    for row in golden_meta["bcube"]:
        P, n, key, code = row["P"], row["n"], row["key"], row["dtype"]
        if row.get("stored_inputs"):
            xs = list(golden[key + "_in"])
        elif code == 2:
            xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        else:
            xs = [synth.stress_f32(P, r, n) for r in range(P)]
        if "inputs_sha256" in row:
            assert hashlib.sha256(np.stack(xs).tobytes()).hexdigest() == row["inputs_sha256"]
        outs = [[x.copy()] for x in xs]
        host.allreduce_threads(outs, None, dtype_code=code, reducer_fn=fnptr(O, names[code]),
                               algorithm="bcube")
        for r in range(P):
            got = outs[r][0]
            if key in golden:
                assert np.array_equal(got.view(np.uint8), golden[key].view(np.uint8)), (key, r)
            else:
                assert hashlib.sha256(got.tobytes()).hexdigest() == row["output_sha256"], key


def test_bcube_multi_pointer_out_of_place(O):
    """BCUBE's local reduce (step 0, per chunk) and local broadcast (per received chunk) with
    several inputs and outputs, vs the C restatement (pinned to the reference in test_oracle)."""
    P, n, nptr = 6, 10007, 3
    xs = [[synth.stress_f32(P, r, n, seed=90 + i) for i in range(nptr)] for r in range(P)]
    outs = [[np.full(n, 5, np.float32) for _ in range(nptr)] for _ in range(P)]
    exp = [[np.full(n, 5, np.float32) for _ in range(nptr)] for _ in range(P)]
    host.allreduce_threads(outs, [[x.copy() for x in r] for r in xs],
                           reducer_fn=fnptr(O, "orc_sum_f32"), algorithm="bcube")
    O.allreduce(P, exp, [[x.copy() for x in r] for r in xs], algorithm=2)
    for r in range(P):
        for i in range(nptr):
            assert np.array_equal(outs[r][i].view(np.uint32), exp[r][i].view(np.uint32))


# ---- gloo::reduce (reduce.cc:21-262): the other new-style caller of the reduce function ----
def _reduce_case_inputs(row):
    P, n = row["P"], row["n"]
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    if row["inplace"]:
        return [x.copy() for x in xs], None
    return [np.zeros(n, np.float32) for _ in xs], [x.copy() for x in xs]


def test_reduce_every_rank_vs_golden(golden, golden_meta, O):
    """Host runtime reduce() against the reference's own outputs on EVERY rank: the root holds
    the reduction, the other ranks what the reference's schedule leaves (its extra ring
    iterations, reduce.cc:182-223) -- so the schedule itself is pinned, not just the result."""
    for row in golden_meta["reduce"]:
        if "dtype" in row:
            code = row["dtype"]
            xs = list(golden[row["key"] + "_inputs"])
            outs = [x.copy() for x in xs]
            fn = fnptr(O, "orc_sum_i32" if code == 2 else "orc_sum_f16")
            host.reduce_threads(outs, None, row["root"], dtype_code=code,
                                max_segment=row["max_segment"], reducer_fn=fn)
            assert np.array_equal(np.stack(outs), golden[row["key"]]), row["key"]
            continue
        outs, ins = _reduce_case_inputs(row)
        host.reduce_threads(outs, ins, row["root"], max_segment=row["max_segment"],
                            reducer_fn=fnptr(O, "orc_sum_f32"))
        if row["key"] in golden.files:
            exp = golden[row["key"]]
            assert np.array_equal(np.stack(outs).view(np.uint32), exp.view(np.uint32)), row["key"]
        else:
            exp = golden[row["key"] + "_root"]
            got = outs[row["root"]]
            assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), row["key"]


def test_reduce_oracle_vs_golden(golden, golden_meta, O):
    """The C restatement's root result against the reference's, every fp32 case (fold order
    under reduce's own segment geometry) and the in-place int32/float16 cases."""
    for row in golden_meta["reduce"]:
        root = row["root"]
        if "dtype" in row:
            xs = list(golden[row["key"] + "_inputs"])
            outs = [x.copy() for x in xs]
            O.reduce(outs, None, root, dtype_code=row["dtype"], max_segment=row["max_segment"])
            assert np.array_equal(outs[root], golden[row["key"]][root]), row["key"]
            continue
        outs, ins = _reduce_case_inputs(row)
        O.reduce(outs, ins, root, max_segment=row["max_segment"])
        exp = golden[row["key"]][root] if row["key"] in golden.files else \
            golden[row["key"] + "_root"]
        assert np.array_equal(outs[root].view(np.uint32), exp.view(np.uint32)), row["key"]


@pytest.mark.parametrize("P", [1, 2, 4, 7])
@pytest.mark.parametrize("inplace", [True, False])
def test_reduce_test_default(O, P, inplace):
    """ReduceTest.Default (test/reduce_test.cc:22-86): uint64, maxSegmentSize 128, every rank
    takes a turn as root, closed form j*P^2 + P(P-1)/2 on the root."""
    for n in (1, 10, 100, 1000, 10000):
        for root in range(P):
            vals = [np.arange(n, dtype=np.uint64) * P + r for r in range(P)]
            if inplace:
                outs, ins = [v.copy() for v in vals], None
            else:
                outs, ins = [np.zeros(n, np.uint64) for _ in range(P)], vals
            host.reduce_threads(outs, ins, root, max_segment=128,
                                reducer_fn=fnptr(O, "orc_sum_u64"))
            exp = np.arange(n, dtype=np.uint64) * P * P + np.uint64(P * (P - 1) // 2)
            assert np.array_equal(outs[root], exp), (P, n, root, inplace)


def test_reduce_timeout_raises_io_exception(golden_meta):
    """ReduceTest.TestTimeout (reduce_test.cc:91-108): same text as the reference's."""
    rc, what = host.reduce_timeout_probe(10)
    assert rc == 0 and "Timed out waiting 10ms for recv operation to complete" in what
    assert "Timed out waiting 10ms for recv operation to complete" in \
        golden_meta["reduce_timeout_probe"]


def test_reduce_large_vs_reference(O):
    """Past the 1 MiB segment cap (many segments per rank), fp32 stress inputs: root bit-exact
    against the live reference when it is built, else the C restatement."""
    P, n = 3, 1_000_003
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = [np.zeros(n, np.float32) for _ in range(P)]
    host.reduce_threads(outs, [x.copy() for x in xs], 2, reducer_fn=fnptr(O, "orc_sum_f32"))
    exp = [np.zeros(n, np.float32) for _ in range(P)]
    if O.ref_available():
        O.ref_reduce(exp, [x.copy() for x in xs], 2)
        for r in range(P):
            assert np.array_equal(outs[r].view(np.uint32), exp[r].view(np.uint32)), r
    else:
        O.reduce(exp, [x.copy() for x in xs], 2)
        assert np.array_equal(outs[2].view(np.uint32), exp[2].view(np.uint32))


@pytest.mark.parametrize("chunked", [False, True])
def test_allreduce_test_single_pointer_p1_to_15(O, chunked):
    """AllreduceTest SinglePointer (test/allreduce_test.cc:138-164, 236-244) on the host
    runtime's old-style AllreduceRing<float> / AllreduceRingChunked<float>: P = 1..15 ranks
    each holding `rank`, n in {4, 100, 1000, 10000}; every rank must hold P(P-1)/2."""
    fn = fnptr(O, "orc_isum_f32")
    for P in range(1, 16):
        for n in (4, 100, 1000, 10000):
            bufs = [[np.full(n, float(r), np.float32)] for r in range(P)]
            host.allreduce_ring_old_threads(bufs, dtype_code=6, reducer_fn=fn, chunked=chunked)
            for r in range(P):
                assert np.all(bufs[r][0] == P * (P - 1) / 2), (P, n, r)


@pytest.mark.extra
def test_halving_doubling_vs_golden(O, golden_algo):
    """hydra::AllreduceHalvingDoubling<T> (allreduce_halving_doubling.h:37-358) reproduces the
    reference's result on every rank and pointer: one, two and three binary blocks (P = 1..12),
    tiny and ragged n (oracle in-place sum as the reducer)."""
    golden, meta = golden_algo
    names = {6: "orc_isum_f32", 2: "orc_isum_i32", 8: "orc_isum_f16"}
    for row in meta["halving_doubling"]:
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_halving_doubling_threads(bufs, dtype_code=row["dtype"],
                                                reducer_fn=fnptr(O, names[row["dtype"]]))
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                got = bufs[r][i]
                assert np.array_equal(got.view(f"u{got.itemsize}"),
                                      exp.view(f"u{exp.itemsize}")), (key, r, i)


@pytest.mark.extra
@pytest.mark.parametrize("P,n", [(4, (1 << 20) + 7), (6, 300001), (7, 1 << 18), (13, 70001)])
def test_halving_doubling_large(O, P, n):
    """Messages far beyond the socket buffers (the FIFO transport must not deadlock) with
    every cross-block leg active; bit-exact vs the oracle."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    bufs = [[x.copy()] for x in xs]
    host.allreduce_halving_doubling_threads(bufs, reducer_fn=fnptr(O, "orc_isum_f32"))
    exp = [[x.copy()] for x in xs]
    O.allreduce_halving_doubling(exp)
    for r in range(P):
        assert np.array_equal(bufs[r][0].view(np.uint32), exp[r][0].view(np.uint32)), r


@pytest.mark.extra
def test_bcube_old_vs_golden(O, golden_algo):
    """Old-style hydra::AllreduceBcube<T> (allreduce_bcube.h:255-691) reproduces the
    reference's own class on every rank and pointer (P = 1, 2, 4, 8; 1-2 pointers; f32 / i32
    / f16), with the oracle in-place sum as the reducer."""
    golden, meta = golden_algo
    names = {6: "orc_isum_f32", 2: "orc_isum_i32", 8: "orc_isum_f16"}
    for row in meta["bcube_old"]:
        key, P, k = row["key"], row["P"], row["nptr"]
        ins = golden[key + "_in"]
        bufs = [[ins[r, i].copy() for i in range(k)] for r in range(P)]
        host.allreduce_bcube_old_threads(bufs, dtype_code=row["dtype"],
                                         reducer_fn=fnptr(O, names[row["dtype"]]))
        exp = golden[key + "_out"]
        for r in range(P):
            for i in range(k):
                got = bufs[r][i]
                assert np.array_equal(got.view(f"u{got.itemsize}"),
                                      exp.view(f"u{exp.itemsize}")), (key, r, i)


@pytest.mark.extra
def test_bcube_old_rejects_non_power_of_two(O):
    """The reference's ranks disagree for such P; the drop-in refuses them."""
    bufs = [[np.ones(10, np.float32)] for _ in range(3)]
    with pytest.raises(Exception, match="power of the base"):
        host.allreduce_bcube_old_threads(bufs, reducer_fn=fnptr(O, "orc_isum_f32"))


@pytest.mark.extra
@pytest.mark.parametrize("P,nptr,n", [(1, 1, 100), (1, 3, 1000), (2, 4, 4099), (3, 2, 0)])
def test_allreduce_local(O, P, nptr, n):
    """gloo::AllreduceLocal<T> (allreduce_local.cc:28-38): each rank's pointers left-folded in
    pointer order into ptrs[0] (x = x op ptrs[i]), then copied to every pointer; ranks do not
    communicate."""
    xs = [[synth.stress_f32(nptr, i, n, seed=90 + r) for i in range(nptr)] for r in range(P)]
    bufs = [[x.copy() for x in r] for r in xs]
    host.allreduce_ring_old_threads(bufs, reducer_fn=fnptr(O, "orc_isum_f32"), local=True)
    for r in range(P):
        exp = xs[r][0].copy()
        for i in range(1, nptr):
            exp = exp + xs[r][i]  # float32 numpy add == the in-place fp32 sum, RNE
        for i in range(nptr):
            assert np.array_equal(bufs[r][i].view(np.uint32), exp.view(np.uint32)), (r, i)


def test_slow_peer_after_timeout_lands_nowhere():
    """a timeout must poison the context like the reference's signalException
    (tcp/unbound_buffer.cc:66-76), not leave the op queued on its pair.  Rank 0 times out, rank 1
    (slow, not dead) sends 300 ms later: rank 0 raises "Timed out waiting ...", its refilled
    bucket stays untouched by the late bytes, and later collectives on the context fail."""
    rc, what, intact = host.slow_peer_probe(50, 300)
    assert rc == 0, (rc, what)
    assert "Timed out waiting 50ms" in what
    assert intact
