"""The multi-GPU schedules (hydra_amd/csrc/xgmi_plan.h), checked on the CPU.

1. Functional: every rank's plan, interpreted with numpy copies for the p2p groups and the
   oracle's reduction for REDUCE/FOLD, reproduces the reference ring's result bit-exactly
   (fold order!) for P = 2..8, ragged sizes, maxSegmentSize 128 / 1 MiB and several chunk sizes.
2. Races: on the two-stream execution model the RCCL executor uses (comm stream: p2p groups;
   compute stream: REDUCE/FOLD; cross-stream edges: the plan's wait0/wait1), every pair of
   conflicting accesses (same bytes, at least one write) is ordered by happens-before.
"""
import numpy as np
import pytest

from benchkit import allreduce as bench_ar
from hydra_amd import _lib, ring, synth

from plan_interp import (ALLGATHER, ALLTOALL, FOLD, GROUP, RECV, REDUCE, SEND,  # noqa: E402,F401
                         fold_slot, interpret, run_plan_numpy)


CASES = [(P, n, ms, ch) for P in (2, 3, 4, 5, 8) for (n, ms, ch) in
         [(1, 0, 0), (7, 128, 0), (1000, 128, 64), (4099, 128, 1024), (10007, 1 << 20, 4096),
          (262145, 0, 0), (262145, 0, 65536)]]


A2A_CASES = [(P, n, ms) for P in (2, 3, 4, 5, 8) for (n, ms) in
             [(1 << 16, 0), (3 * 5 * 7 * 1024, 1024), (1 << 20, 4096)]]


def _a2a_ok(P, n, ms, es=4):
    ns, sb, S = _lib.ring_plan(P, n, es, ms or (1 << 20))
    return S * sb * P == n * es


@pytest.mark.parametrize("P,n,ms", A2A_CASES)
def test_a2a_plan_matches_reference_fold(O, P, n, ms):
    if not _a2a_ok(P, n, ms):
        with pytest.raises(_lib.HydraError):
            ring.plan("a2a", P, 0, n, 4, ms, 0)
        return
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, "a2a", xs, ms, 0)
    exp = O.ring_result(xs, ms or (1 << 20))
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp.view(np.uint32))
    for r in range(P):
        race_check(ring.plan("a2a", P, r, n, 4, ms, 0)[0])


def test_a2a_covers_baseline_buckets():
    """BASELINE config 4 (64 Mi fp32) and 5 (256 Mi bf16) have equal blocks at P = 2..8."""
    for P in (2, 4, 8):
        assert _a2a_ok(P, 64 << 20, 0, 4) and _a2a_ok(P, 256 << 20, 0, 2)


@pytest.mark.parametrize("algo", ["ring", "direct"])
@pytest.mark.parametrize("P,n,ms,ch", CASES)
def test_plan_matches_reference_fold(O, algo, P, n, ms, ch):
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, algo, xs, ms, ch)
    exp = O.ring_result(xs, ms or (1 << 20))
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp.view(np.uint32)), (algo, r)


@pytest.mark.parametrize("algo", ["ring", "direct"])
def test_plan_int32_and_f16(O, algo):
    P, n = 4, 5003
    xs = [synth.int32_bucket(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, algo, xs, 256, 512, code=2)
    exp = O.ring_result(xs, 256)
    assert all(np.array_equal(o, exp) for o in outs)
    rng = np.random.default_rng(2)
    hs = [np.array([O.f2h(float(v)) for v in rng.uniform(-4, 4, n)], np.uint16) for _ in range(P)]
    outs = run_plan_numpy(O, algo, hs, 256, 512, code=8)
    exp = O.ring_result(hs, 256, dtype_code=8)
    assert all(np.array_equal(o, exp) for o in outs)


def _accesses(o, P=None):
    """(buffer, lo, hi, is_write) byte ranges an op touches (collectives: conservatively the
    whole region they read/write on this rank)."""
    if o["kind"] in (SEND, RECV):
        return [(o["buf"], o["off"], o["off"] + o["bytes"], o["kind"] == RECV)]
    if o["kind"] in (ALLTOALL, ALLGATHER):
        span = o["bytes"] * (P or 1)
        if o["kind"] == ALLTOALL:
            return [(0, o["off"], o["off"] + span, False),
                    (1, o["src_off"], o["src_off"] + span, True)]
        return [(0, o["off"], o["off"] + span, True), (0, o["off"], o["off"] + span, False)]
    acc = [(0, o["off"], o["off"] + o["bytes"], True), (0, o["off"], o["off"] + o["bytes"], False)]
    if o["kind"] == REDUCE:
        acc.append((1, o["src_off"], o["src_off"] + o["bytes"], False))
    else:
        for j in range(1, o["nsrc"]):
            lo = fold_slot(o, j)
            acc.append((1, lo, lo + o["bytes"], False))
    return acc


def race_check(ops):
    """Units: each p2p group (its SEND/RECVs + GROUP) on the comm stream; each REDUCE/FOLD on
    the compute stream.  Edges: stream order + wait0/wait1.  Every conflicting pair of units on
    different streams must be ordered (in plan order) by happens-before."""
    units = []  # (stream, accesses, waits(list of op idx), op index of unit end)
    unit_of = {}
    P = max([o["nsrc"] for o in ops if o["kind"] == FOLD] + [1])
    i = 0
    while i < len(ops):
        o = ops[i]
        if o["kind"] in (ALLTOALL, ALLGATHER):
            units.append(("c", _accesses(o, P), [o["wait0"], o["wait1"]], i))
            unit_of[i] = len(units) - 1
            i += 1
            continue
        if o["kind"] in (REDUCE, FOLD):
            units.append(("k", _accesses(o), [o["wait0"], o["wait1"]], i))
            unit_of[i] = len(units) - 1
            i += 1
        else:
            g = i
            acc = []
            while ops[g]["kind"] != GROUP:
                acc += _accesses(ops[g])
                g += 1
            units.append(("c", acc, [ops[g]["wait0"], ops[g]["wait1"]], g))
            for j in range(i, g + 1):
                unit_of[j] = len(units) - 1
            i = g + 1
    U = len(units)
    preds = [set() for _ in range(U)]
    last = {"c": None, "k": None}
    for u, (st, _, waits, _) in enumerate(units):
        if last[st] is not None:
            preds[u].add(last[st])
        for w in waits:
            if w >= 0:
                preds[u].add(unit_of[w])
        last[st] = u
    hb = [set() for _ in range(U)]  # transitive predecessors
    for u in range(U):
        for p in preds[u]:
            hb[u] |= hb[p] | {p}
    for b in range(U):
        for a in range(b):
            if units[a][0] == units[b][0] or a in hb[b]:
                continue
            for (ba, la, ha, wa) in units[a][1]:
                for (bb, lb, hb_, wb) in units[b][1]:
                    if ba == bb and la < hb_ and lb < ha and (wa or wb):
                        raise AssertionError(f"race: unit {a} {units[a][0]} vs {b} {units[b][0]}")


@pytest.mark.parametrize("algo", ["ring", "direct"])
@pytest.mark.parametrize("P,n,ms,ch", [c for c in CASES if c[1] > 100])
def test_plan_is_race_free(algo, P, n, ms, ch):
    for r in range(P):
        ops, _ = ring.plan(algo, P, r, n, 4, ms, ch)
        race_check(ops)


def test_race_checker_catches_missing_wait():
    ops, _ = ring.plan("direct", 4, 0, 100000, 4, 1024, 4096)
    bad = [dict(o) for o in ops]
    for o in bad:
        if o["kind"] == FOLD:
            o["wait0"] = -1
            break
    with pytest.raises(AssertionError):
        race_check(bad)


def test_scratch_is_small_for_small_buckets():
    ops, scr = ring.plan("direct", 8, 0, 1000, 4)
    assert scr <= 2 * 7 * 512


def test_plan_geometry_matches_ring_plan():
    """Block ownership comes from allreduce.cc:199-221: the FOLD/REDUCE of the last hop covers
    exactly this rank's block [rS*sb, (r+1)S*sb)."""
    P, n = 5, 3000001
    ns, sb, S = _lib.ring_plan(P, n, 4, 1 << 20)
    for r in range(P):
        ops, _ = ring.plan("direct", P, r, n, 4, 0, 0)
        folds = [o for o in ops if o["kind"] == FOLD]
        lo = min(o["off"] for o in folds)
        hi = max(o["off"] + o["bytes"] for o in folds)
        assert lo == min(4 * n, r * S * sb) and hi == min(4 * n, (r + 1) * S * sb)


@pytest.mark.parametrize("P,n,ch", [(2, 1, 0), (3, 1000, 256), (5, 4099, 1024), (8, 100003, 4096),
                                    (4, 262145, 0)])
def test_ring_old_plan(O, P, n, ch):
    """Old-style AllreduceRing<T> on device (plan RING_OLD): per-rank left folds, bit-exact vs
    the oracle restatement (pinned to the reference by tests/test_oracle.py), and race-free."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, "ring_old", xs, 0, ch)
    bufs = [[x.copy()] for x in xs]
    O.allreduce_ring_old(bufs)
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), bufs[r][0].view(np.uint32)), r
        race_check(ring.plan("ring_old", P, r, n, 4, 0, ch)[0])


@pytest.mark.parametrize("P,n", [(2, 1), (2, 100), (3, 1000), (5, 4099), (8, 4099), (8, 100003),
                                 (4, 262145), (7, 1 << 16)])
def test_ring_chunked_plan(O, P, n):
    """AllreduceRingChunked<T> on device (plan RING_CHUNKED): every rank bit-exact vs the oracle
    restatement (pinned to the reference by tests/test_oracle.py), and race-free."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, "ring_chunked", xs, 0, 0)
    bufs = [[x.copy()] for x in xs]
    O.allreduce_ring_chunked(bufs)
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), bufs[r][0].view(np.uint32)), r
        race_check(ring.plan("ring_chunked", P, r, n, 4, 0, 0)[0])


def test_ring_chunked_plan_traffic():
    """Each rank sends and receives 4P-4 chunks (2P-2 folds), as allreduce_ring_chunked.h does."""
    P, n = 8, 1 << 20
    for r in range(P):
        ops, scr = ring.plan("ring_chunked", P, r, n, 4, 0, 0)
        kinds = [o["kind"] for o in ops]
        assert kinds.count(SEND) == kinds.count(RECV) == 4 * P - 4
        assert kinds.count(REDUCE) == 2 * P - 2
        assert scr == 2 * (n // (2 * P)) * 4


def test_bench_self_check_helpers(O):
    """bench.py's numpy self-checks agree with the oracle (they run on the GPU box, where the
    oracle is not used by the product path)."""
    P, n = 5, 4099
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    a = [[x.copy()] for x in xs]
    O.allreduce_ring_chunked(a)
    assert np.array_equal(bench_ar.expected_chunked_ring_f32(xs).view(np.uint32),
                          a[0][0].view(np.uint32))
    b = [[x.copy()] for x in xs]
    O.allreduce_ring_old(b)
    for r in range(P):
        assert np.array_equal(bench_ar.expected_old_ring_f32(xs, r).view(np.uint32),
                              b[r][0].view(np.uint32))
    assert np.array_equal(bench_ar.expected_fold_f32(xs).view(np.uint32),
                          O.ring_result(xs).view(np.uint32))
    for P2 in (1, 2, 6, 8, 12):
        ys = [synth.stress_f32(P2, r, n) for r in range(P2)]
        assert np.array_equal(bench_ar.expected_bcube_f32(ys).view(np.uint32),
                              O.bcube_result(ys).view(np.uint32)), P2


@pytest.mark.parametrize("P,n", [(2, 1), (2, 1000), (3, 7), (4, 4099), (6, 100003), (8, 262145),
                                 (12, 30011), (5, 100)])
def test_bcube_plan(O, P, n):
    """BCUBE on device (plan BCUBE): bit-exact vs the oracle's BCUBE (pinned to the reference by
    tests/test_oracle.py) on every rank, and race-free."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, "bcube", xs, 0, 0)
    exp = O.bcube_result(xs)
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp.view(np.uint32)), r
        race_check(ring.plan("bcube", P, r, n, 4, 0, 0)[0])


def _reduce_plans(root, P, n, es, ms, ch):
    plans, scr = [], 0
    for r in range(P):
        ops, s = ring.plan_reduce(root, P, r, n, es, ms, ch)
        plans.append(ops)
        scr = max(scr, s)
    return plans, scr


@pytest.mark.parametrize("P,n,ms,ch", [(2, 1, 0, 0), (2, 1000, 128, 256), (3, 4099, 128, 1024),
                                       (4, 262145, 0, 0), (7, 10007, 4096, 2048),
                                       (8, 300001, 0, 1 << 16)])
def test_reduce_root_plan_matches_reference(O, P, n, ms, ch):
    """hydra_reduce_root (gloo::reduce to a root on device): the root's bucket equals the
    reference's root output bit for bit (gloo::reduce's own geometry, reference fold order),
    for every root; every rank's plan is race-free."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    for root in range(P):
        plans, scr = _reduce_plans(root, P, n, 4, ms, ch)
        outs = run_plan_numpy(O, None, xs, ms, ch, plans=plans, scr=scr)
        exp = [x.copy() for x in xs]
        O.reduce(exp, None, root, max_segment=ms or (1 << 20))
        assert np.array_equal(outs[root].view(np.uint32), exp[root].view(np.uint32)), root
        for ops in plans:
            race_check(ops)


def test_reduce_root_geometry_is_gloo_reduce():
    """The plan's blocks follow gloo::reduce's segment geometry (reduce.cc:87-135), which is
    not the allreduce ring's: e.g. 5 MiB of fp32 at P = 2 gives 6 segments of 1 MiB
    (the ring: 6 segments of 873 816 B)."""
    from oracle import oracle as Oc

    assert Oc.reduce_plan(2, 1310720, 4, 1 << 20) == (6, 1 << 20, 3)
    assert Oc.ring_plan(2, 1310720, 4, 1 << 20) == (6, 873816, 3)
    for P, n, ms in [(3, 4099, 128), (8, 1 << 24, 1 << 20), (7, 1, 128), (2, 1310720, 1 << 20)]:
        ns, sb, S = Oc.reduce_plan(P, n, 4, ms)
        ops, _ = ring.plan_reduce(0, P, 0, n, 4, ms, 0)
        # the root receives exactly the other owners' blocks
        got = sorted((o["off"], o["off"] + o["bytes"]) for o in ops
                     if o["kind"] == RECV and o["buf"] == 0)
        blocks = []
        for q in range(1, P):
            lo, hi = min(n * 4, q * S * sb), min(n * 4, (q + 1) * S * sb)
            if hi > lo:
                blocks.append((lo, hi))
        def merge(spans):
            out = []
            for lo, hi in sorted(spans):
                if out and out[-1][1] == lo:
                    out[-1] = (out[-1][0], hi)
                else:
                    out.append((lo, hi))
            return out

        assert merge(got) == merge(blocks), (P, n, ms)


def test_bench_reduce_self_check_helper(O):
    """bench.py's gloo::reduce self-check (bench_ar.expected_reduce_f32, not the oracle) equals the
    oracle's root result, and its geometry helper equals the oracle's."""
    for P, n in [(1, 100), (2, 1 << 20), (3, 1_000_003), (8, 1 << 20), (5, 77)]:
        assert bench_ar.reduce_geometry(P, n, 4) == O.reduce_plan(P, n, 4, 1 << 20)
        xs = [synth.stress_f32(P, r, n) for r in range(P)]
        exp = [x.copy() for x in xs]
        O.reduce(exp, None, P - 1)
        assert np.array_equal(bench_ar.expected_reduce_f32(xs).view(np.uint32),
                              exp[P - 1].view(np.uint32)), (P, n)


@pytest.mark.extra
@pytest.mark.parametrize("P,n", [(2, 1), (2, 1000), (3, 7), (4, 4099), (5, 100), (6, 100003),
                                 (7, 262145), (8, 30011), (11, 5000), (12, 3), (13, 20011)])
def test_halving_doubling_plan(O, P, n):
    """AllreduceHalvingDoubling<T> on device (plan HALVING_DOUBLING): bit-exact vs the oracle's
    restatement (pinned to the reference by tests/test_oracle.py) on every rank, one to three
    binary blocks and fewer elements than chunks, and race-free."""
    xs = [synth.stress_f32(P, r, n) for r in range(P)]
    outs = run_plan_numpy(O, "halving_doubling", xs, 0, 0)
    exp = [[x.copy()] for x in xs]
    O.allreduce_halving_doubling(exp)
    for r in range(P):
        assert np.array_equal(outs[r].view(np.uint32), exp[r][0].view(np.uint32)), r
        race_check(ring.plan("halving_doubling", P, r, n, 4, 0, 0)[0])


BOUNDS_ALGOS = ["ring", "direct", "ring_old", "ring_chunked", "bcube", pytest.param("halving_doubling", marks=pytest.mark.extra)]


@pytest.mark.parametrize("algo", BOUNDS_ALGOS)
def test_every_plan_passes_the_executor_bounds_check(algo):
    """Regression for the round-1 GPU fault hunt: hydra_plan now runs the same validate_plan the
    RCCL executor, the simulator and the run_plan hook run before enqueueing anything (every
    access inside n*E user bytes and plan_scratch_bytes, groups closed, waits backwards).  Sweep
    every rank of ragged geometries, every element size and RING_OLD's small chunks (the
    round-1 suspect); a plan that reaches outside its buffers raises here, on the CPU."""
    sizes = [1, 2, 7, 100, 1000, 4099, 30011, 300000]
    for P in (2, 3, 5, 8, 16):
        for n in sizes:
            for es in (1, 2, 4, 8):
                for ms, ch in ((0, 0), (128, 1024), (64, 16), (1 << 20, 1 << 18)):
                    if n * es // max(ch, 1 << 12) > 64 or (ms and n * es // ms > 256):
                        continue  # keep plans small: the geometry, not the length, is under test
                    for r in sorted({0, 1, P // 2, P - 1}):
                        ops, scr = ring.plan(algo, P, r, n, es, ms, ch)
                        for o in ops:  # belt and braces: the same bounds, restated
                            if o["kind"] in (SEND, RECV):
                                cap = n * es if o["buf"] == 0 else scr
                                assert 0 <= o["off"] and o["off"] + o["bytes"] <= cap
                            elif o["kind"] == REDUCE:
                                assert o["off"] + o["bytes"] <= n * es
                                assert o["src_off"] + o["bytes"] <= scr


def test_plan_bounds_check_covers_reduce_root():
    for P in (2, 3, 7):
        for n in (1, 1000, 4099, 262145):
            for root in range(P):
                for r in range(P):
                    ring.plan_reduce(root, P, r, n, 4, 128, 1024)


def test_auto_is_a2a_on_equal_blocks_and_default_chunk_is_16mib():
    """HYDRA_ALGO_AUTO resolves to A2A (three launches: ncclAllToAll, one fold, ncclAllGather)
    when the reference geometry gives P equal blocks, else DIRECT; the default pipelining chunk
    is 16 MiB, which keeps config 4's DIRECT enqueue at 62 plan ops."""
    kinds = lambda ops: {o["kind"] for o in ops}  # noqa: E731
    ops, _ = ring.plan("auto", 8, 0, 64 << 20, 4, 0, 0)
    assert kinds(ops) == {_lib.OP_ALLTOALL, _lib.OP_FOLD, _lib.OP_ALLGATHER}, kinds(ops)
    ops3, _ = ring.plan("auto", 3, 0, 1 << 20, 4, 0, 0)  # 1 Mi fp32 at P=3: unequal blocks
    assert _lib.OP_ALLTOALL not in kinds(ops3) and _lib.OP_SEND in kinds(ops3)
    d_default, _ = ring.plan("direct", 8, 0, 64 << 20, 4, 0, 0)
    d16, _ = ring.plan("direct", 8, 0, 64 << 20, 4, 0, 16 << 20)
    d4, _ = ring.plan("direct", 8, 0, 64 << 20, 4, 0, 4 << 20)
    assert len(d_default) == len(d16) == 62 and len(d4) == 248, (len(d_default), len(d4))
