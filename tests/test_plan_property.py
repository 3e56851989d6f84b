"""Property-based parity of the device allreduce plans (xgmi_plan.h), on the CPU.

hypothesis draws the geometry -- ranks, element count, maxSegmentSize, pipelining chunk, input
seed -- and every rank's plan is executed by the numpy interpreter (tests/plan_interp.py, the
HIP kernels' fold order restated with the oracle's element ops).  The expected bytes come from
the REFERENCE ITSELF when oracle/_ref is built (its own gloo::allreduce RING / BCUBE,
AllreduceRing<T>, AllreduceRingChunked<T>, AllreduceHalvingDoubling<T> and gloo::reduce on
loopback thread-ranks), else from the C restatement.  Bit-exact on every rank (fp32
fold-order-sensitive inputs); derandomized, so a failure reproduces."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from hydra_amd import ring, synth

from plan_interp import run_plan_numpy  # noqa: E402

SETTINGS = dict(max_examples=60, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])

geometry = dict(P=st.integers(2, 8), n=st.integers(1, 3000),
                ms=st.sampled_from([4, 8, 12, 128, 1000, 4096, 1 << 20]),
                ch=st.sampled_from([0, 16, 48, 1024, 4096]), seed=st.integers(0, 10 ** 6))


def inputs(P, n, seed):
    return [synth.stress_f32(P, r, n, seed=seed + r) for r in range(P)]


def expect_new_style(O, xs, ms, algorithm=1):
    outs = [[x.copy()] for x in xs]
    if O.ref_available():
        O.ref_allreduce(len(xs), outs, None, max_segment=ms, algorithm=algorithm)
    else:
        O.allreduce(len(xs), outs, None, max_segment=ms, algorithm=algorithm)
    return [o[0] for o in outs]


def assert_ranks(got, exp, ctx):
    for r, (g, e) in enumerate(zip(got, exp)):
        assert np.array_equal(g.view(np.uint32), e.view(np.uint32)), (ctx, r)


@pytest.mark.parametrize("algo", ["ring", "direct"])
@settings(**SETTINGS)
@given(**geometry)
def test_ring_and_direct_plans_vs_reference(O, algo, P, n, ms, ch, seed):
    """RING and DIRECT: gloo::allreduce's RING bits (allreduce.cc:147-422) on every rank."""
    xs = inputs(P, n, seed)
    got = run_plan_numpy(O, algo, xs, ms, ch)
    assert_ranks(got, expect_new_style(O, xs, ms), (algo, P, n, ms, ch))


@settings(**SETTINGS)
@given(**geometry)
def test_bcube_plan_vs_reference(O, P, n, ms, ch, seed):
    """BCUBE: gloo::allreduce's BCUBE bits (allreduce.cc:423-700); it ignores maxSegmentSize
    and the pipelining chunk, which the draw varies anyway."""
    xs = inputs(P, n, seed)
    got = run_plan_numpy(O, "bcube", xs, ms, ch)
    assert_ranks(got, expect_new_style(O, xs, ms, algorithm=2), ("bcube", P, n))


@pytest.mark.parametrize("algo", ["ring_old", "ring_chunked", pytest.param("halving_doubling", marks=pytest.mark.extra)])
@settings(**SETTINGS)
@given(P=st.integers(2, 8), n=st.integers(1, 3000), ch=st.sampled_from([0, 16, 48, 1024]),
       seed=st.integers(0, 10 ** 6))
def test_old_style_plans_vs_reference(O, algo, P, n, ch, seed):
    """The old-style classes: AllreduceRing<T> (each rank its own left fold), AllreduceRingChunked
    <T> and AllreduceHalvingDoubling<T> -- every rank's bits."""
    xs = inputs(P, n, seed)
    got = run_plan_numpy(O, algo, xs, 0, ch)
    bufs = [[x.copy()] for x in xs]
    ref = O.ref_available()
    if algo == "ring_old":
        (O.ref_allreduce_ring_old if ref else O.allreduce_ring_old)(bufs)
    elif algo == "ring_chunked":
        (O.ref_allreduce_ring_chunked if ref else O.allreduce_ring_chunked)(bufs)
    else:
        (O.ref_allreduce_halving_doubling if ref else O.allreduce_halving_doubling)(bufs)
    assert_ranks(got, [b[0] for b in bufs], (algo, P, n, ch))


@settings(**SETTINGS)
@given(**geometry)
def test_reduce_root_plan_vs_reference(O, P, n, ms, ch, seed):
    """gloo::reduce to a drawn root (reduce.cc:21-262): the root's bucket."""
    root = seed % P
    xs = inputs(P, n, seed)
    plans, scr = [], 0
    for r in range(P):
        ops, s = ring.plan_reduce(root, P, r, n, 4, ms, ch)
        plans.append(ops)
        scr = max(scr, s)
    got = run_plan_numpy(O, "reduce", xs, ms, ch, plans=plans, scr=scr)
    exp = [x.copy() for x in xs]
    (O.ref_reduce if O.ref_available() else O.reduce)(exp, None, root, max_segment=ms)
    assert np.array_equal(got[root].view(np.uint32), exp[root].view(np.uint32)), (P, n, ms, root)
