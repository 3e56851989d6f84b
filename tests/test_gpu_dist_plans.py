"""The device allreduce plans across PROCESSES with the product's gfx950 kernels: world size 2
and 4, every process on the test box's one GPU (RCCL refuses two ranks on one GPU, so the
messages travel over torch.distributed gloo, staged through host memory --
tests/gloo_plan_exec.py execute_device).  Each rank's REDUCE / FOLD ops are the library's own
hydra_reduce / hydra_fold launches on its GPU bucket, exactly as the RCCL executor issues them
(xgmi_allreduce.cpp launch_compute), so the cross-process schedule, the block ownership and the
fold order are checked end to end on the hardware against the reference's outputs (the oracle's
ring result, `allreduce.cc:147-422`; gloo::reduce; the old-style rings; bcube).  bf16 with fp32
accumulation (config 5; pinned to the reference ring in test_gpu_xgmi.py) is compared with the CPU
restatement of k_fold<bf16, ACC32> run on the same ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGOS = ["ring", "direct", "a2a", "ring_old", "ring_chunked", "bcube", "reduce"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _expected(O, algo, xs, rank, ms, root):
    if algo in ("ring_old", "ring_chunked"):
        olds = [[x.copy()] for x in xs]
        {"ring_old": O.allreduce_ring_old, "ring_chunked": O.allreduce_ring_chunked}[algo](olds)
        return olds[rank][0]
    if algo == "bcube":
        return O.bcube_result(xs)
    if algo == "reduce":
        outs = [x.copy() for x in xs]
        O.reduce(outs, None, root, max_segment=ms or (1 << 20))
        return outs[root]
    return O.ring_result(xs, ms or (1 << 20))


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    from gloo_plan_exec import BF16, execute, execute_device
    from hydra_amd import ring, synth
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    results = {}
    try:
        dev = torch.device("cuda", 0)
        root = world - 1
        for algo in ALGOS:
            n, ms, ch = (100003, 4096, 16384) if algo != "a2a" else (3 << 16, 4096, 0)
            if algo == "reduce":
                ops, scr = ring.plan_reduce(root, world, rank, n, 4, ms, ch)
            else:
                ops, scr = ring.plan(algo, world, rank, n, 4, ms, ch)
            xs = [synth.stress_f32(world, r, n) for r in range(world)]
            user = torch.from_numpy(xs[rank].copy().view(np.uint8)).to(dev)
            execute_device(ops, scr, user)
            got = user.cpu().numpy().view(np.float32)
            exp = _expected(O, algo, xs, rank, ms, root)
            if algo == "reduce" and rank != root:
                ok = True  # only the root's bucket is defined
            else:
                ok = bool(np.array_equal(got.view(np.uint32), exp.view(np.uint32)))
            results[algo] = ok
        # int32 (bit-exact by construction) and config 5's bf16 + fp32 accumulation
        n = 3 << 16
        for algo in ("direct", "a2a"):
            xi = synth.int32_bucket(world, rank, n)
            ops, scr = ring.plan(algo, world, rank, n, 4, 4096, 16384)
            user = torch.from_numpy(xi.copy().view(np.uint8)).to(dev)
            execute_device(ops, scr, user, code=2)
            ref = torch.from_numpy(xi.copy().view(np.uint8))
            execute(O, ops, scr, ref, code=2)
            results[f"{algo}_i32"] = bool(torch.equal(user.cpu(), ref))
            xb = synth.bf16_bits(synth.stress_f32(world, rank, n))
            ops, scr = ring.plan(algo, world, rank, n, 2, 4096, 16384)
            user = torch.from_numpy(xb.copy().view(np.uint8)).to(dev)
            execute_device(ops, scr, user, code=BF16)
            ref = torch.from_numpy(xb.copy().view(np.uint8))
            execute(O, ops, scr, ref, code=BF16)
            results[f"{algo}_bf16_acc32"] = bool(torch.equal(user.cpu(), ref))
        q.put((rank, results))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_plans_across_processes_with_gpu_kernels(gpu, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=110) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    bad = {r: v for r, v in res.items() if not (isinstance(v, dict) and all(v.values()))}
    assert not bad, bad
    assert set(res[0]) == set(ALGOS) | {"direct_i32", "a2a_i32", "direct_bf16_acc32",
                                        "a2a_bf16_acc32"}
