"""World-size-2 (and 3) CPU runs of the N>1 path over torch.distributed gloo: the rank-local
plans from libhydra_hip.so executed with real inter-process p2p (tests/gloo_plan_exec.py), the
oracle's reduction standing in for the HIP kernels (CPU-only test of the distributed
orchestration), plus the bench harness helpers (unique-id broadcast, max-over-ranks timing)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, algo, n, ms, ch, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from gloo_plan_exec import execute
    from benchkit import allreduce as bench_ar
    from hydra_amd import ring, synth
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = synth.stress_f32(world, rank, n)
        root = world - 1  # algo "reduce": hydra_reduce_root's plan (gloo::reduce to a root)
        if algo == "reduce":
            ops, scr = ring.plan_reduce(root, world, rank, n, 4, ms, ch)
        else:
            ops, scr = ring.plan(algo, world, rank, n, 4, ms, ch)
        user = torch.from_numpy(x.copy().view(np.uint8))
        execute(O, ops, scr, user)
        got = user.numpy().view(np.float32)
        # harness helpers
        uid = ring.exchange_unique_id(rank, make_id=lambda: bytes(range(128)))
        assert uid == bytes(range(128))
        mx = bench_ar.max_over_ranks(float(rank + 1))
        assert mx == float(world)
        wall = bench_ar.timed_steps(lambda: None, 3, 1, lambda: None, dist.barrier)
        assert wall >= 0
        xs = [synth.stress_f32(world, r, n) for r in range(world)]
        if algo in ("ring_old", "ring_chunked", "halving_doubling"):  # the Algorithm classes
            olds = [[x.copy()] for x in xs]
            {"ring_old": O.allreduce_ring_old, "ring_chunked": O.allreduce_ring_chunked,
             "halving_doubling": O.allreduce_halving_doubling}[algo](olds)
            exp = olds[rank][0]
        elif algo == "bcube":
            exp = O.bcube_result(xs)
        elif algo == "reduce":  # only the root's bucket is defined
            outs = [x.copy() for x in xs]
            O.reduce(outs, None, root, max_segment=ms or (1 << 20))
            exp = outs[root] if rank == root else got
        else:
            exp = O.ring_result(xs, ms or (1 << 20))
        q.put((rank, bool(np.array_equal(got.view(np.uint32), exp.view(np.uint32)))))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("algo", ["ring", "direct", "a2a", "ring_old", "ring_chunked",
                                  "bcube", "reduce", pytest.param("halving_doubling", marks=pytest.mark.extra)])
def test_gloo_multiprocess_plan(algo, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    n, ms, ch = (100003, 4096, 16384) if algo != "a2a" else (3 << 16, 4096, 0)
    procs = [ctx.Process(target=_worker, args=(r, world, port, algo, n, ms, ch, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=120) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert all(v is True for v in res.values()), res
