"""The N>1 bench orchestration (benchkit.allreduce.bench_allreduce, what `bench.py --gpus N` runs on
each rank) at world size 2, 3, 4 and 8 (the driver's node) on the CPU: the same code path the driver's 8-GPU run takes --
fold-order parity self-checks of every schedule, the safe DIRECT headline, the autotune over
bit-exact candidates, full-size exactness, the timed region with max over ranks, the context
schedules' parity and timings, gloo::reduce to a root, the two-rail split, and the JSON line --
with the communicator swapped for tests/gloo_plan_exec.GlooPlanComm (the library's own plans
over gloo p2p, the oracle folding) and the device sync for a no-op.  Every rank must take the
same branches (a divergence deadlocks a collective and fails the test by its timeout) and the
line must report every schedule bit-exact."""
import argparse
import os
import socket

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, stall_rank=-1, stall_waits=0, extra_legs=False, peer="auto",
            peer_fail_at=-1):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    import bench
    from gloo_plan_exec import GlooPlanComm
    from benchkit import allreduce as bench_ar
    from oracle import oracle as O

    dist.init_process_group("gloo", rank=rank, world_size=world)
    comms = []

    left = [stall_waits]  # bounded waits that expire on stall_rank (-1: every one)

    class Stalled(GlooPlanComm):
        """As if this rank's work never finished: its bounded waits expire."""

        def wait(self, timeout_ms, stream=None):
            from hydra_amd._lib import HydraError

            if left[0] != 0:
                left[0] -= 1
                raise HydraError(5, f"Timed out waiting {timeout_ms}ms for allreduce to complete")

    def make_comm():
        comms.append((Stalled if rank == stall_rank else GlooPlanComm)(O))
        return comms[-1]

    class FakePeer:
        """hydra_amd.peer.PeerComm's interface over the gloo plans (DIRECT: the same reference
        fold order as the peer kernel): the peer leg's orchestration on the CPU."""

        def __init__(self):
            self.comm, self.closed = GlooPlanComm(O), False
            self.registered = []
            self.calls, self.err = 0, 0
            if peer_fail_at != -1:  # the device group's bounded barriers: a gloo group whose
                # collectives time out when a peer never arrives (then the group is poisoned)
                from datetime import timedelta

                self.group = dist.new_group(backend="gloo", timeout=timedelta(seconds=3))

        def register(self, t):
            self.registered.append(t.data_ptr())

        def set_option(self, key, value):
            pass

        def allreduce_(self, t, algo="peer2", **kw):
            assert t.data_ptr() in self.registered, "allreduce of an unregistered bucket"
            from hydra_amd._lib import HydraError

            self.calls += 1
            bf16 = kw.get("dtype_code") is not None
            if peer_fail_at == -1 or (peer_fail_at == -2 and not bf16):
                self.comm.allreduce_(t, algo="direct", **kw)
                return
            if self.err:  # a poisoned group refuses at once (hydra_peer_allreduce)
                raise HydraError(3, "peer group is broken: an earlier barrier timed out")
            if rank == 1 and (peer_fail_at == -2 or peer_fail_at < self.calls):
                # this rank's call fails locally (-2: its first config-5 call)
                raise HydraError(1, f"injected failure at peer call {self.calls}")
            if bf16:  # (-2) the other rank's call: its barrier waits for rank 1, and expires
                try:
                    dist.all_gather([torch.empty_like(t) for _ in range(world)], t,
                                    group=self.group)
                except RuntimeError:
                    self.err = 1
                return
            got = [torch.empty_like(t) for _ in range(world)]
            try:  # every rank's bucket, then the reference fold (the peer kernel's result)
                dist.all_gather(got, t, group=self.group)
            except RuntimeError:
                self.err = 1  # the barrier timed out: the kernel's error word
                return
            t.copy_(torch.from_numpy(bench_ar.expected_fold_f32([g.numpy() for g in got])))

        def error(self):
            return self.err

        def close(self):
            self.closed = True

    peers = []

    def make_peer():
        peers.append(FakePeer())
        return peers[-1]

    try:
        args = argparse.Namespace(elements=1 << 16, steps=3, warmup=1, algo="auto",
                                  watchdog_s=600.0, no_config5=False, config5_elements=1 << 20,
                                  peer=peer, extra_legs=extra_legs)
        base = ((lambda P, n: bench.ring_cpu_baseline(P, n, 0.5)) if O.ref_available() else None)
        res = bench_ar.bench_allreduce(args, torch.device("cpu"), make_comm=make_comm,
                                   sync=lambda: None, cpu_baseline=base, make_peer=make_peer)
        q.put((rank, res, all(c.closed for c in comms + peers) and len(comms) == 2))
    except Exception as e:  # report instead of hanging the parent
        import traceback

        q.put((rank, repr(e) + traceback.format_exc(), False))
    finally:
        dist.destroy_process_group()


def ph_algo_ok(pl):
    """the phase entry is the timed schedule's"""
    return pl["phases"].get("algo") == pl["algo"]


def _start(world, stall_rank=-1, stall_waits=0, extra_legs=False, peer="auto", peer_fail_at=-1):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, stall_rank, stall_waits,
                                               extra_legs, peer, peer_fail_at))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = {}
        for _ in range(world):
            r, res, closed = q.get(timeout=300)
            out[r] = (res, closed)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return out


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_bench_allreduce_orchestration(world):
    """The default line: north_star's schedules only (DIRECT / A2A / RING / RCCL, config 5, the
    two rails), the communicator's own rank count, and the reference ring's CPU baseline."""
    from oracle import oracle as O

    out = _start(world)
    for r, (res, closed) in out.items():
        assert isinstance(res, dict), res
        assert closed, f"rank {r} left a communicator open"
    res = out[0][0]
    assert res["n_gpus"] == world and res["scaling"] == "weak" and res["value"] > 0
    par = res["parity"]["fold_order_1M"]
    for a in ("direct", "ring", "apipe"):
        assert par[a] == "bit-exact", (a, par)
    # no leg outside north_star by default
    assert not set(par) & {"ring_old", "ring_chunked", "bcube", "reduce_root"}, par
    assert not set(res["other_algos_ms"]) & {"ring_old", "ring_chunked", "bcube",
                                             "halving_doubling", "reduce_root0"}, res
    # A2A needs P equal reference blocks: 1 Mi fp32 has them at P = 2, 4 and 8, not at P = 3
    assert (par["a2a"] == "bit-exact" if world != 3 else par["a2a"].startswith("n/a")), par
    assert all(res["parity"]["full_size_exact"].values()), res["parity"]
    # the full-size gate is fold-order-sensitive -- DIRECT's bucket on
    # synth.stress_at data, pinned to the reference fold on sampled indices and equal across
    # ranks; every other schedule must equal it bit for bit
    g = res["parity"]["full_size_gate"]
    assert g["ok"] and g["data"] == "stress_at" and g["sampled_equal_reference_fold"], g
    assert g["sha256_equal_across_ranks"] and g["sampled_indices"] >= (1 << 16) // 2, g
    assert res["config"]["algo"] in ("direct", "a2a", "ring")
    assert res["config"]["autotune_ms"], res["config"]
    for a in ("ring", "direct", "rccl", "rccl_rs_ag", "apipe_direct"):
        if a == "rccl_rs_ag" and (1 << 16) % world:  # RCCL's reduce-scatter needs n % P == 0
            assert res["other_algos_ms"][a].startswith("n/a"), res["other_algos_ms"]
        elif a != res["config"]["algo"]:
            assert isinstance(res["other_algos_ms"][a], float), (a, res["other_algos_ms"])
    c5 = res["config5_bf16"]  # config 5's leg (bf16, fp32 accumulate) ran, at 1 Mi here
    assert "error" not in c5 and c5["elements"] == 1 << 20 and c5["ms"] > 0, c5
    assert res["parity"]["full_size_exact"]["config5_bf16_acc32"] is True, res["parity"]
    g5 = c5["full_size_gate"]  # config 5's gate: stress_cancel_at, bf16 acc32 reference fold
    assert g5["ok"] and g5["data"] == "stress_cancel_at", g5
    # the communicator's own rank count, the same on every rank
    rc = res["rccl_comm"]
    assert rc["nccl_comm_count"] == rc["min_over_ranks"] == rc["max_over_ranks"] == world, rc
    # the reference ring on P thread-ranks beside the line (rank 0 only)
    cb = res["cpu_baseline"]
    if O.ref_available():
        assert cb["kind"] == "reference" and cb["value"] > 0 and cb["cores"] == 2 * world, cb
    # every rank reports the same (max-over-ranks) timing
    assert all(out[r][0]["ms_per_step"] == res["ms_per_step"] for r in out)
    # the line's own roofline evidence: one profiled allreduce split into link and fold time
    # (VERDICT r03 next #1), for config 4 and config 5, and the fused-sum bytes as traffic
    rf = res["roofline"]
    assert rf["traffic"] == int((world - 1) / world * (1 << 16) * 12), rf
    assert rf["traffic_kind"].startswith("algorithmic"), rf
    for ph, esize, n in ((rf["phases"], 4, 1 << 16), (c5["phases"], 2, 1 << 20)):
        assert isinstance(ph, dict), ph
        assert ph["calls"] == 1 and ph["link_ms"] > 0 and ph["fold_ms"] > 0, ph
        assert ph["span_ms"] >= max(ph["link_ms"], ph["fold_ms"]) * 0.999, ph
        assert ph["bound"] in ("link", "fold") and ph["overlap_ms"] >= 0, ph
        lk, fd = ph["link"], ph["fold"]
        # every schedule moves at least the reference ring's per-rank link bytes
        assert lk["algorithmic_bytes"] == int(2 * (world - 1) / world * n * esize), lk
        assert lk["sent_bytes"] >= lk["algorithmic_bytes"] * 0.999, lk
        assert 1 <= lk["peers"] <= world - 1 and lk["per_link_GBps"] > 0, lk
        assert "frac_of_link" in lk and "frac_of_hbm" in fd, ph
        assert fd["fused_sum_bytes"] == int((world - 1) / world * n * 3 * esize), fd
        assert fd["kernel_hbm_bytes"] > 0 and fd["ops"] >= 1, fd
    # the peer leg (auto): no GPU peer links here, so it states why it did not run
    pl = res["peer_leg"]
    assert pl["enabled"] is False and pl["mode"] == "auto", pl
    assert pl["reason"].startswith("skipped: no GPU peer links"), pl


@pytest.mark.parametrize("world", [2, 4])
def test_bench_peer_leg_orchestration(world):
    """the reduce-on-read leg (forced on here; on an xGMI node "auto" turns
    it on) runs last -- parity of both schedules, full-size exactness, workgroup autotune, the
    timed region under the bench contract, and one event-timed phase entry against the link and
    HBM rooflines -- and replaces the headline only when it is faster."""
    out = _start(world, peer="on")
    for r, (res, closed) in out.items():
        assert isinstance(res, dict), res
        assert closed, f"rank {r} left a communicator or peer group open"
    res = out[0][0]
    pl = res["peer_leg"]
    assert pl["enabled"] and pl["mode"] == "on" and "error" not in pl, pl
    assert pl["parity_fold_order_1M"] == {"peer2": "bit-exact", "peer2w": "bit-exact",
                                          "peer1": "bit-exact"}, pl
    assert pl["full_size_exact"] is True and pl["ms_per_step"] > 0, pl
    assert pl["full_size_exact_by_algo"] == {"peer2w": True, "peer2": True}, pl
    # both two-shot schedules x the workgroup counts; a GPU per rank (no shared-GPU cap): two
    # workgroups per CU is a candidate too
    assert set(pl["autotune_ms"]) == {f"{a}/{w}wg" for a in ("peer2", "peer2w")
                                      for w in (0, 512, 128, 64)}, pl
    assert pl["algo"] in ("peer2", "peer2w") and ph_algo_ok(pl), pl
    ph = pl["phases"]
    assert ph["kernel_ms"] > 0 and ph["link"]["algorithmic_bytes"] == int(
        2 * (world - 1) / world * (1 << 16) * 4), ph
    assert ph["link"]["peers"] == world - 1 and ph["fold"]["frac_of_hbm"] > 0, ph
    assert pl["full_size_gate"].startswith("equal to this run's DIRECT bucket"), pl
    # config 5 through the peer schedule too: gated against config 5's DIRECT bucket, timed
    p5 = pl["config5"]
    assert p5["full_size_exact"] is True and p5["ms"] > 0 and p5["algo"] == pl["algo"], p5
    assert res["config5_bf16"]["peer"] == p5, res["config5_bf16"]
    if pl["promoted"]:
        a = pl["algo"]
        assert res["config"]["algo"] == a and res["ms_per_step"] == pl["ms_per_step"]
        assert res["parity"]["full_size_exact"][a] is True
        # the promoted headline carries its own phase entry and parity
        assert res["roofline"]["phases"] == ph, res["roofline"]
        assert res["parity"]["fold_order_1M"][a] == "bit-exact", res["parity"]
    else:
        assert not res["config"]["algo"].startswith("peer") and \
            res["ms_per_step"] <= pl["ms_per_step"]
    assert all(out[r][0]["peer_leg"]["promoted"] == pl["promoted"] for r in out)


@pytest.mark.parametrize("fail_at,stage", [(5, "autotune"), (61, "timed region")])
def test_bench_peer_leg_one_rank_fails_mid_loop(fail_at, stage):
    """a peer call that fails on ONE rank inside the autotune (its 6th call: after 3
    parity and 2 full-size calls) or the timed region (its 62nd: after 2 x 4 x 7 autotune calls,
    the first timed step) -- that rank records it and keeps issuing the
    same collectives; its peers' calls end at their bounded barrier (the fake group's 3 s
    timeout, the kernel's error word on a GPU) -- so the leg ends with an error entry of that
    stage on every rank, nobody is stranded and the RCCL headline stands."""
    out = _start(2, peer="on", peer_fail_at=fail_at)
    for r, (res, closed) in out.items():
        assert isinstance(res, dict), res
        assert closed, f"rank {r} left a communicator or peer group open"
        pl = res["peer_leg"]
        assert pl.get("error", "").startswith(stage) and not pl.get("promoted"), pl
        assert res["config"]["algo"] != "peer2" and res["value"] > 0, res["config"]
    assert "injected failure" in out[1][0]["peer_leg"]["error"], out[1][0]["peer_leg"]


def test_bench_peer_leg_config5_fails_on_one_rank():
    """Config 5 through the peer schedule fails on ONE rank (its first bf16 call, the gate): the
    other rank's call ends at its bounded barrier, both record the error in the config-5 entry,
    and the config-4 peer result -- gated and timed before -- stands."""
    out = _start(2, peer="on", peer_fail_at=-2)
    for r, (res, closed) in out.items():
        assert isinstance(res, dict), res
        assert closed, f"rank {r} left a communicator or peer group open"
        pl = res["peer_leg"]
        assert "error" not in pl and pl["full_size_exact"] and pl["ms_per_step"] > 0, pl
        p5 = pl["config5"]
        assert p5["error"].startswith("full size") and "ms" not in p5, p5
        assert res["config5_bf16"]["peer"] == p5 and res["config5_bf16"]["ms"] > 0
    assert "injected failure" in out[1][0]["peer_leg"]["config5"]["error"]


def test_bench_allreduce_extra_legs():
    """--extra-legs adds the schedules outside north_star's path, each bit-exact."""
    out = _start(3, extra_legs=True)
    res = out[0][0]
    assert isinstance(res, dict), res
    par = res["parity"]["fold_order_1M"]
    for a in ("ring_old", "ring_chunked", "bcube", "reduce_root"):
        assert par[a] == "bit-exact", (a, par)
    for a in ("ring_old", "ring_chunked", "bcube", "halving_doubling", "reduce_root0"):
        assert isinstance(res["other_algos_ms"][a], float), (a, res["other_algos_ms"])


def _run(world, stall_rank, stall_waits):
    out = _start(world, stall_rank, stall_waits, extra_legs=True)
    for r, (res, _) in out.items():
        assert isinstance(res, dict), res
    return {r: res for r, (res, _) in out.items()}


def test_context_waits_expiring_on_one_rank():
    """Every bounded wait after the headline expires on rank 1 (its communicator would be
    aborted): every context leg is n/a on EVERY rank, the headline and its parity stand, and the
    run completes -- nobody is stranded in a collective."""
    out = _run(3, 1, -1)
    for r, res in out.items():
        par = res["parity"]["fold_order_1M"]
        for a in ("ring_old", "ring_chunked", "bcube", "reduce_root", "apipe"):
            assert par[a].startswith("n/a"), (r, a, par)
        assert all(str(v).startswith("n/a") for v in res["other_algos_ms"].values()), res
        assert "error" in res["config5_bf16"], res["config5_bf16"]
    res = out[0]
    assert res["parity"]["fold_order_1M"]["direct"] == "bit-exact" and res["value"] > 0
    assert "another rank failed" in res["parity"]["fold_order_1M"]["ring_old"]
    assert "Timed out" in out[1]["parity"]["fold_order_1M"]["ring_old"]


def test_one_expired_wait_costs_one_leg():
    """Only rank 1's first bounded wait (the old-style ring's parity check) expires: that entry
    is n/a on every rank, every later leg is measured."""
    out = _run(2, 1, 1)
    res = out[0]
    par = res["parity"]["fold_order_1M"]
    assert par["ring_old"].startswith("n/a"), par
    for a in ("ring_chunked", "bcube", "reduce_root", "apipe"):
        assert par[a] == "bit-exact", (a, par)
    assert all(isinstance(v, float) for v in res["other_algos_ms"].values()), res
    assert "error" not in res["config5_bf16"], res["config5_bf16"]
