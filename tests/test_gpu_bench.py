"""bench.py's N>1 path (benchkit/allreduce.py bench_allreduce) at world size 1 on the GPU: the same
code the driver's multi-GPU scale run executes per rank -- RCCL communicators, the fold-order
parity self-check of every schedule, the full-size exactness check, the autotune and the
context phase -- must finish with rc 0 and a JSON line whose parity entries are all bit-exact
(or n/a for a schedule that does not apply).  World size 1 is the most this pool allows; the
schedules' N>1 behaviour is covered on the CPU by tests/test_dist_gloo.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra=()):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "-u", "bench.py", "--force-dist", "--steps", "5",
                        "--warmup", "1", "--config5-elements", str(1 << 20),
                        "--watchdog-s", "100", "--cpu-seconds", "2", *extra],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_bench_multi_path_world1(gpu):
    """The default line: north_star's schedules, RCCL's own rank count, the reference ring's
    CPU baseline (rank 0), config 5, the two rails."""
    res = _run()
    assert res["n_gpus"] == 1 and res["value"] > 0
    parity = res["parity"]["fold_order_1M"]
    for algo in ("direct", "ring", "a2a", "apipe"):
        assert parity[algo] == "bit-exact", (algo, parity)
    assert not any(v == "MISMATCH" for v in parity.values()), parity
    assert all(res["parity"]["full_size_exact"].values()), res["parity"]
    assert "watchdog" not in res, res
    # every context leg measured (bounded waits, none expired), config 5 checked and timed
    assert all(isinstance(v, float) for v in res["other_algos_ms"].values()), res
    assert "ring_old" not in res["other_algos_ms"] and "ring_old" not in parity, res
    assert "error" not in res["config5_bf16"] and res["config5_bf16"]["elements"] == 1 << 20
    assert res["parity"]["full_size_exact"]["config5_bf16_acc32"] is True
    # what RCCL itself counted (ncclCommCount) and the reference ring's CPU baseline
    rc = res["rccl_comm"]
    assert rc["nccl_comm_count"] == rc["min_over_ranks"] == rc["max_over_ranks"] == 1, rc
    assert rc["backend"] == "rccl" and rc["device"] == 0, rc
    cb = res["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["value"] > 0 and cb["cores"] == 2, cb
    # the peer leg states why it did not run at world 1 (auto mode)
    pl = res["peer_leg"]
    assert pl["enabled"] is False and pl["reason"] == "skipped: one rank: no peer to read from", pl


def test_bench_rehearsal_world2_peer_leg(gpu):
    """The N>1 line at world 2 with two real RCCL ranks sharing the one GPU
    (HYDRA_BENCH_SHARED_GPU=1: each rank its own NCCL_HOSTID, sockets), as the driver launches it
    (torch.distributed.run), with the peer-access leg forced on: every schedule bit-exact, and the
    peer leg's parity, full-size check, autotune, timed region and phase entry all present."""
    env = dict(os.environ, HYDRA_BENCH_SHARED_GPU="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(_free_port()), "bench.py", "--gpus", "2", "--steps", "5", "--warmup",
                        "1", "--elements", str(1 << 20), "--config5-elements", str(1 << 20),
                        "--cpu-seconds", "1", "--watchdog-s", "150", "--peer", "on"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-3000:])
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["value"] > 0 and "rehearsal" in res, res
    assert res["rccl_comm"]["nccl_comm_count"] == 2, res["rccl_comm"]
    par = res["parity"]["fold_order_1M"]
    for algo in ("direct", "ring", "a2a", "apipe"):
        assert par[algo] == "bit-exact", (algo, par)
    # the full-size gate on fold-order-sensitive data
    g = res["parity"]["full_size_gate"]
    assert g["ok"] and g["data"] == "stress_at" and g["sha256_equal_across_ranks"], g
    pl = res["peer_leg"]
    assert pl["enabled"] and "error" not in pl, pl
    assert pl["parity_fold_order_1M"] == {"peer2": "bit-exact", "peer2w": "bit-exact",
                                          "peer1": "bit-exact"}, pl
    assert pl["full_size_exact"] is True and pl["ms_per_step"] > 0, pl
    assert pl["full_size_exact_by_algo"] == {"peer2w": True, "peer2": True}, pl
    assert pl["phases"]["kernel_ms"] > 0 and pl["phases"]["link"]["peers"] == 1, pl
    # BASELINE config 5 (bf16, fp32 accumulate) through the chosen peer schedule, gated against
    # the config-5 DIRECT bucket before it is timed
    p5 = pl["config5"]
    assert "error" not in p5 and p5["full_size_exact"] is True and p5["ms"] > 0, p5
    assert res["config5_bf16"]["peer"] == p5, res["config5_bf16"]
    if pl["promoted"]:
        assert res["config"]["algo"] == pl["algo"] in ("peer2", "peer2w"), res["config"]


@pytest.mark.extra
def test_bench_multi_path_world1_extra_legs(gpu):
    res = _run(["--extra-legs"])
    parity = res["parity"]["fold_order_1M"]
    for algo in ("ring_old", "ring_chunked", "bcube", "reduce_root"):
        assert parity[algo] == "bit-exact", (algo, parity)
    assert all(isinstance(v, float) for v in res["other_algos_ms"].values()), res


def test_bench_single_gpu_line(gpu):
    """bench.py at N = 1 (the driver's default command, smaller here): the contract's fields --
    roofline with HIP-event achieved bytes, the CPU baseline pinned to the GPU's NUMA node with
    every repetition, and the host-buffer (PCIe-inclusive) context leg, exact on its first call."""
    p = subprocess.run([sys.executable, "-u", "bench.py", "--elements", str(1 << 22), "--steps",
                        "20", "--warmup", "2", "--cpu-seconds", "0.5"],
                       cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["dtype"] == "f32", res
    rf = res["roofline"]
    assert rf["bound"] == "hbm" and rf["peak"] == 8000.0 and 0 < rf["frac"] < 1, rf
    cb = res["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["cores"] == 1 and cb["value"] > 0, cb
    assert len(cb["repetitions_GBps"]) == 3 and cb["pinned_cpu"] != 0, cb
    hp = res["host_path"]
    for kind in ("pinned_zero_copy", "pageable_staged"):
        assert hp[kind]["first_call_exact"] and hp[kind]["GBps"] > 0, hp
    # config 2's size range: every size 4 Ki .. 64 Mi, both residencies,
    # the smallest labelled dispatch-bound and the largest HBM-bound
    sw = res["sweep"]
    assert "error" not in sw, sw
    assert [r["elements"] for r in sw["rows"]] == [1 << k for k in range(12, 27, 2)], sw
    for r in sw["rows"]:
        for kind in ("hbm_resident", "mall_assisted", "hbm_resident_graph"):
            assert r[kind]["GBps"] > 0 and 0 < r[kind]["frac_of_peak"] < 3, r
    assert sw["rows"][0]["bound"] == "dispatch" and sw["rows"][-1]["bound"] == "hbm", sw
    si = res["sweep_int32"]  # the same range for int32 (SURVEY 8(d) names both dtypes)
    assert "error" not in si and len(si["rows"]) == len(sw["rows"]), si
