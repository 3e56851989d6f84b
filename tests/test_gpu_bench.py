"""bench.py's N>1 path (hydra_amd/ring.py bench_allreduce) at world size 1 on the GPU: the same
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


def test_bench_multi_path_world1(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    p = subprocess.run([sys.executable, "-u", "bench.py", "--force-dist", "--steps", "5",
                        "--warmup", "1", "--config5-elements", str(1 << 20),
                        "--watchdog-s", "100"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["value"] > 0
    parity = res["parity"]["fold_order_1M"]
    for algo in ("direct", "ring", "a2a", "ring_old", "ring_chunked", "bcube", "reduce_root",
                 "apipe"):
        assert parity[algo] == "bit-exact", (algo, parity)
    assert not any(v == "MISMATCH" for v in parity.values()), parity
    assert all(res["parity"]["full_size_exact"].values()), res["parity"]
    assert "watchdog" not in res, res
    # every context leg measured (bounded waits, none expired), config 5 checked and timed
    assert all(isinstance(v, float) for v in res["other_algos_ms"].values()), res
    assert "error" not in res["config5_bf16"] and res["config5_bf16"]["elements"] == 1 << 20
    assert res["parity"]["full_size_exact"]["config5_bf16_acc32"] is True
