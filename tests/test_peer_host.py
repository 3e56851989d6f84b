"""Host logic of hydra_amd.peer on CPU (gloo, world size 2): setup and registration fail
COLLECTIVELY -- a rank whose HIP call fails still joins every exchange, so its peer raises
HydraError instead of waiting for it forever (the bench relies on this to drop the peer
algorithms cleanly).  The C-ABI is replaced by a fake; no GPU call is made."""
import ctypes
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakeLib:
    """The hydra_peer_* entry points the Python layer calls; `fail` names the one that fails."""

    def __init__(self, fail):
        self.fail = fail
        self.calls = []

    def _rc(self, name):
        self.calls.append(name)
        return 2 if name == self.fail else 0

    def hydra_last_error(self):
        return b"injected failure"

    def hydra_peer_create(self, world, rank, dev, hptr, sig):
        ctypes.memset(sig, 0x5A, 128)
        return self._rc("create")

    def hydra_peer_connect(self, h, allsig):
        assert len(allsig) == 2 * 128
        return self._rc("connect")

    def hydra_peer_register(self, h, ptr, nbytes, blob):
        ctypes.memset(blob, 0x33, 128)
        return self._rc("register")

    def hydra_peer_open(self, h, ptr, nbytes, allh):
        return self._rc("open")

    def hydra_peer_close(self, h, ptr):
        self.calls.append("close")
        return 0

    def hydra_peer_set_option(self, h, k, v):
        return 0

    def hydra_peer_detach(self, h):
        self.calls.append("detach")
        return 0

    def hydra_peer_destroy(self, h):
        return 0


class FakeTensor:
    is_cuda = True

    def is_contiguous(self):
        return True

    def numel(self):
        return 1024

    def element_size(self):
        return 4

    def data_ptr(self):
        return 0x1000


def _worker(rank, port, fail_rank, fail_at, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from hydra_amd import _lib, peer

    fake = FakeLib(fail_at if rank == fail_rank else None)
    _lib.lib = lambda: fake  # the module reads _lib.lib() at call time
    dist.init_process_group("gloo", rank=rank, world_size=2)
    out = {}
    try:
        try:
            pc = peer.PeerComm(rank, 2, 0)
            out["init"] = "ok"
        except _lib.HydraError as e:
            out["init"] = f"raised: {e}"
            pc = None
        if pc is not None:
            try:
                pc.register(FakeTensor())
                out["register"] = "ok"
            except _lib.HydraError as e:
                out["register"] = f"raised: {e}"
        out["calls"] = fake.calls
        dist.barrier()
    finally:
        dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.parametrize("fail_at", ["create", "connect", "register", "open", None])
def test_peer_setup_fails_collectively(fail_at):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, 1, fail_at, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    if fail_at is None:
        assert all(res[r]["init"] == "ok" and res[r]["register"] == "ok" for r in (0, 1))
    elif fail_at in ("create", "connect"):
        assert all(res[r]["init"].startswith("raised") for r in (0, 1)), res
    else:
        assert all(res[r]["init"] == "ok" for r in (0, 1))
        assert all(res[r]["register"].startswith("raised") for r in (0, 1)), res
        if fail_at == "open":  # the rank that did map undoes it, so both agree
            assert "close" in res[0]["calls"]
        assert "injected failure" in res[1]["register"]
