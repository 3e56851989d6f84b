"""Peer-access bucket allreduce over xGMI (hydra_peer_*, include/hydra_hip.h).

The MI355X-first form of gloo::allreduce RING (allreduce.cc:147-422) for device-resident
buckets: every rank maps the other ranks' buckets by hipIpc handles, and ONE gfx950 kernel per
allreduce reads the peers' blocks straight over xGMI and folds them in the reference's order
(hydra_amd/csrc/peer_fold.h), so the result is bit-identical to RING / DIRECT.

Handle exchange rides on torch.distributed (all_gather_object: gloo or nccl process groups);
the library itself only produces and consumes byte blobs.

    peer = PeerComm(rank, world, device_index)   # collective
    peer.register(bucket)                        # collective, once per bucket tensor
    peer.allreduce_(bucket, algo="peer2")        # one kernel on the current stream
"""
from __future__ import annotations

import ctypes
import sys

from . import _lib
from ._lib import HydraError, OPS, PEER_ALGOS, check

_is_finalizing = sys.is_finalizing


def _all_gather_bytes(blob: bytes, group=None) -> list:
    import torch.distributed as dist

    out = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, blob, group=group)
    return out


def _agree(ok: bool, group=None) -> bool:
    """Collective AND: every rank learns whether every rank succeeded."""
    return all(_all_gather_bytes(b"1" if ok else b"0", group)[i] == b"1"
               for i in range(_world(group)))


def _world(group=None) -> int:
    import torch.distributed as dist

    return dist.get_world_size(group)


class PeerComm:
    """hydra_peer_t: signal area + IPC mappings of the registered buckets of all ranks.

    Setup steps are collective and fail collectively: a rank whose HIP call fails still joins
    every exchange, so its peers raise HydraError too instead of waiting for it forever."""

    def __init__(self, rank: int, world: int, device_index: int, group=None,
                 timeout_ms: int | None = None, blocks: int | None = None):
        self._h = ctypes.c_void_p()
        self.rank, self.world, self.group = rank, world, group
        self._registered: dict[int, int] = {}  # data_ptr -> bytes
        sig = ctypes.create_string_buffer(_lib.PEER_HANDLE_BYTES)
        err = None
        rc = _lib.lib().hydra_peer_create(world, rank, device_index, ctypes.byref(self._h), sig)
        if rc:
            err = HydraError(rc, _lib.lib().hydra_last_error().decode(errors="replace"))
        allsig = _all_gather_bytes(sig.raw if err is None else b"", group)
        if err is None and any(len(b) != _lib.PEER_HANDLE_BYTES for b in allsig):
            err = HydraError(3, "a peer failed to create its signal area")
        if err is None:
            rc = _lib.lib().hydra_peer_connect(self._h, b"".join(allsig))
            if rc:
                err = HydraError(rc, _lib.lib().hydra_last_error().decode(errors="replace"))
        if not _agree(err is None, group):
            self.close()
            raise err or HydraError(3, "a peer failed to map the signal areas")
        if timeout_ms is not None:
            self.set_option(_lib.PEER_OPT_TIMEOUT_MS, timeout_ms)
        if blocks is not None:
            self.set_option(_lib.PEER_OPT_BLOCKS, blocks)

    def set_option(self, key: int, value: int) -> None:
        check(_lib.lib().hydra_peer_set_option(self._h, key, int(value)))

    def register(self, t) -> None:
        """Collective: share device tensor t's memory with every rank (same call order on all
        ranks).  t must stay alive while registered; allreduce_ accepts t or any view of it."""
        nbytes = t.numel() * t.element_size()
        blob = ctypes.create_string_buffer(_lib.PEER_HANDLE_BYTES)
        err = None
        if not t.is_cuda or not t.is_contiguous():
            err = HydraError(1, "register: contiguous device tensor required")
        else:
            rc = _lib.lib().hydra_peer_register(self._h, t.data_ptr(), nbytes, blob)
            if rc:
                err = HydraError(rc, _lib.lib().hydra_last_error().decode(errors="replace"))
        allh = _all_gather_bytes(blob.raw if err is None else b"", self.group)
        if err is None and any(len(b) != _lib.PEER_HANDLE_BYTES for b in allh):
            err = HydraError(3, "a peer failed to export its buffer")
        if err is None:
            rc = _lib.lib().hydra_peer_open(self._h, t.data_ptr(), nbytes, b"".join(allh))
            if rc:
                err = HydraError(rc, _lib.lib().hydra_last_error().decode(errors="replace"))
        if not _agree(err is None, self.group):
            if err is None:  # mapped here, failed elsewhere: undo so every rank agrees
                _lib.lib().hydra_peer_close(self._h, t.data_ptr())
            raise err or HydraError(3, "a peer failed to map the buffer")
        self._registered[t.data_ptr()] = nbytes

    def unregister(self, t) -> None:
        """Collective: every rank closes its mappings of t's peers, then all meet, so t (on
        any rank) may be freed once this returns (teardown rule in include/hydra_hip.h)."""
        rc = _lib.lib().hydra_peer_close(self._h, t.data_ptr())
        self._registered.pop(t.data_ptr(), None)
        _agree(rc == 0, self.group)
        check(rc)

    def allreduce_(self, t, algo: str = "peer2", op: str = "sum", dtype_code: int | None = None,
                   flags: int = 0, max_segment: int = 0, stream: int | None = None) -> None:
        """In-place allreduce of registered device tensor t on the current (or given) stream.
        algo: "peer2" (two-shot), "peer2w" (two-shot push: the fold stores into every bucket),
        "peer1" (one-shot), "peer" (AUTO: the push, or one-shot up to PEER_OPT_ONE_SHOT_MAX bytes)."""
        import torch

        from .reduce import _torch_dtype_code
        from .ring import _count

        code = dtype_code if dtype_code is not None else _torch_dtype_code(t)
        if not t.is_contiguous():
            raise HydraError(1, "allreduce_: contiguous tensor required")
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        check(_lib.lib().hydra_peer_allreduce(self._h, PEER_ALGOS[algo], OPS[op], code, flags,
                                              t.data_ptr(), _count(t, code), max_segment, s))

    def error(self) -> int:
        """0 while healthy; a barrier-timeout code once a peer failed to arrive."""
        c = ctypes.c_int()
        check(_lib.lib().hydra_peer_error(self._h, ctypes.byref(c)))
        return c.value

    def close(self, collective: bool = True) -> None:
        """Collective teardown (include/hydra_hip.h): detach every mapping of the other ranks'
        memory, meet them, then free this rank's signal area -- no rank ever frees memory a
        peer still maps.  collective=False (garbage collection) skips the meeting."""
        if self._h:
            _lib.lib().hydra_peer_detach(self._h)
            if collective:
                try:
                    _agree(True, self.group)
                except Exception:  # the process group is gone: nobody left to wait for
                    pass
            _lib.lib().hydra_peer_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        if _is_finalizing():  # no HIP calls while the interpreter is finalizing
            return
        try:
            self.close(collective=False)
        except Exception:
            pass
