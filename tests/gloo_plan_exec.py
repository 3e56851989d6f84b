"""Executor of the device allreduce plans over torch.distributed gloo (test infrastructure).

`execute` runs one rank's op list (hydra_plan / hydra_reduce_root_plan, xgmi_plan.h) with real
inter-process p2p: SEND/RECV groups through batch_isend_irecv, ALLTOALL as p2p (gloo has no
alltoall), ALLGATHER through all_gather.  REDUCE / FOLD run
  * on a CPU bucket (default): through the oracle's element ops in the kernels' fold order (the
    C restatement standing in for the HIP kernels) -- the CPU suite's world-size 2/3 runs;
  * on a GPU bucket (`execute_device`): through the library's own gfx950 kernels
    (hydra_reduce / hydra_fold, exactly as the RCCL executor's launch_compute calls them), the
    gloo transport staging each message through host memory -- several processes sharing the
    one GPU of the test box (RCCL refuses two ranks on one GPU), so the plans run across
    processes with the product kernels (tests/test_gpu_dist_plans.py).
`GlooPlanComm` wraps the CPU form in XgmiComm's interface, so the N>1 bench orchestration
(benchkit.allreduce.bench_allreduce) runs unchanged at world size 2 and 3 on the CPU."""
import numpy as np

SEND, RECV, GROUP, REDUCE, FOLD, ALLTOALL, ALLGATHER = 1, 2, 3, 4, 5, 6, 7
_NP = {2: np.int32, 6: np.float32, 9: np.uint16}  # hydra_dtype_t INT32, FLOAT32, BFLOAT16
BF16 = 9


def _f32(h):
    return (h.astype(np.uint32) << np.uint32(16)).view(np.float32)


def _bf16(x):  # round to nearest even (finite values)
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    return ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) \
        .astype(np.uint16)


def fold_slot(o, j):
    """xgmi_plan.h fold_slot: scratch offset of contribution j of a FOLD."""
    if o["peer"] < 0:
        return o["src_off"] + (j - 1) * o["slot_stride"]
    return o["src_off"] + ((o["peer"] + j) % o["nsrc"]) * o["slot_stride"]


class _Prof:
    """hydra_comm_phases' totals for the synchronous executor (perf_counter per op)."""

    def __init__(self):
        import time

        self.clock = time.perf_counter
        self.d = dict(calls=0, link_ops=0, fold_ops=0, link_ms=0.0, fold_ms=0.0, span_ms=0.0,
                      sent_bytes=0, recv_bytes=0, fold_hbm_bytes=0, peers=0)
        self.peers = set()

    def op(self, comm, t0, sent=0, recv=0, hbm=0, peers=()):
        ms = (self.clock() - t0) * 1e3
        self.d["link_ms" if comm else "fold_ms"] += ms
        self.d["link_ops" if comm else "fold_ops"] += 1
        self.d["sent_bytes"] += sent
        self.d["recv_bytes"] += recv
        self.d["fold_hbm_bytes"] += hbm
        self.peers.update(peers)
        self.d["peers"] = len(self.peers)


def execute(O, ops, scratch_bytes, user, code=6, op="sum", prof=None):
    """Run `ops` on `user` (a contiguous CPU uint8 tensor, modified in place) on this rank.
    code BFLOAT16 is the ACC_F32 form (config 5): each fold in fp32 in the same order, one
    round to bf16 at the end, as k_fold<bf16, ACC32> computes it (sum only).  prof: a _Prof
    that accumulates per-op times and bytes as hydra_comm_phases does."""
    import time

    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(), dist.get_world_size()
    dt = _NP[code]
    scratch = torch.zeros(scratch_bytes + 16, dtype=torch.uint8)
    others = [q for q in range(world) if q != rank]
    c0 = time.perf_counter()
    i = 0
    while i < len(ops):
        o = ops[i]
        t0 = time.perf_counter()
        if o["kind"] in (ALLTOALL, ALLGATHER) and prof is not None:
            prof.peers.update(others)  # a collective sends to every other rank
        if o["kind"] == ALLTOALL:  # ncclAllToAll semantics via p2p
            B = o["bytes"]
            scratch[o["src_off"] + rank * B:o["src_off"] + (rank + 1) * B] = \
                user[o["off"] + rank * B:o["off"] + (rank + 1) * B]
            p2p = []
            for pr in range(world):
                if pr == rank:
                    continue
                p2p.append(dist.P2POp(dist.isend, user[o["off"] + pr * B:o["off"] + (pr + 1) * B],
                                      pr))
                p2p.append(dist.P2POp(dist.irecv, scratch[o["src_off"] + pr * B:
                                                          o["src_off"] + (pr + 1) * B], pr))
            for req in dist.batch_isend_irecv(p2p):
                req.wait()
            if prof is not None:
                prof.op(True, t0, B * (world - 1), B * (world - 1))
            i += 1
            continue
        if o["kind"] == ALLGATHER:
            B = o["bytes"]
            mine = user[o["off"] + rank * B:o["off"] + (rank + 1) * B].clone()
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            for pr in range(world):
                user[o["off"] + pr * B:o["off"] + (pr + 1) * B] = parts[pr]
            if prof is not None:
                prof.op(True, t0, B * (world - 1), B * (world - 1))
            i += 1
            continue
        if o["kind"] in (REDUCE, FOLD):
            u = user.numpy()
            sc = scratch.numpy()
            local = u[o["off"]:o["off"] + o["bytes"]].view(dt).copy()
            if code == BF16:
                srcs = ([sc[o["src_off"]:o["src_off"] + o["bytes"]]] if o["kind"] == REDUCE else
                        [sc[fold_slot(o, j):fold_slot(o, j) + o["bytes"]]
                         for j in range(1, o["nsrc"])])
                acc = _f32(srcs[-1].view(dt))
                for s_ in reversed(srcs[:-1]):
                    acc = _f32(s_.view(dt)) + acc
                out = _bf16(_f32(local) + acc)
            elif o["kind"] == REDUCE:
                recv = sc[o["src_off"]:o["src_off"] + o["bytes"]].view(dt)
                out = O.op(local, recv, op, code)
            else:
                slots = [sc[fold_slot(o, j):fold_slot(o, j) + o["bytes"]].view(dt)
                         for j in range(1, o["nsrc"])]
                acc = slots[-1].copy()
                for s in reversed(slots[:-1]):
                    acc = O.op(s.copy(), acc, op, code)
                out = O.op(local, acc, op, code)
            u[o["off"]:o["off"] + o["bytes"]] = out.view(np.uint8)
            if prof is not None:
                prof.op(False, t0, hbm=o["bytes"] * (3 if o["kind"] == REDUCE else o["nsrc"] + 1))
            i += 1
            continue
        g = i
        p2p = []
        sent = recv = 0
        dests = set()
        while ops[g]["kind"] != GROUP:
            it = ops[g]
            t = (user if it["buf"] == 0 else scratch)[it["off"]:it["off"] + it["bytes"]]
            p2p.append(dist.P2POp(dist.isend if it["kind"] == SEND else dist.irecv, t, it["peer"]))
            if it["kind"] == SEND:
                sent += it["bytes"]
                dests.add(it["peer"])
            else:
                recv += it["bytes"]
            g += 1
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()
        if prof is not None:
            prof.op(True, t0, sent, recv, peers=dests)
        i = g + 1
    if prof is not None:
        prof.d["calls"] += 1
        prof.d["span_ms"] += (time.perf_counter() - c0) * 1e3


_OPC = {"sum": 0, "product": 1, "max": 2, "min": 3}


def execute_device(ops, scratch_bytes, user, code=6, op="sum"):
    """`execute` on a GPU bucket (`user`: contiguous uint8 CUDA tensor, modified in place):
    REDUCE / FOLD are the library's kernels on the current stream; every p2p message is staged
    through host memory for gloo.  code BFLOAT16 folds with HYDRA_ACC_F32 (config 5)."""
    import ctypes

    import torch
    import torch.distributed as dist

    from hydra_amd import _lib

    L = _lib.lib()
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = user.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    scratch = torch.zeros(scratch_bytes + 16, dtype=torch.uint8, device=dev)
    es = np.dtype(_NP[code]).itemsize
    flags = 1 if code == BF16 else 0
    ub, sb = user.data_ptr(), scratch.data_ptr()

    def exchange(sends, recvs):  # [(device view, peer)] -> gloo p2p through host copies
        p2p, back = [], []
        for t, pr in sends:
            p2p.append(dist.P2POp(dist.isend, t.cpu(), pr))
        for t, pr in recvs:
            h = torch.empty(t.numel(), dtype=torch.uint8)
            p2p.append(dist.P2POp(dist.irecv, h, pr))
            back.append((t, h))
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()
        for t, h in back:
            t.copy_(h)

    i = 0
    while i < len(ops):
        o = ops[i]
        if o["kind"] == ALLTOALL:
            B = o["bytes"]
            scratch[o["src_off"] + rank * B:o["src_off"] + (rank + 1) * B] = \
                user[o["off"] + rank * B:o["off"] + (rank + 1) * B]
            exchange([(user[o["off"] + pr * B:o["off"] + (pr + 1) * B], pr)
                      for pr in range(world) if pr != rank],
                     [(scratch[o["src_off"] + pr * B:o["src_off"] + (pr + 1) * B], pr)
                      for pr in range(world) if pr != rank])
            i += 1
            continue
        if o["kind"] == ALLGATHER:
            B = o["bytes"]
            mine = user[o["off"] + rank * B:o["off"] + (rank + 1) * B].cpu()
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            for pr in range(world):
                if pr != rank:
                    user[o["off"] + pr * B:o["off"] + (pr + 1) * B].copy_(parts[pr])
            i += 1
            continue
        if o["kind"] == REDUCE:
            _lib.check(L.hydra_reduce(_OPC[op], code, ub + o["off"], ub + o["off"],
                                      sb + o["src_off"], o["bytes"] // es, stream))
            i += 1
            continue
        if o["kind"] == FOLD:
            srcs = (ctypes.c_void_p * o["nsrc"])(
                ub + o["off"], *[sb + fold_slot(o, j) for j in range(1, o["nsrc"])])
            _lib.check(L.hydra_fold(_OPC[op], code, flags, ub + o["off"], srcs, o["nsrc"],
                                    o["bytes"] // es, stream))
            i += 1
            continue
        g = i
        sends, recvs = [], []
        while ops[g]["kind"] != GROUP:
            it = ops[g]
            t = (user if it["buf"] == 0 else scratch)[it["off"]:it["off"] + it["bytes"]]
            (sends if it["kind"] == SEND else recvs).append((t, it["peer"]))
            g += 1
        exchange(sends, recvs)
        i = g + 1
    torch.cuda.current_stream(dev).synchronize()


class GlooPlanComm:
    """XgmiComm's interface over `execute` (the library still plans and validates every
    schedule: argument and geometry errors are the library's own HydraErrors)."""

    def __init__(self, O):
        import torch.distributed as dist

        self.O = O
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.closed = False
        self._prof = None

    def profile(self, enable):
        """XgmiComm.profile: per-op timing of the following calls (perf_counter here)."""
        self._prof = _Prof() if enable else None

    def phases(self):
        """XgmiComm.phases: hydra_comm_phases' fields."""
        return dict(self._prof.d) if self._prof is not None else dict(_Prof().d)

    def _code(self, t, dtype_code):
        from hydra_amd._lib import HydraError

        code = dtype_code if dtype_code is not None else {4: 6}.get(t.element_size(), -1)
        if code not in _NP:
            raise HydraError(2, "GlooPlanComm folds fp32, int32 and bf16 (ACC_F32) only")
        return code

    def allreduce_(self, t, algo="auto", op="sum", dtype_code=None, flags=0, max_segment=0,
                   chunk_bytes=0, stream=None):
        import torch
        import torch.distributed as dist

        from hydra_amd import ring
        from hydra_amd._lib import HydraError

        code = self._code(t, dtype_code)
        if (code == BF16) != bool(flags):
            raise HydraError(2, "GlooPlanComm: bf16 only with ACC_F32, ACC_F32 only for bf16")
        if code == BF16 and algo in ("rccl", "rccl_rs_ag"):
            raise HydraError(2, "ACC_F32 with RCCL")
        n = t.numel()
        if algo == "rccl_rs_ag" and n % self.world:
            raise HydraError(3, "RCCL_RS_AG needs n to be a multiple of the rank count")
        if algo in ("rccl", "rccl_rs_ag"):  # (RCCL's own orders: a tolerance, not the ring's)
            dist.all_reduce(t)
            return
        if n == 0 or self.world == 1:
            return
        ops, scr = ring.plan(algo, self.world, self.rank, n,
                             t.element_size(), max_segment, chunk_bytes)
        execute(self.O, ops, scr, t.view(-1).view(torch.uint8), code, op, self._prof)

    def reduce_(self, t, root, op="sum", dtype_code=None, flags=0, max_segment=0,
                chunk_bytes=0, stream=None):
        import torch

        from hydra_amd import ring

        code = self._code(t, dtype_code)
        n = t.numel()
        if n == 0 or self.world == 1:
            return
        ops, scr = ring.plan_reduce(root, self.world, self.rank, n, t.element_size(), max_segment,
                                    chunk_bytes)
        execute(self.O, ops, scr, t.view(-1).view(torch.uint8), code, op)

    def apipe_allreduce_(self, rail2, t, table=0, algo="auto", op="sum", dtype_code=None,
                         flags=0, max_segment=0, chunk_bytes=0, stream=None):
        """The two rails one after the other (hydra_apipe_allreduce runs them concurrently on
        two communicators; every rank issues them in the same order either way)."""
        from hydra_amd import ring

        e1, _ = ring.split_elements(table, self.world, t.numel())
        flat = t.view(-1)
        kw = dict(algo=algo, op=op, dtype_code=dtype_code, flags=flags,
                  max_segment=max_segment, chunk_bytes=chunk_bytes)
        if e1:
            self.allreduce_(flat[:e1], **kw)
        if e1 < flat.numel():
            rail2.allreduce_(flat[e1:], **kw)

    def info(self):
        """XgmiComm.info's shape (no RCCL here: the process group's own size and rank)."""
        import torch.distributed as dist

        return {"nccl_comm_count": dist.get_world_size(), "nccl_user_rank": dist.get_rank(),
                "nccl_device": -1, "backend": "gloo (test executor)"}

    def wait(self, timeout_ms, stream=None):
        """XgmiComm.wait: the executor is synchronous, so there is never anything pending."""

    def close(self):
        self.closed = True
