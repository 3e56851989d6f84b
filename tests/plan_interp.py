"""numpy interpreter of the device allreduce plans (test infrastructure): lock-step execution of
every rank's op list with p2p groups matched per (src, dst) FIFO, the fold order of the HIP
kernels restated with the oracle's element ops."""
import numpy as np

from hydra_amd import ring

SEND, RECV, GROUP, REDUCE, FOLD, ALLTOALL, ALLGATHER = 1, 2, 3, 4, 5, 6, 7


def fold_slot(o, j):
    """xgmi_plan.h fold_slot: scratch offset of contribution j of a FOLD."""
    if o["peer"] < 0:
        return o["src_off"] + (j - 1) * o["slot_stride"]
    return o["src_off"] + ((o["peer"] + j) % o["nsrc"]) * o["slot_stride"]


def interpret(plans, bufs, scratch, reduce_fn):
    """Sequential lock-step execution of all ranks (p2p groups matched per (src,dst) FIFO)."""
    P = len(plans)
    pcs = [0] * P
    sends, recvs = {}, {}
    posted = [None] * P
    coll_wait = [False] * P
    while any(pcs[r] < len(plans[r]) for r in range(P)):
        progress = False
        for r in range(P):
            ops = plans[r]
            while pcs[r] < len(ops):
                o = ops[pcs[r]]
                if o["kind"] in (ALLTOALL, ALLGATHER):
                    coll_wait[r] = True
                    if all(coll_wait[q] and plans[q][pcs[q]]["kind"] == o["kind"]
                           for q in range(P)):
                        B, off = o["bytes"], o["off"]
                        for sr in range(P):
                            for dr in range(P):
                                if o["kind"] == ALLTOALL:
                                    d0 = o["src_off"] + sr * B
                                    scratch[dr][d0:d0 + B] = bufs[sr][off + dr * B:off + dr * B + B]
                                elif sr != dr:
                                    bufs[dr][off + sr * B:off + sr * B + B] = \
                                        bufs[sr][off + sr * B:off + sr * B + B]
                        for q in range(P):
                            coll_wait[q] = False
                            pcs[q] += 1
                        progress = True
                        continue
                    break
                if o["kind"] in (REDUCE, FOLD):
                    reduce_fn(r, o)
                    pcs[r] += 1
                    progress = True
                    continue
                if posted[r] is None:
                    g = pcs[r]
                    while ops[g]["kind"] != GROUP:
                        g += 1
                    items = ops[pcs[r]:g]
                    posted[r] = [g, len(items)]
                    for it in items:
                        key = (r, it["peer"]) if it["kind"] == SEND else (it["peer"], r)
                        (sends if it["kind"] == SEND else recvs).setdefault(key, []).append((r, it))
                    progress = True
                    for key in list(sends):
                        sq, rq = sends[key], recvs.setdefault(key, [])
                        while sq and rq:
                            (sr, so), (dr, ro) = sq.pop(0), rq.pop(0)
                            assert so["bytes"] == ro["bytes"]
                            src = (bufs if so["buf"] == 0 else scratch)[sr]
                            dst = (bufs if ro["buf"] == 0 else scratch)[dr]
                            dst[ro["off"]:ro["off"] + ro["bytes"]] = \
                                src[so["off"]:so["off"] + so["bytes"]]
                            posted[sr][1] -= 1
                            posted[dr][1] -= 1
                if posted[r][1] == 0:
                    pcs[r] = posted[r][0] + 1
                    posted[r] = None
                    progress = True
                    continue
                break
        assert progress, "deadlock"


def run_plan_numpy(O, algo, xs, max_segment, chunk, code=6, plans=None, scr=0):
    """Execute the library's plans for len(xs) ranks (or the given `plans`) in numpy."""
    P = len(xs)
    es = xs[0].itemsize
    n = xs[0].size
    if plans is None:
        plans, scr = [], 0
        for r in range(P):
            ops, s = ring.plan(algo, P, r, n, es, max_segment, chunk)
            plans.append(ops)
            scr = max(scr, s)
    bufs = [x.copy().view(np.uint8) for x in xs]
    scratch = [np.zeros(scr + 16, np.uint8) for _ in range(P)]
    dt = xs[0].dtype

    def reduce_fn(r, o):
        u, sc = bufs[r], scratch[r]
        cnt = o["bytes"] // es
        local = u[o["off"]:o["off"] + o["bytes"]].view(dt).copy()
        if o["kind"] == REDUCE:
            recv = sc[o["src_off"]:o["src_off"] + o["bytes"]].view(dt)
            out = O.op(local, recv, "sum", code)
        else:
            slots = [sc[fold_slot(o, j):fold_slot(o, j) + o["bytes"]].view(dt)
                     for j in range(1, o["nsrc"])]
            acc = slots[-1].copy()
            for s in reversed(slots[:-1]):
                acc = O.op(s.copy(), acc, "sum", code)
            out = O.op(local, acc, "sum", code)
        assert out.size == cnt
        u[o["off"]:o["off"] + o["bytes"]] = out.view(np.uint8)

    interpret(plans, bufs, scratch, reduce_fn)
    return [b.view(dt) for b in bufs]
