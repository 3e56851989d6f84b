#!/usr/bin/env python3
"""probe_rank_faults.py -- the device allreduce's failure detection across real RCCL ranks.

World 2 on the box's one GPU (per-rank NCCL_HOSTID, RCCL over loopback sockets).
  mode "absent": rank 1 never joins the allreduce (the reference's TestTimeout,
      allreduce_test.cc:381-397): rank 0's hydra_comm_wait must return HYDRA_ERR_TIMEOUT
      ("Timed out waiting ...") and abort its communicator.
  mode "dead": rank 1 exits abruptly after the communicators are up (the reference's
      process-kill fault tests): rank 0's wait must end with an error, not hang.
Every step is logged with a timestamp to gpurun_out/<tag>/fault_<mode>_rank<r>.log.

    timeout -k 10 120 python scripts/probe_rank_faults.py TAG MODE
"""
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, out, mode):
    os.environ.update({"NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
                       "NCCL_HOSTID": f"hydra-probe-rank-{rank}", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    log = open(os.path.join(out, f"fault_{mode}_rank{rank}.log"), "w", buffering=1)
    faulthandler.enable(file=log)
    faulthandler.dump_traceback_later(50, repeat=True, file=log)
    t0 = time.time()

    def say(msg):
        log.write(f"{time.time() - t0:8.3f} {msg}\n")

    import torch
    import torch.distributed as dist

    from hydra_amd import _lib, ring

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = ring.XgmiComm(rank, world, 0, ring.exchange_unique_id(rank))
    t = torch.ones(1 << 20, dtype=torch.float32, device=dev)
    comm.allreduce_(t, algo="direct")  # both ranks: one good allreduce first
    comm.wait(30000)
    say(f"warm-up ok, t[0] = {float(t[0])}")
    dist.barrier()
    if rank == 1:
        if mode == "dead":
            say("exiting abruptly")
            os._exit(0)
        say("not joining; waiting for rank 0's verdict")
        dist.barrier()  # rank 0 reports after its wait ended
        say("rank 0 done; closing")
        comm.close()
        say("closed")
    else:
        if mode == "dead":
            time.sleep(2.0)  # rank 1 is gone by now
        comm.allreduce_(t, algo="direct")
        t1 = time.time()
        try:
            comm.wait(3000)
            say("wait returned OK (unexpected)")
        except _lib.HydraError as e:
            say(f"wait raised after {time.time() - t1:.2f} s: code {e.code}: {e}")
        if mode == "absent":
            dist.barrier()
        comm.close()
        say("closed")
    say("done")
    faulthandler.cancel_dump_traceback_later()
    if mode == "absent":
        dist.destroy_process_group()
    os._exit(0)


def main():
    import torch.multiprocessing as mp

    tag, mode = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "gpurun_out", tag)
    os.makedirs(out, exist_ok=True)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=worker, args=(r, 2, port, out, mode)) for r in range(2)]
    for p in procs:
        p.start()
    deadline = time.time() + 90
    for p in procs:
        p.join(timeout=max(1, deadline - time.time()))
    rc = 0
    for p in procs:
        if p.is_alive():
            p.kill()
            rc = 3
    for r in range(2):
        print(open(os.path.join(out, f"fault_{mode}_rank{r}.log")).read()[-3000:])
    print("exit codes:", [p.exitcode for p in procs])
    sys.exit(rc)


if __name__ == "__main__":
    main()
