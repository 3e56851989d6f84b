#!/usr/bin/env python3
"""Long stress of the peer-access allreduce on one GPU (P processes by IPC): thousands of calls
with changing integer-valued inputs, random per-rank arrival delays and every word checked
(tests/peer_worker.py's `stress` case), for rare ordering / visibility failures that the test
suite's 40-call version could miss.  Not part of the test suite.

Usage: python scripts/peer_stress.py [--P 4] [--iters 2000] [--n 262147] [--blocks 64]
Prints one JSON line: wrong words per rank per algorithm (all zeros = pass).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "peer_worker.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=4)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--n", type=int, default=262147)
    ap.add_argument("--blocks", type=int, default=64)
    a = ap.parse_args()
    cases = [dict(name=f"stress_{algo}", algo=algo, data="stress", dtype=6, n=a.n,
                  iters=a.iters, offset_bytes=4) for algo in ("peer2", "peer1")]
    with tempfile.TemporaryDirectory() as d:
        cpath = os.path.join(d, "cases.json")
        with open(cpath, "w") as f:
            json.dump(cases, f)
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        procs = [subprocess.Popen([sys.executable, "-u", WORKER, "--rank", str(r), "--world",
                                   str(a.P), "--port", str(port), "--out", d, "--cases", cpath,
                                   "--blocks", str(a.blocks)],
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                 for r in range(a.P)]
        outs = [p.communicate(timeout=1200)[0].decode(errors="replace") for p in procs]
        rcs = [p.returncode for p in procs]
        status = []
        for r in range(a.P):
            try:
                with open(os.path.join(d, f"status{r}.json")) as f:
                    status.append(json.load(f))
            except OSError:
                status.append(None)
    print(json.dumps({"P": a.P, "iters": a.iters, "n": a.n, "rc": rcs, "wrong_words": status}))
    if any(rcs):
        for o in outs:
            print(o[-2000:], file=sys.stderr)
        raise SystemExit(1)


if __name__ == "__main__":
    main()
