#!/usr/bin/env python3
"""Probe: which path does the HIP runtime take for torch's pageable host<->device copies --
through its own pinned staging buffers, or by pinning the caller's pageable memory for the copy
("HSA Copy Using Pinned resource" vs "... Staging resource" in the runtime's debug log)?  Run
with AMD_LOG_LEVEL=4, stderr to a file; each copy is bracketed by a marker line on stderr.
DESIGN.md §10: every late-reported device fault so far surfaced at such a copy.  Nothing here
touches memory it does not own, so it cannot fault."""
import sys

import numpy as np
import torch


def mark(s):
    print(f"=== {s}", file=sys.stderr, flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    for kib in (64, 1024, 2048, 4096, 16384, 65536, 262144):
        a = np.ones(kib * 256, np.float32)
        for rep in range(2):  # the same host buffer twice
            mark(f"h2d {kib} KiB rep {rep} host {a.ctypes.data:#x}")
            t = torch.from_numpy(a).to(dev)
            torch.cuda.synchronize()
        mark(f"d2h {kib} KiB")
        b = t.cpu()
        mark(f"d2h {kib} KiB done host {b.data_ptr():#x}")
        addr = a.ctypes.data
        del a, b
        a2 = np.ones(kib * 256, np.float32)  # often the same address again
        mark(f"h2d {kib} KiB realloc same_addr={a2.ctypes.data == addr}")
        t = torch.from_numpy(a2).to(dev)
        torch.cuda.synchronize()
        del a2, t
    mark("end")


if __name__ == "__main__":
    main()
