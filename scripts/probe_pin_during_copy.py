#!/usr/bin/env python3
"""Probe (attribute queries only; nothing here lets the GPU touch the memory in question): while
one thread runs pageable host->device and device->host copies of a buffer (the HIP runtime's
page-locking copy path locks the caller's pages for the copy), does hipPointerGetAttributes in
another thread ever report that buffer as mapped host memory (type 1 with a device pointer)?

If it does, hydra_reduce_host's lookup of caller-made mappings (host_map.cpp caller_mapping)
could adopt a transient lock the runtime is about to drop -- round 2's advisor finding; if it
never does across many copies of several sizes, the lookup only ever sees mappings the caller
made.  Output: one JSON line per size: polls, hits (type 1 / device pointer seen), copies done.
"""
import ctypes
import json
import threading
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int),
                ("allocationFlags", ctypes.c_uint)]


hip.hipPointerGetAttributes.argtypes = [ctypes.POINTER(Attr), ctypes.c_void_p]
hip.hipGetLastError.restype = ctypes.c_int


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    for nbytes in (1 << 20, 4 << 20, 16 << 20, 64 << 20):
        a = np.ones(nbytes // 4, np.float32)
        d = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
        probes = [a.ctypes.data + off for off in (0, nbytes // 2, nbytes - 4)]
        stop = threading.Event()
        copies = [0]

        def copier():
            t = torch.from_numpy(a)
            while not stop.is_set():
                d.copy_(t)             # pageable H2D
                torch.cuda.synchronize()
                t.copy_(d.cpu())       # pageable D2H (into a fresh pageable tensor, then a)
                copies[0] += 1

        th = threading.Thread(target=copier)
        th.start()
        polls = hits = 0
        first_hit = None
        t0 = time.time()
        while time.time() - t0 < 3.0:
            for p in probes:
                at = Attr()
                rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(p))
                hip.hipGetLastError()
                polls += 1
                if rc == 0 and (at.type == 1 or at.devicePointer):
                    hits += 1
                    if first_hit is None:
                        first_hit = {"type": at.type, "dev": at.devicePointer,
                                     "host": at.hostPointer, "flags": at.allocationFlags}
        stop.set()
        th.join()
        print(json.dumps({"nbytes": nbytes, "polls": polls, "hits": hits, "copies": copies[0],
                          "first_hit": first_hit}), flush=True)


if __name__ == "__main__":
    main()
