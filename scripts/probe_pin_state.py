#!/usr/bin/env python3
"""Probe (no GPU access to the memory in question, so nothing here can fault): does the HIP
runtime still consider a host range pinned/registered after the registration that pinned it is
gone -- after hipHostUnregister, after a pageable copy the runtime may pin on the fly, and after
the host memory is freed and the same address handed out again?  DESIGN.md §10 (r02h2): every
late-reported device fault so far surfaced at a torch pageable copy; a stale pinning picked up
at a reused host address is one explanation that these attribute queries can confirm or rule
out without provoking a fault.

Output: one JSON line per case with hipPointerGetAttributes' view (type 0 = unregistered,
1 = host, 2 = device) of each address at each step."""
import ctypes
import json
import mmap

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int),
                ("allocationFlags", ctypes.c_uint)]


hip.hipPointerGetAttributes.argtypes = [ctypes.POINTER(Attr), ctypes.c_void_p]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipGetLastError.restype = ctypes.c_int


def view(p):
    a = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
    hip.hipGetLastError()
    return {"rc": rc, "type": a.type, "dev": a.devicePointer, "host": a.hostPointer}


def out(case, **kw):
    print(json.dumps({"case": case, **kw}), flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()

    # A: the runtime's own handling of pageable copies (H2D and D2H), 2 MiB and 64 MiB
    for nbytes in (2 << 20, 64 << 20):
        a = np.ones(nbytes // 4, np.float32)
        pa = a.ctypes.data
        before = view(pa)
        t = torch.from_numpy(a).to(dev)
        torch.cuda.synchronize()
        after_h2d = view(pa)
        back = t.cpu()
        pb = back.data_ptr()
        after_d2h = view(pb)
        del a
        a2 = np.ones(nbytes // 4, np.float32)  # often the same address again
        out("runtime_pageable_copy", nbytes=nbytes, before=before, after_h2d=after_h2d,
            d2h_dst_after=after_d2h, realloc_same_addr=a2.ctypes.data == pa,
            realloc_view=view(a2.ctypes.data))
        del back, t, a2

    # B: sub-page ranges in one page (two operands of one hydra_reduce_host call), then the
    #    exact whole range; each registered, viewed, unregistered, viewed
    buf = np.zeros(1 << 20, np.uint8)
    p = buf.ctypes.data
    for phase in ({"sub_a": (100, 300), "sub_b": (500, 900)}, {"exact": (0, 1 << 20)}):
        steps = {}
        for name, (off, n) in phase.items():
            steps[name + "_reg_rc"] = hip.hipHostRegister(ctypes.c_void_p(p + off), n, 0)
            hip.hipGetLastError()
        steps["during"] = {k: view(p + o) for k, (o, _) in phase.items()}
        steps["page_start_during"] = view(p)
        for name, (off, _) in phase.items():
            steps[name + "_unreg_rc"] = hip.hipHostUnregister(ctypes.c_void_p(p + off))
            hip.hipGetLastError()
        steps["after"] = {k: view(p + o) for k, (o, _) in phase.items()}
        out("register_unregister", **steps)

    # C: a registered mmap range unregistered, unmapped, and mapped again at the same address
    m = mmap.mmap(-1, 4 << 20)
    arr = np.frombuffer(m, np.uint8)
    pm = arr.ctypes.data
    r1 = hip.hipHostRegister(ctypes.c_void_p(pm), 4 << 20, 0)
    hip.hipGetLastError()
    during = view(pm)
    u1 = hip.hipHostUnregister(ctypes.c_void_p(pm))
    hip.hipGetLastError()
    del arr
    m.close()
    m2 = mmap.mmap(-1, 4 << 20)
    arr2 = np.frombuffer(m2, np.uint8)
    out("unmap_remap", reg_rc=r1, unreg_rc=u1, during=during,
        same_addr=arr2.ctypes.data == pm, remapped_view=view(arr2.ctypes.data))
    del arr2
    m2.close()


if __name__ == "__main__":
    main()
