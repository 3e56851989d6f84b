#!/usr/bin/env python3
"""oracle/gen_golden.py -- TEST INFRASTRUCTURE ONLY.

Regenerates tests/golden/* from the REFERENCE ITSELF (oracle/_ref/libgloo_ref.so, built from
/root/reference/gloo by oracle/Makefile).  Run in the survey/build container, where
/root/reference exists:

    make -C oracle all && python3 oracle/gen_golden.py

Fixtures are data only (inputs + the reference's outputs); inputs for the ring cases come from
hydra_amd.synth (deterministic integer hashing), so only their sha256 is stored next to the
reference outputs.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[0] = ROOT  # run as a script from oracle/: import the package, not oracle.py

from hydra_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")

REF_TYPES = {  # name -> (numpy dtype, hydra dtype code)
    "i8": (np.int8, 0), "u8": (np.uint8, 1), "i32": (np.int32, 2), "u32": (np.uint32, 3),
    "i64": (np.int64, 4), "u64": (np.uint64, 5), "f32": (np.float32, 6), "f64": (np.float64, 7),
    "f16": (np.uint16, 8),
}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def operands(name: str, n: int, rng: np.random.Generator):
    dt, _ = REF_TYPES[name]
    if name in ("f32", "f64"):
        a = rng.uniform(-1e3, 1e3, n).astype(dt)
        b = rng.uniform(-1e3, 1e3, n).astype(dt)
        specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45 if dt == np.float32
                             else 5e-324, -1e-40, 3.4e38, -3.4e38, 1.0, 2.0 ** -24], dtype=dt)
        k = len(specials)
        a[:k * k] = np.repeat(specials, k)
        b[:k * k] = np.tile(specials, k)
    elif name == "f16":
        vals = rng.uniform(-70000, 70000, n).astype(np.float32)
        a = np.array([O.f2h(float(v)) for v in vals], dtype=np.uint16)
        vals = rng.uniform(-1000, 1000, n).astype(np.float32)
        b = np.array([O.f2h(float(v)) for v in vals], dtype=np.uint16)
        specials = np.array([0x0000, 0x8000, 0x7C00, 0xFC00, 0x7E00, 0x0001, 0x8001, 0x7BFF,
                             0xFBFF, 0x3C00, 0x03FF, 0x7D00], dtype=np.uint16)
        k = len(specials)
        a[:k * k] = np.repeat(specials, k)
        b[:k * k] = np.tile(specials, k)
    else:
        info = np.iinfo(dt)
        lo, hi = (max(info.min, -(1 << 20)), min(info.max, 1 << 20)) if info.bits > 16 else \
            (info.min, info.max)
        a = rng.integers(lo, hi, n, dtype=np.int64, endpoint=True).astype(dt)
        b = rng.integers(lo, hi, n, dtype=np.int64, endpoint=True).astype(dt)
        if info.bits <= 8:  # exercise the reference's narrowing wrap on 8-bit types
            a[:4] = [info.max, info.min, info.max, info.min]
            b[:4] = [1, -1 if info.min < 0 else 0, info.max, info.min]
    return a, b


def gen_ops(out: dict, meta: dict) -> None:
    rng = np.random.default_rng(20240212)
    n = 1000
    for name, (dt, code) in REF_TYPES.items():
        a, b = operands(name, n, rng)
        out[f"ops_{name}_a"] = a
        out[f"ops_{name}_b"] = b
        for kind in ("sum", "product", "max", "min"):
            if kind == "product" and name == "i32":
                # signed overflow is UB in the reference: keep |a*b| < 2^31 for int32
                pa, pb = (a % 40000).astype(dt), (b % 40000).astype(dt)
                out[f"ops_{name}_pa"], out[f"ops_{name}_pb"] = pa, pb
                out[f"ops_{name}_{kind}"] = O.op(pa, pb, kind, code, lib="ref")
                continue
            c = O.op(a, b, kind, code, lib="ref")
            out[f"ops_{name}_{kind}"] = c
    meta["ops_n"] = n


RING_CASES = [(P, n, ms) for P in (1, 2, 3, 4, 5, 7, 8) for n in (1, 7, 100, 1000, 4099)
              for ms in (128, 1 << 20)]
RING_BIG = [(2, 262145, 1 << 20), (3, 262145, 1 << 20), (8, 262145, 1 << 20),
            (4, 1048577, 1 << 20), (8, 1048576 + 12345, 1 << 20), (5, 3000001, 1 << 20)]


def gen_ring(out: dict, meta: dict) -> None:
    rows = []
    for (P, n, ms) in RING_CASES + RING_BIG:
        xs = [synth.stress_f32(P, r, n) for r in range(P)]
        outs = [[x.copy()] for x in xs]
        O.ref_allreduce(P, outs, None, max_segment=ms)
        res = outs[0][0]
        for r in range(1, P):
            assert np.array_equal(outs[r][0].view(np.uint32), res.view(np.uint32))
        key = f"ring_f32_P{P}_n{n}_ms{ms}"
        row = {"P": P, "n": n, "max_segment": ms, "inputs_sha256": sha(np.stack(xs)),
               "output_sha256": sha(res), "key": key}
        if n <= 4099:
            out[key] = res
        else:
            out[key + "_head"] = res[:1024]
            out[key + "_tail"] = res[-1024:]
        rows.append(row)
    # int32 stress (wraps never happen: |x| < 2^20, P <= 8)
    for (P, n) in [(2, 1000), (3, 1000), (8, 1000), (7, 4099)]:
        xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        outs = [[x.copy()] for x in xs]
        O.ref_allreduce(P, outs, None, max_segment=128)
        key = f"ring_i32_P{P}_n{n}"
        out[key] = outs[0][0]
        rows.append({"P": P, "n": n, "max_segment": 128, "key": key,
                     "inputs_sha256": sha(np.stack(xs)), "output_sha256": sha(outs[0][0])})
    meta["ring"] = rows


def gen_bcube(out: dict, meta: dict) -> None:
    """gloo::allreduce BCUBE (allreduce.cc:423-700): power-of-two and factor-3/5/7 group sizes,
    fp32 stress inputs (regenerated from synth, sha-pinned), int32, and f16 (stored inputs);
    multi-pointer in/out-of-place on a few cases."""
    rows = []
    rng = np.random.default_rng(79)
    for P in (1, 2, 3, 4, 6, 8, 12):
        for n in (1, 7, 100, 1000, 4099, 100003):
            xs = [synth.stress_f32(P, r, n) for r in range(P)]
            outs = [[x.copy()] for x in xs]
            O.ref_allreduce(P, outs, None, algorithm=2)
            res = outs[0][0]
            for r in range(1, P):
                assert np.array_equal(outs[r][0].view(np.uint32), res.view(np.uint32))
            key = f"bcube_f32_P{P}_n{n}"
            row = {"P": P, "n": n, "dtype": 6, "key": key, "inputs_sha256": sha(np.stack(xs)),
                   "output_sha256": sha(res)}
            if n <= 4099:
                out[key] = res
            else:
                out[key + "_head"] = res[:1024]
                out[key + "_tail"] = res[-1024:]
            rows.append(row)
    for P, n in ((2, 1000), (6, 4099), (8, 1000)):
        xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        outs = [[x.copy()] for x in xs]
        O.ref_allreduce(P, outs, None, algorithm=2)
        key = f"bcube_i32_P{P}_n{n}"
        out[key] = outs[0][0]
        rows.append({"P": P, "n": n, "dtype": 2, "key": key, "inputs_sha256": sha(np.stack(xs)),
                     "output_sha256": sha(outs[0][0])})
    for P, n in ((2, 1000), (3, 4099), (8, 1000)):
        xs = [np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)], np.uint16)
              for _ in range(P)]
        outs = [[x.copy()] for x in xs]
        O.ref_allreduce(P, outs, None, dtype_code=8, algorithm=2)
        key = f"bcube_f16_P{P}_n{n}"
        out[key + "_in"] = np.stack(xs)
        out[key] = outs[0][0]
        rows.append({"P": P, "n": n, "dtype": 8, "key": key, "stored_inputs": True})
    meta["bcube"] = rows


def gen_old_ring(out: dict, meta: dict) -> None:
    """Old-style AllreduceRing<T> (allreduce_ring.h:20-125): per-rank outputs (they differ)."""
    rows = []
    rng = np.random.default_rng(77)
    for name, code in (("f32", 6), ("i32", 2), ("f16", 8)):
        for P in (1, 2, 3, 5, 8):
            for n in (1, 100, 4099):
                for nptr in (1, 2):
                    if name == "f32":
                        bufs = [[synth.stress_f32(P, r, n, seed=500 + i) for i in range(nptr)]
                                for r in range(P)]
                    elif name == "i32":
                        bufs = [[synth.int32_bucket(P, r, n, seed=500 + i) for i in range(nptr)]
                                for r in range(P)]
                    else:
                        bufs = [[np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)],
                                          np.uint16) for _ in range(nptr)] for _ in range(P)]
                    key = f"oldring_{name}_P{P}_n{n}_k{nptr}"
                    out[key + "_in"] = np.stack([np.stack(b) for b in bufs])
                    O.ref_allreduce_ring_old(bufs, dtype_code=code)
                    out[key + "_out"] = np.stack([np.stack(b) for b in bufs])
                    rows.append({"key": key, "P": P, "n": n, "nptr": nptr, "dtype": code})
    meta["old_ring"] = rows


def gen_chunked_ring(out: dict, meta: dict) -> None:
    """AllreduceRingChunked<T> (allreduce_ring_chunked.h:20-248): 2P chunks of
    max(256, ceil(n/2P)); sizes cover one chunk, partial and empty trailing chunks."""
    rows = []
    rng = np.random.default_rng(78)
    for name, code in (("f32", 6), ("i32", 2), ("f16", 8)):
        for P in (1, 2, 3, 5, 8):
            for n in (1, 100, 1000, 4099):
                for nptr in (1, 2):
                    if name == "f32":
                        bufs = [[synth.stress_f32(P, r, n, seed=600 + i) for i in range(nptr)]
                                for r in range(P)]
                    elif name == "i32":
                        bufs = [[synth.int32_bucket(P, r, n, seed=600 + i) for i in range(nptr)]
                                for r in range(P)]
                    else:
                        bufs = [[np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)],
                                          np.uint16) for _ in range(nptr)] for _ in range(P)]
                    key = f"chunkring_{name}_P{P}_n{n}_k{nptr}"
                    out[key + "_in"] = np.stack([np.stack(b) for b in bufs])
                    O.ref_allreduce_ring_chunked(bufs, dtype_code=code)
                    res = np.stack([np.stack(b) for b in bufs])
                    assert all(np.array_equal(res[0].view(np.uint8), res[r].view(np.uint8))
                               for r in range(P)), key  # every rank holds the same bits
                    out[key + "_out"] = res[0, 0]
                    rows.append({"key": key, "P": P, "n": n, "nptr": nptr, "dtype": code})
    meta["chunked_ring"] = rows


def gen_halving_doubling(out: dict, meta: dict) -> None:
    """AllreduceHalvingDoubling<T> (allreduce_halving_doubling.h:37-358): P covers one binary
    block (1, 2, 4, 8), two (3, 5, 6, 12) and three (7, 11); n covers fewer elements than
    chunks, ragged last chunks and empty steps."""
    rows = []
    rng = np.random.default_rng(79)
    for name, code in (("f32", 6), ("i32", 2), ("f16", 8)):
        for P in (1, 2, 3, 4, 5, 6, 7, 8, 11, 12):
            for n in ((1, 7, 100, 1001, 4099) if P in (3, 7, 8) else (1, 7, 100, 1001)):
                for nptr in ((1, 2) if n <= 100 else (1,)):
                    if name == "f32":
                        bufs = [[synth.stress_f32(P, r, n, seed=700 + i) for i in range(nptr)]
                                for r in range(P)]
                    elif name == "i32":
                        bufs = [[synth.int32_bucket(P, r, n, seed=700 + i) for i in range(nptr)]
                                for r in range(P)]
                    else:
                        bufs = [[np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)],
                                          np.uint16) for _ in range(nptr)] for _ in range(P)]
                    key = f"hd_{name}_P{P}_n{n}_k{nptr}"
                    out[key + "_in"] = np.stack([np.stack(b) for b in bufs])
                    O.ref_allreduce_halving_doubling(bufs, dtype_code=code)
                    res = np.stack([np.stack(b) for b in bufs])
                    assert all(np.array_equal(res[0].view(np.uint8), res[r].view(np.uint8))
                               for r in range(P)), key  # every rank holds the same bits
                    out[key + "_out"] = res[0, 0]
                    rows.append({"key": key, "P": P, "n": n, "nptr": nptr, "dtype": code})
    meta["halving_doubling"] = rows


def gen_bcube_old(out: dict, meta: dict) -> None:
    """Old-style AllreduceBcube<T> (allreduce_bcube.h:255-691, context base 2): P a power of
    two (for other P its ranks disagree, see tests/test_oracle.py), 1-2 pointers."""
    rows = []
    rng = np.random.default_rng(80)
    for name, code in (("f32", 6), ("i32", 2), ("f16", 8)):
        for P in (1, 2, 4, 8):
            for n in (1, 7, 100, 1001):
                for nptr in (1, 2):
                    if name == "f32":
                        bufs = [[synth.stress_f32(P, r, n, seed=800 + i) for i in range(nptr)]
                                for r in range(P)]
                    elif name == "i32":
                        bufs = [[synth.int32_bucket(P, r, n, seed=800 + i) for i in range(nptr)]
                                for r in range(P)]
                    else:
                        bufs = [[np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)],
                                          np.uint16) for _ in range(nptr)] for _ in range(P)]
                    key = f"bcube_old_{name}_P{P}_n{n}_k{nptr}"
                    out[key + "_in"] = np.stack([np.stack(b) for b in bufs])
                    O.ref_allreduce_bcube_old(bufs, dtype_code=code)
                    res = np.stack([np.stack(b) for b in bufs])
                    assert all(np.array_equal(res[0].view(np.uint8), res[r].view(np.uint8))
                               for r in range(P)), key
                    out[key + "_out"] = res[0, 0]
                    rows.append({"key": key, "P": P, "n": n, "nptr": nptr, "dtype": code})
    meta["bcube_old"] = rows


def main_algo() -> None:
    """Fixtures added after golden.npz was frozen go to their own file (golden_algo.*)."""
    out: dict = {}
    meta: dict = {"generator": "oracle/gen_golden.py --algo",
                  "reference": "hydra-ppopp2024/hydra snapshot 2025-02-12, gloo core built by "
                               "oracle/Makefile (g++ -O3 -DNDEBUG)"}
    gen_halving_doubling(out, meta)
    gen_bcube_old(out, meta)
    np.savez_compressed(os.path.join(GOLD, "golden_algo.npz"), **out)
    with open(os.path.join(GOLD, "golden_algo.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"wrote {len(out)} arrays to golden_algo.npz")


# Every band edge of the two split tables (pipeallreduce-a.h:137-376), as written there.
SPLIT_EDGES = (6144, 6145, 65536, 65537, 114975, 131072, 262144, 262145, 524287, 524288, 524289,
               828343, 828344, 1048576, 1048577, 2097152, 2097153, 4194304, 4194305, 8388608,
               8388609, 16777216, 16777217, 33554432, 33554433, 67108864, 67108865)


def split_cases() -> list:
    ns = set(range(0, 130)) | {1000, 1500000, 1500001, 200003, 1 << 28, (1 << 28) + 77}
    for e in SPLIT_EDGES:
        ns |= {e + d for d in range(-3, 4)}
    rng = np.random.default_rng(2024)
    ns |= {int(v) for v in rng.integers(1, 1 << 27, 400)}
    return sorted(ns)


def main_split() -> None:
    """The two-rail split from the reference's own compiled methods
    (oracle/split_ref.py -> _ref/libsplit_ref.so): (table, P, n) -> (e1, e2) for both tables,
    P = 1..9, every band edge +-3, the first 130 n and 400 random n < 2^27."""
    from oracle import split_ref

    lib = split_ref.load(split_ref.build())
    rows = []
    for table in (0, 1):
        for P in range(1, 10):
            for n in split_cases():
                e1, e2 = split_ref.ref_split(lib, table, P, n)
                rows.append([table, P, n, e1, e2])
    meta = {"generator": "oracle/gen_golden.py --split",
            "reference": "APipeAllreduceOptions::calculateElements_AA / _AG "
                         "(gloo/gloo/pipeallreduce-a.h:137-376), compiled by oracle/split_ref.py "
                         "(g++ -O3 -DNDEBUG)",
            "columns": ["table (0 = AA, 1 = AG)", "P", "n", "e1", "e2"], "rows": rows}
    with open(os.path.join(GOLD, "golden_split.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))
    print(f"wrote {len(rows)} split rows to golden_split.json")


# Config 5's arithmetic (bf16 bucket, fp32 accumulation, one rounding) on the reference: its own
# ring over the bf16 values widened exactly to fp32 is the fp32 fold in the reference order; one
# round-to-nearest-even to bf16 gives what k_fold<bf16, ACC32> must produce.  n is a multiple of
# 2P below P x 512 Ki, so the fp32 and the bf16 geometries cut identical element blocks.
BF16_CASES = [(P, 2 * P * k) for P in (2, 3, 4, 8) for k in (7, 20001)]


def main_bf16() -> None:
    if not O.ref_available():
        raise SystemExit("oracle/_ref/libgloo_ref.so missing: make -C oracle ref")
    out: dict = {}
    rows = []
    for P, n in BF16_CASES:
        ns4, sb4, S4 = O.ring_plan(P, n, 4)
        ns2, sb2, S2 = O.ring_plan(P, n, 2)
        assert (ns4, sb4 // 4, S4) == (ns2, sb2 // 2, S2), (P, n)  # same element blocks
        xb = [synth.bf16_bits(synth.stress_f32(P, r, n)) for r in range(P)]
        outs = [[synth.bf16_to_f32(x).copy()] for x in xb]
        O.ref_allreduce(P, outs)
        for r in range(1, P):
            assert np.array_equal(outs[r][0].view(np.uint32), outs[0][0].view(np.uint32))
        key = f"bf16acc32_P{P}_n{n}"
        out[key] = synth.bf16_bits(outs[0][0])
        rows.append({"key": key, "P": P, "n": n, "inputs_sha256": sha(np.stack(xb))})
    np.savez_compressed(os.path.join(GOLD, "golden_bf16.npz"), **out)
    with open(os.path.join(GOLD, "golden_bf16.json"), "w") as f:
        json.dump({"generator": "oracle/gen_golden.py --bf16",
                   "what": "bf16 inputs synth.bf16_bits(synth.stress_f32(P, r, n)); the "
                           "reference's gloo::allreduce RING (maxSegmentSize 1 MiB) on their "
                           "exact fp32 widening; output = RNE of its fp32 result to bf16",
                   "cases": rows}, f, indent=1)
    print(f"wrote {len(out)} bf16 cases to golden_bf16.npz")


def gen_new_test(meta: dict) -> None:
    """AllreduceNewTest.Default (test/allreduce_test.cc:302-362): confirm the reference meets the
    closed form k*stride^2 + stride(stride-1)/2 for uint64, every combination we test."""
    checked = 0
    for P in (1, 2, 4, 7):
        for nptr in (1, 2, 3):
            for n in (1, 10, 100, 1000):
                for inplace in (True, False):
                    stride = P * nptr
                    vals = [[(np.arange(n, dtype=np.uint64) * stride + r * nptr + i)
                             for i in range(nptr)] for r in range(P)]
                    if inplace:
                        outs = [[v.copy() for v in vr] for vr in vals]
                        ins = None
                    else:
                        outs = [[np.zeros(n, np.uint64) for _ in range(nptr)] for _ in range(P)]
                        ins = vals
                    O.ref_allreduce(P, outs, ins, max_segment=128)
                    exp = (np.arange(n, dtype=np.uint64) * stride * stride
                           + np.uint64(stride * (stride - 1) // 2))
                    for r in range(P):
                        for i in range(nptr):
                            assert np.array_equal(outs[r][i], exp), (P, nptr, n, inplace)
                    checked += 1
    meta["allreduce_new_test_closed_form_cases"] = checked


REDUCE_CASES = [(P, n, ms) for P in (1, 2, 3, 4, 7) for n in (1, 10, 100, 1000, 4099)
                for ms in (128, 1 << 20)]


def gen_reduce(out: dict, meta: dict) -> None:
    """gloo::reduce (reduce.cc:21-262) to a root: fp32 stress inputs, in place and out of
    place (outputs start zeroed, as ReduceTest clears them: reduce_test.cc:50-56).  Every
    rank's output is stored for n <= 1000 (non-root outputs are whatever the reference's
    schedule leaves there); the root's only for n = 4099.  Plus int32 and in-place float16."""
    rows = []
    for (P, n, ms) in REDUCE_CASES:
        for inplace in (True, False):
            root = (n + P) % P  # varies with the case
            xs = [synth.stress_f32(P, r, n) for r in range(P)]
            if inplace:
                outs, ins = [x.copy() for x in xs], None
            else:
                outs, ins = [np.zeros(n, np.float32) for _ in xs], [x.copy() for x in xs]
            O.ref_reduce(outs, ins, root, max_segment=ms)
            key = f"reduce_f32_P{P}_n{n}_ms{ms}_{'in' if inplace else 'out'}"
            if n <= 1000:
                out[key] = np.stack(outs)
            else:
                out[key + "_root"] = outs[root]
            rows.append({"P": P, "n": n, "max_segment": ms, "inplace": inplace, "root": root,
                         "key": key, "inputs_sha256": sha(np.stack(xs)),
                         "root_sha256": sha(outs[root])})
    for (P, n, dt, code) in [(3, 1000, np.int32, 2), (4, 4099, np.int32, 2),
                             (3, 1000, np.uint16, 8), (7, 999, np.uint16, 8)]:
        if code == 2:
            xs = [synth.int32_bucket(P, r, n) for r in range(P)]
        else:
            rng = np.random.default_rng(P * 1000 + n)
            xs = [np.array([O.f2h(float(v)) for v in rng.uniform(-8, 8, n)], np.uint16)
                  for _ in range(P)]
        outs = [x.copy() for x in xs]
        root = 1
        O.ref_reduce(outs, None, root, dtype_code=code, max_segment=128)
        key = f"reduce_{'i32' if code == 2 else 'f16'}_P{P}_n{n}_in"
        out[key + "_inputs"] = np.stack(xs)
        out[key] = np.stack(outs)
        rows.append({"P": P, "n": n, "max_segment": 128, "inplace": True, "root": root,
                     "dtype": code, "key": key})
    meta["reduce"] = rows
    # ReduceTest.Default's closed form (reduce_test.cc:22-86) on the reference, uint64
    checked = 0
    for P in (1, 2, 4, 7):
        for n in (1, 10, 100, 1000):
            for inplace in (True, False):
                for root in range(P):
                    vals = [np.arange(n, dtype=np.uint64) * P + r for r in range(P)]
                    if inplace:
                        outs, ins = [v.copy() for v in vals], None
                    else:
                        outs, ins = [np.zeros(n, np.uint64) for _ in range(P)], vals
                    O.ref_reduce(outs, ins, root, max_segment=128)
                    exp = np.arange(n, dtype=np.uint64) * P * P + np.uint64(P * (P - 1) // 2)
                    assert np.array_equal(outs[root], exp), (P, n, inplace, root)
                    checked += 1
    meta["reduce_test_closed_form_cases"] = checked
    meta["reduce_timeout_probe"] = O.ref_reduce_timeout(10)


def main() -> None:
    if not O.ref_available():
        raise SystemExit("oracle/_ref/libgloo_ref.so missing: make -C oracle ref")
    os.makedirs(GOLD, exist_ok=True)
    out: dict = {}
    meta: dict = {"generator": "oracle/gen_golden.py",
                  "reference": "hydra-ppopp2024/hydra snapshot 2025-02-12, gloo core built by "
                               "oracle/Makefile (g++ -O3 -DNDEBUG)"}
    gen_ops(out, meta)
    gen_ring(out, meta)
    gen_old_ring(out, meta)
    gen_bcube(out, meta)
    gen_chunked_ring(out, meta)
    gen_new_test(meta)
    gen_reduce(out, meta)
    import ctypes
    buf = ctypes.create_string_buffer(512)
    rc = O.ref().ref_allreduce_timeout(10, buf, 512)
    meta["timeout_probe"] = {"rc": rc, "what": buf.value.decode()}
    np.savez_compressed(os.path.join(GOLD, "golden.npz"), **out)
    with open(os.path.join(GOLD, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    sz = os.path.getsize(os.path.join(GOLD, "golden.npz"))
    print(f"wrote {len(out)} arrays ({sz/1e6:.2f} MB) + golden.json")


if __name__ == "__main__":
    if "--split" in sys.argv[1:]:  # needs only /root/reference's pipeallreduce-a.h and g++
        main_split()
        raise SystemExit(0)
    if "--bf16" in sys.argv[1:]:
        main_bf16()
        raise SystemExit(0)
    if not O.ref_available():
        raise SystemExit("oracle/_ref/libgloo_ref.so missing: make -C oracle ref")
    main_algo() if "--algo" in sys.argv[1:] else main()
