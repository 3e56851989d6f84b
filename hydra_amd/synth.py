"""Deterministic synthetic buckets (no RNG-version dependence: pure integer hashing).

Patterns follow the reference's benchmark initialisers so sizes/values mean the same thing:
  * ``new_inputs``  -- NewAllreduceBenchmark::initialize, gloo/gloo/benchmark/main.cc:329-337
                       in[j] = j*(P*inputs) + rank*inputs + i
  * ``bew_inputs``  -- aAllreduceBenchmark::initialize,   gloo/gloo/benchmark/main.cc:643-649
                       in[i] = i*(rank+1.0)
  * ``stress_f32``  -- ordering stress: uniform[-1,1) * 2^(3r mod 17), so that a wrong fold
                       order changes low-order bits (SURVEY.md §8(d) item iii)
  * ``uniform_f32`` -- microbench operand b, uniform[-1,1)
"""
from __future__ import annotations

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix(idx: np.ndarray, seed: int) -> np.ndarray:
    """splitmix64 finaliser of (idx + seed*golden) -> uint64, vectorised."""
    with np.errstate(over="ignore"):
        z = idx.astype(np.uint64) + np.uint64((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform_f32(n: int, seed: int) -> np.ndarray:
    """uniform [-1, 1) fp32 with 24 random mantissa bits."""
    bits = _splitmix(np.arange(n, dtype=np.uint64), seed) >> np.uint64(40)
    return (bits.astype(np.float64) * (2.0 / (1 << 24)) - 1.0).astype(np.float32)


def stress_f32(P: int, rank: int, n: int, seed: int = 1234) -> np.ndarray:
    scale = np.float32(2.0 ** ((3 * rank) % 17))
    return uniform_f32(n, seed * 1000003 + P * 1009 + rank) * scale


def int32_bucket(P: int, rank: int, n: int, seed: int = 7) -> np.ndarray:
    """int32 values in [-2^20, 2^20): an 8-rank sum cannot overflow."""
    bits = _splitmix(np.arange(n, dtype=np.uint64), seed * 7919 + P * 131 + rank) >> np.uint64(43)
    return (bits.astype(np.int64) - (1 << 20)).astype(np.int32)


def new_inputs(P: int, rank: int, n: int, inputs: int = 1, dtype=np.float32) -> list[np.ndarray]:
    stride = P * inputs
    j = np.arange(n, dtype=np.float64)
    return [(j * stride + rank * inputs + i).astype(dtype) for i in range(inputs)]


def bew_inputs(rank: int, n: int) -> np.ndarray:
    i = np.arange(n, dtype=np.float64)
    # the reference computes in double then stores to float (main.cc:644)
    return (i * (rank + 1.0)).astype(np.float32)


def bf16_bits(x: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 bit pattern, round-to-nearest-even (finite inputs)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return u.astype(np.uint16)


def bf16_to_f32(h: np.ndarray) -> np.ndarray:
    return (h.astype(np.uint32) << np.uint32(16)).view(np.float32)


# ---- order-sensitive values at arbitrary element indices (numpy or torch, any device) ----------
_MASK32 = 0xFFFFFFFF


def _mul32(h, c: int):
    """(h * c) mod 2^32 for 0 <= h < 2^32 in int64 arithmetic: no partial product reaches 2^49,
    so numpy and torch (CPU or GPU) give the same bits with no signed overflow."""
    return (h * (c & 0xFFFF) + (((h * (c >> 16)) & 0xFFFF) << 16)) & _MASK32


def _fmix32(h):
    """murmur3's 32-bit finaliser."""
    h = h ^ (h >> 16)
    h = _mul32(h, 0x85EBCA6B)
    h = h ^ (h >> 13)
    h = _mul32(h, 0xC2B2AE35)
    return h ^ (h >> 16)


def stress_at(P: int, rank: int, idx, seed: int = 77):
    """stress_f32's distribution -- uniform[-1, 1) with 24 random mantissa bits, times
    2^(3r mod 17) -- at element indices `idx` (an int64 numpy array or torch tensor): the same
    fp32 bits from numpy and from torch on any device, so a full-size bucket is generated on the
    GPU and any sample of it re-derived on the CPU (BASELINE configs 4/5 at full size)."""
    s = (seed * 1000003 + P * 1009 + rank * 7919) & _MASK32
    h = _fmix32((_mul32(idx & _MASK32, 0x9E3779B1) + s) & _MASK32)
    m = h >> 8  # 24 bits
    scale = float(2.0 ** ((3 * rank) % 17))
    if isinstance(idx, np.ndarray):
        f = m.astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1.0)
        return f * np.float32(scale)
    import torch

    return (m.to(torch.float32) * (2.0 ** -23) - 1.0) * scale


def fill_at(gen, P: int, rank: int, n: int, device, dtype, chunk: int = 16 << 20, out=None):
    """gen(P, rank, idx) (stress_at / stress_cancel_at) over all n indices as a torch tensor of
    `dtype` on `device` (bf16: RNE, as bf16_bits), generated `chunk` elements at a time: the
    int64 indices and hashing temporaries of a 256 Mi bucket would otherwise take several GiB.
    Writes into `out` when given."""
    import torch

    if out is None:
        out = torch.empty(n, dtype=dtype, device=device)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        out[lo:hi] = gen(P, rank, torch.arange(lo, hi, device=device, dtype=torch.int64)).to(dtype)
    return out


def stress_cancel_at(P: int, rank: int, idx, seed: int = 91):
    """Fold-order stress for buckets that are rounded once more after the fold (config 5: fp32
    accumulation of bf16 data, one rounding to bf16).  stress_at's values differ between fold
    orders only in fp32's last bits, which the final bf16 rounding hides; here, per element, two
    ranks i != j (the same choice on every rank) hold +B and -B, B = 2^k with k in [20, 27], and
    every other rank a small value u * 2^(0..4): the small values added while B is in the running
    sum are rounded to B's fp32 grid, and which of them are depends on the order, so after B
    cancels the difference survives the bf16 rounding.  Exact in bf16 (B is a power of two; the
    caller rounds the small values).  numpy or torch, as stress_at."""
    h = _fmix32((_mul32(idx & _MASK32, 0x9E3779B1) + (seed * 7919 + P * 104729)) & _MASK32)
    i = h % P
    j = (i + 1 + (h >> 8) % max(1, P - 1)) % P
    k = 20 + (h >> 16) % 8
    bbits = (k + 127) << 23  # the fp32 bit pattern of 2^k
    small = stress_at(P, rank, idx, seed=seed + 1)  # u * 2^((3r) mod 17): rescaled below
    hr = _fmix32((_mul32(idx & _MASK32, 0x85EBCA77) + rank * 2654435761 + seed) & _MASK32)
    e = hr % 5
    if isinstance(idx, np.ndarray):
        big = bbits.astype(np.int32).view(np.float32)
        ebits = ((e + 127) << 23).astype(np.int32).view(np.float32)  # 2^e
        u = small / np.float32(2.0 ** ((3 * rank) % 17))
        v = (u * ebits).astype(np.float32)
        return np.where(rank == i, big, np.where(rank == j, -big, v)).astype(np.float32)
    import torch

    big = bbits.to(torch.int32).view(torch.float32)
    ebits = ((e + 127) << 23).to(torch.int32).view(torch.float32)
    u = small / float(2.0 ** ((3 * rank) % 17))
    v = u * ebits
    return torch.where(i == rank, big, torch.where(j == rank, -big, v))
