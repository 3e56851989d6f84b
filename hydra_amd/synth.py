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
