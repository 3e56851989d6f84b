// reduce_ops.h -- device-side element operations shared by the gfx950 kernels
// (reduce_kernels.hip: chunk-sum / fold; peer_kernels.hip: peer-access allreduce).
// Numerics reproduce the reference's x86 build bit for bit: IEEE RNE,
// subnormals kept (no FTZ), x86 NaN propagation (first NaN operand quieted, else default NaN
// 0xFFC00000), integer wrap, and gloo::float16's store quirk.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "reduce_kernels.h"

namespace hydra {
// -------------------------------------------------------------------------------------------
// element ops
// -------------------------------------------------------------------------------------------
struct f16_t { uint16_t x; };
struct bf16_t { uint16_t x; };

__device__ __forceinline__ uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint64_t dbits(double f) { return __builtin_bit_cast(uint64_t, f); }
__device__ __forceinline__ double bitsd(uint64_t u) { return __builtin_bit_cast(double, u); }

// x86 SSE NaN result of a binary arithmetic op: first NaN operand, quieted; else default NaN.
// Branch-free (selects only): the NaN fix-up must not put execz branches in the stream loop.
__device__ __forceinline__ float x86_nan(float a, float b) {
  const uint32_t qa = fbits(a) | 0x00400000u, qb = fbits(b) | 0x00400000u;
  return bitsf((a != a) ? qa : ((b != b) ? qb : 0xFFC00000u));
}
__device__ __forceinline__ double x86_nan(double a, double b) {
  const uint64_t qa = dbits(a) | 0x0008000000000000ull, qb = dbits(b) | 0x0008000000000000ull;
  return bitsd((a != a) ? qa : ((b != b) ? qb : 0xFFF8000000000000ull));
}

template <int OP, typename T>
__device__ __forceinline__ T fop(T a, T b) {  // float / double
  T r;
  if (OP == kSum) r = a + b;
  else if (OP == kProduct) r = a * b;
  else if (OP == kMax) return (a < b) ? b : a;  // std::max operand order (math.h:50-56)
  else return (b < a) ? b : a;                  // std::min (math.h:64-70)
  return (r != r) ? x86_nan(a, b) : r;
}

template <int OP, typename T, typename U>
__device__ __forceinline__ T iop(T a, T b) {  // integers, modulo 2^bits
  if (OP == kSum) return (T)((U)a + (U)b);
  if (OP == kProduct) return (T)((U)a * (U)b);
  if (OP == kMax) return (a < b) ? b : a;
  return (b < a) ? b : a;
}

// gloo::float16 conversions (types.h:207-320): RNE; NaN -> 0x7fff.  The hardware converts
// exactly like the reference for every non-NaN input (RNE, subnormals, overflow at 65520).
__device__ __forceinline__ float h2f(uint16_t h) {
  return (float)__builtin_bit_cast(_Float16, h);
}
__device__ __forceinline__ uint16_t f2h(float f) {
  if (f != f) return 0x7fffu;
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}
// float16::operator= skips the store when new == f2h((float)old_bits) (types.h:112-130).
__device__ __forceinline__ uint16_t f16_assign(uint16_t old_bits, uint16_t new_bits) {
  return (new_bits == f2h((float)old_bits)) ? old_bits : new_bits;
}
template <int OP>
__device__ __forceinline__ uint16_t f16op(uint16_t L, uint16_t R, uint16_t C0) {
  float x = h2f(L), y = h2f(R);
  uint16_t res;
  if (OP == kSum) res = f16_assign(L, f2h(x + y));
  else if (OP == kProduct) res = f16_assign(L, f2h(x * y));
  else if (OP == kMax) res = (x < y) ? R : L;
  else res = (y < x) ? R : L;
  return f16_assign(C0, res);
}

// bf16: fp32 compute (x86 NaN rules), RNE back, NaN kept quiet (oracle/hydra_oracle.c orc_f2bf)
__device__ __forceinline__ float bf2f(uint16_t h) { return bitsf((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = fbits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
template <int OP>
__device__ __forceinline__ uint16_t bf16op(uint16_t a, uint16_t b) {
  float x = bf2f(a), y = bf2f(b);
  if (OP == kMax) return (x < y) ? b : a;
  if (OP == kMin) return (y < x) ? b : a;
  return f2bf(fop<OP>(x, y));
}

// Uniform element interface: E = storage type; apply(L, R, C0).
template <typename E, int OP> struct Elem;
#define HYDRA_IELEM(E, U)                                                                 \
  template <int OP> struct Elem<E, OP> {                                                  \
    static constexpr bool kNeedsOld = false;                                              \
    __device__ __forceinline__ static E apply(E a, E b, E) { return iop<OP, E, U>(a, b); } \
  };
HYDRA_IELEM(int8_t, uint32_t)
HYDRA_IELEM(uint8_t, uint32_t)
HYDRA_IELEM(int32_t, uint32_t)
HYDRA_IELEM(uint32_t, uint32_t)
HYDRA_IELEM(int64_t, uint64_t)
HYDRA_IELEM(uint64_t, uint64_t)
template <int OP> struct Elem<float, OP> {
  static constexpr bool kNeedsOld = false;
  __device__ __forceinline__ static float apply(float a, float b, float) { return fop<OP>(a, b); }
};
template <int OP> struct Elem<double, OP> {
  static constexpr bool kNeedsOld = false;
  __device__ __forceinline__ static double apply(double a, double b, double) {
    return fop<OP>(a, b);
  }
};
template <int OP> struct Elem<f16_t, OP> {
  static constexpr bool kNeedsOld = true;
  __device__ __forceinline__ static f16_t apply(f16_t a, f16_t b, f16_t c0) {
    return f16_t{f16op<OP>(a.x, b.x, c0.x)};
  }
};
template <int OP> struct Elem<bf16_t, OP> {
  static constexpr bool kNeedsOld = false;
  __device__ __forceinline__ static bf16_t apply(bf16_t a, bf16_t b, bf16_t) {
    return bf16_t{bf16op<OP>(a.x, b.x)};
  }
};

// -------------------------------------------------------------------------------------------
// 16-byte vectors
// -------------------------------------------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));  // may be unaligned

template <typename E>
struct Vec {
  static constexpr int N = 16 / sizeof(E);
  union { u32x4 raw; E e[N]; };
};

// Memory policies of the 16-B accesses: plain global, global nontemporal ("nt"), or a buffer
// access with explicit gfx950 cache-policy bits (aux: 1 = sc0, 2 = nt, 16 = sc1).
enum Pol { kPlain = 0, kNT = 1, kBuf = 0x100 };

template <int POL>
__device__ __forceinline__ u32x4 ld(const char* base, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (POL == kNT) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(base + off));
  } else if constexpr (POL & kBuf) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, POL & 0xff);
  } else {
    return *reinterpret_cast<const u32x4_u*>(base + off);
  }
}
template <int POL>
__device__ __forceinline__ void st(char* base, __amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  if constexpr (POL == kNT) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(base + off));
  } else if constexpr (POL & kBuf) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, POL & 0xff);
  } else {
    *reinterpret_cast<u32x4*>(base + off) = v;
  }
}
template <int POL>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char* base, uint32_t bytes) {
  if constexpr ((POL & kBuf) != 0)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, bytes, 0x00020000);
  else
    return __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0);
}
// plain element-aligned 16-B accesses for the predicated paths
__device__ __forceinline__ u32x4 ld_u(const void* p) { return *reinterpret_cast<const u32x4_u*>(p); }
__device__ __forceinline__ void st_a(void* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }

template <typename E, int OP>
__device__ __forceinline__ u32x4 vapply(u32x4 ra, u32x4 rb, u32x4 rc) {
  Vec<E> va, vb, vc, vo;
  va.raw = ra;
  vb.raw = rb;
  vc.raw = rc;
#pragma unroll
  for (int k = 0; k < Vec<E>::N; k++) vo.e[k] = Elem<E, OP>::apply(va.e[k], vb.e[k], vc.e[k]);
  return vo.raw;
}


// -------------------------------------------------------------------------------------------
// P-way fold (the DIRECT allreduce's owner step, xgmi_plan.h):
//   dst = src[0] + (src[1] + (... + (src[P-2] + src[P-1])))
// with src[0] = this rank's own block (x_q) and src[j] = rank q+j's contribution, i.e. exactly
// the per-element sequence of c = local + received hops that the reference's ring performs on
// the owner's block (allreduce.cc:301-305), so the result is bit-identical to the ring.
// dst may equal src[0].  ACC32: bf16 inputs, fp32 accumulation, one RNE rounding to bf16.
// -------------------------------------------------------------------------------------------
struct FoldSrcs {
  const char* p[kMaxRanks];
};

template <bool NT>
__device__ __forceinline__ u32x4 ld_src(const char* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(p));
  else return ld_u(p);
}

template <typename E, int OP, bool ACC32, bool NT>
__device__ __forceinline__ u32x4 fold_vec(const FoldSrcs& S, int nsrc, size_t off) {
  if constexpr (ACC32) {
    static_assert(sizeof(E) == 2, "ACC32 is the bf16 form");
    u32x4 last = ld_src<NT>(S.p[nsrc - 1] + off);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      acc[2 * k] = bitsf(last[k] << 16);
      acc[2 * k + 1] = bitsf(last[k] & 0xffff0000u);
    }
    for (int j = nsrc - 2; j >= 0; j--) {
      u32x4 x = ld_src<NT>(S.p[j] + off);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        acc[2 * k] = fop<OP>(bitsf(x[k] << 16), acc[2 * k]);
        acc[2 * k + 1] = fop<OP>(bitsf(x[k] & 0xffff0000u), acc[2 * k + 1]);
      }
    }
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; k++)
      o[k] = (uint32_t)f2bf(acc[2 * k]) | ((uint32_t)f2bf(acc[2 * k + 1]) << 16);
    return o;
  } else {
    u32x4 acc = ld_src<NT>(S.p[nsrc - 1] + off);
    for (int j = nsrc - 2; j >= 0; j--) {
      u32x4 x = ld_src<NT>(S.p[j] + off);
      acc = vapply<E, OP>(x, acc, x);  // c = local + received, in place on local (C0 = local)
    }
    return acc;
  }
}

template <typename E, int OP, bool ACC32>
__device__ __forceinline__ E fold_elem(const FoldSrcs& S, int nsrc, ptrdiff_t i) {
  if constexpr (ACC32) {
    float acc = bf2f(reinterpret_cast<const uint16_t*>(S.p[nsrc - 1])[i]);
    for (int j = nsrc - 2; j >= 0; j--)
      acc = fop<OP>(bf2f(reinterpret_cast<const uint16_t*>(S.p[j])[i]), acc);
    E r;
    uint16_t h = f2bf(acc);
    __builtin_memcpy(&r, &h, 2);
    return r;
  } else {
    E acc = reinterpret_cast<const E*>(S.p[nsrc - 1])[i];
    for (int j = nsrc - 2; j >= 0; j--) {
      const E x = reinterpret_cast<const E*>(S.p[j])[i];
      acc = Elem<E, OP>::apply(x, acc, x);
    }
    return acc;
  }
}

// S.p[*] and dst already advanced by `head` elements (dst 16-B aligned at the body).

}  // namespace hydra
