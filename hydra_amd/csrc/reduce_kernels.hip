// reduce_kernels.hip -- gfx950 (MI355X, CDNA4) streaming element-wise reduction kernels.
//
// The hot path is c[i] = op(a[i], b[i]) over one ring segment (gloo::sum<T>, math.h:15-23, called
// in place c == a at allreduce.cc:301-305).  It is a pure HBM stream: 12 B per fp32 element
// (read a, read b, write c), no reuse, no MFMA.  Design:
//   * 16 B per lane per access (global_load_dwordx4 / global_store_dwordx4), wave64 lanes on
//     consecutive 16-B slots -> every wave-instruction moves 1 KiB, fully coalesced;
//   * UNROLL independent vectors per operand per lane in flight before the first use;
//   * aligned on the *store* stream c; a and b may sit at any element alignment relative to c
//     (the ring's tmp slot 1 is at +segmentBytes, a multiple of 4 only: allreduce.cc:236) --
//     gfx950 runs under unaligned-access mode, so under-aligned 16-B loads stay dwordx4;
//   * the ragged head (until c is 16-B aligned) and tail (< one vector) are done lane-per-element
//     by two wavefronts of block 0, so the vector loop carries no per-element predicate;
//   * a grid-stride loop over contiguous tiles; the launcher picks the grid from the size.
// Numerics reproduce the reference's x86 build bit for bit: IEEE RNE, subnormals
// kept (no FTZ), x86 NaN propagation (first NaN operand quieted, else default NaN 0xFFC00000),
// integer wrap, and gloo::float16's store quirk.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "errors.h"
#include "reduce_kernels.h"
#include "reduce_ops.h"

namespace hydra {
namespace {

// -------------------------------------------------------------------------------------------
// the streaming kernel
//   c, a, b   : element pointers at the first element of the vector body (c 16-B aligned)
//   nvec      : number of 16-B vectors in the body
//   head/tail : scalar elements before (at c - head) / after the body, each < Vec<E>::N
//   C_OLD     : load c's old bits (float16 store quirk when c is not a)
// -------------------------------------------------------------------------------------------
// MAP 1: XCD-contiguous tiles -- the dispatcher deals workgroups round-robin to the 8 XCDs, so
// block b runs on XCD b % 8; remapping it to tile (b % 8) * (grid / 8) + b / 8 gives each XCD
// one contiguous eighth of the stream instead of every eighth tile (measurement variant).
template <typename E, int OP, int UNROLL, int LDP, int STP, bool C_OLD, int BS = kBlock,
          int MAP = 0>
__global__ __launch_bounds__(BS) void k_reduce(E* c_, const E* a_, const E* b_, size_t nvec,
                                               int head, int tail) {
  constexpr int N = Vec<E>::N;
  constexpr size_t TILE = (size_t)BS * UNROLL;
  static_assert(BS >= 128, "waves 0 and 1 of block 0 do the ragged head and tail");
  char* c = reinterpret_cast<char*>(c_);
  const char* a = reinterpret_cast<const char*>(a_);
  const char* b = reinterpret_cast<const char*>(b_);
  const int t = threadIdx.x;

  // ragged edges: wave 0 of block 0 takes the head, wave 1 the tail (one element per lane)
  if (blockIdx.x == 0) {
    if (t < head) {
      const int i = t - head;
      E ea = a_[i], eb = b_[i];
      E ec = C_OLD ? c_[i] : ea;
      c_[i] = Elem<E, OP>::apply(ea, eb, ec);
    } else if (t >= 64 && t - 64 < tail) {
      const size_t i = nvec * N + (size_t)(t - 64);
      E ea = a_[i], eb = b_[i];
      E ec = C_OLD ? c_[i] : ea;
      c_[i] = Elem<E, OP>::apply(ea, eb, ec);
    }
  }

  const size_t ntiles = (nvec + TILE - 1) / TILE;
  size_t first = blockIdx.x;
  if (MAP == 1 && (gridDim.x & 7) == 0) first = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  for (size_t tile = first; tile < ntiles; tile += gridDim.x) {
    const size_t tbase = tile * TILE * 16;  // byte offset of this tile
    if ((tile + 1) * TILE <= nvec) {        // full tile: no predicates
      const char* at = a + tbase;
      const char* bt = b + tbase;
      char* ct = c + tbase;
      const auto ra_ = rsrc<LDP>(at, TILE * 16), rb_ = rsrc<LDP>(bt, TILE * 16);
      const auto rc_ = rsrc<LDP>(ct, TILE * 16), wc_ = rsrc<STP>(ct, TILE * 16);
      u32x4 ra[UNROLL], rb[UNROLL], rc[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        const uint32_t off = (uint32_t)(u * BS + t) * 16;
        ra[u] = ld<LDP>(at, ra_, off);
        rb[u] = ld<LDP>(bt, rb_, off);
        if (C_OLD) rc[u] = ld<LDP>(ct, rc_, off);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        const uint32_t off = (uint32_t)(u * BS + t) * 16;
        st<STP>(ct, wc_, off, vapply<E, OP>(ra[u], rb[u], C_OLD ? rc[u] : ra[u]));
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        const size_t v = tile * TILE + (size_t)u * BS + t;
        if (v < nvec) {
          const size_t off = v * 16;
          u32x4 x = ld_u(a + off), y = ld_u(b + off);
          u32x4 z = C_OLD ? ld_u(c + off) : x;
          st_a(c + off, vapply<E, OP>(x, y, z));
        }
      }
    }
  }
}

#ifdef HYDRA_MEASURE  // k_reduce_lds / k_reduce_shfl: measurement variants 13, 18, 44 (libhydra_measure.so)
// -------------------------------------------------------------------------------------------
// LDS-DMA double-buffered variant (the staging the north star names; A/B'd against k_reduce).
// Each wave streams its own wave-tiles (64 lanes x 16 B x U per operand) with
// global_load_lds_dwordx4 (nt) into a private 2-deep LDS ring, so no workgroup barrier is
// needed: the wave's own counted vmcnt orders its ds_reads behind its DMA.  Loads of wave-tile
// k+1 are in flight while tile k is read back, summed and stored.  Full wave-tiles only; the
// remainder (< 64*U vectors) is done by the register path of global wave 0.
// -------------------------------------------------------------------------------------------
template <int U>
__device__ __forceinline__ void wait_vm(int k_gt0, int has_next) {
  // vector-memory ops younger than wave-tile k's loads: stores of k-1 (U) + loads of k+1 (2U)
  if (k_gt0) {
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * U) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(U) : "memory");
  } else {
    if (has_next) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * U) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <typename E, int OP, int U, bool C_OLD>
__global__ __launch_bounds__(kBlock) void k_reduce_lds(E* c_, const E* a_, const E* b_,
                                                       size_t nvec, int head, int tail) {
  constexpr int N = Vec<E>::N;
  constexpr int WT = 64 * U;                  // vectors per wave-tile
  constexpr int SLOT = 64 * U;                // u32x4 per (buffer, operand) per wave
  __shared__ u32x4 lds[4][2][2][SLOT];        // [wave][buffer][a|b][..]
  char* c = reinterpret_cast<char*>(c_);
  const char* a = reinterpret_cast<const char*>(a_);
  const char* b = reinterpret_cast<const char*>(b_);
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);

  if (blockIdx.x == 0) {
    if (t < head) {
      const int i = t - head;
      E ea = a_[i], eb = b_[i];
      c_[i] = Elem<E, OP>::apply(ea, eb, C_OLD ? c_[i] : ea);
    } else if (t >= 64 && t - 64 < tail) {
      const size_t i = nvec * N + (size_t)(t - 64);
      E ea = a_[i], eb = b_[i];
      c_[i] = Elem<E, OP>::apply(ea, eb, C_OLD ? c_[i] : ea);
    }
  }

  const size_t nwt = nvec / WT;                       // full wave-tiles
  const size_t gw = (size_t)blockIdx.x * 4 + wave;    // global wave id
  const size_t GW = (size_t)gridDim.x * 4;
  using lds_ptr = __attribute__((address_space(3))) void*;
  auto issue = [&](size_t wt, int buf) {
    const size_t base = wt * WT * 16;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t off = base + (size_t)(u * 64 + lane) * 16;
      __builtin_amdgcn_global_load_lds(a + off, (lds_ptr)&lds[wave][buf][0][u * 64], 16, 0, 2);
      __builtin_amdgcn_global_load_lds(b + off, (lds_ptr)&lds[wave][buf][1][u * 64], 16, 0, 2);
    }
  };
  size_t wt = gw;
  int k = 0;
  if (wt < nwt) issue(wt, 0);
  for (; wt < nwt; wt += GW, k++) {
    const int buf = k & 1;
    const int has_next = (wt + GW < nwt);
    if (has_next) issue(wt + GW, buf ^ 1);
    wait_vm<U>(k > 0, has_next);
    const size_t base = wt * WT * 16;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t off = base + (size_t)(u * 64 + lane) * 16;
      u32x4 x = lds[wave][buf][0][u * 64 + lane];
      u32x4 y = lds[wave][buf][1][u * 64 + lane];
      u32x4 z = C_OLD ? ld_u(c + off) : x;
      __builtin_nontemporal_store(vapply<E, OP>(x, y, z), reinterpret_cast<u32x4*>(c + off));
    }
  }
  // remainder vectors (< WT), register path, global wave 0
  if (gw == 0) {
    for (size_t v = nwt * WT + lane; v < nvec; v += 64) {
      const size_t off = v * 16;
      u32x4 x = ld_u(a + off), y = ld_u(b + off);
      st_a(c + off, vapply<E, OP>(x, y, C_OLD ? ld_u(c + off) : x));
    }
  }
}

// -------------------------------------------------------------------------------------------
// Wavefront-shuffle realignment (the north star's "wavefront-shuffle" on gfx950).
// An operand whose address is not co-aligned with c mod 16 B (the ring's tmp slot 1 sits at
// +segmentBytes, a multiple of E only: allreduce.cc:236; user sub-buffers) is read with ALIGNED
// 16-B loads only: lane i loads the aligned slot under the start of its window, receives slot
// i+1 from lane i+1 through a DPP wave_shl:1 (one v_mov_dpp per dword, VALU, no LDS), and cuts
// its window out of the 32-byte pair with v_alignbyte.  Lane 63's window reaches into the next
// wave's first slot, so lane 63 alone reads its window directly (unaligned, within bounds).
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_shl1(uint32_t x) {
  // DPP_WF_SL1 (0x130, GFX9 family): lane i reads lane i+1; lane 63 keeps `old` (ignored)
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, false);
}

// bytes [k, k+16) of the 32-byte pair (x, y); k = 4q + r, 1 <= k <= 15, q and r wave-uniform
__device__ __forceinline__ u32x4 realign(u32x4 x, u32x4 y, int q, uint32_t r) {
  const uint32_t d[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  auto cut = [&](auto Q) {  // constant dword offset: four v_alignbyte, no per-lane select
    constexpr int s = decltype(Q)::value;
    return u32x4{__builtin_amdgcn_alignbyte(d[s + 1], d[s], r),
                 __builtin_amdgcn_alignbyte(d[s + 2], d[s + 1], r),
                 __builtin_amdgcn_alignbyte(d[s + 3], d[s + 2], r),
                 __builtin_amdgcn_alignbyte(d[s + 4], d[s + 3], r)};
  };
  switch (q) {  // wave-uniform: one scalar branch
    case 0: return cut(std::integral_constant<int, 0>{});
    case 1: return cut(std::integral_constant<int, 1>{});
    case 2: return cut(std::integral_constant<int, 2>{});
    default: return cut(std::integral_constant<int, 3>{});
  }
}

// x = the aligned slot under this lane's window, u = lane 63's own window (unaligned load);
// k = the operand's misalignment (wave-uniform).  Returns this lane's window.
__device__ __forceinline__ u32x4 shfl_window(u32x4 x, u32x4 u, uint32_t k, int lane) {
  if (k == 0) return x;
  u32x4 y;
#pragma unroll
  for (int j = 0; j < 4; j++) y[j] = wave_shl1(x[j]);
  const u32x4 o = realign(x, y, (int)(k >> 2), k & 3);
  return lane == 63 ? u : o;
}

template <typename E, int OP, bool C_OLD>
__global__ __launch_bounds__(kBlock) void k_reduce_shfl(E* c_, const E* a_, const E* b_,
                                                        size_t nvec, int head, int tail) {
  constexpr int N = Vec<E>::N;
  constexpr size_t TILE = kBlock;  // one 16-B vector per lane per operand (the tuned default)
  char* c = reinterpret_cast<char*>(c_);
  const char* a = reinterpret_cast<const char*>(a_);
  const char* b = reinterpret_cast<const char*>(b_);
  const int t = threadIdx.x, lane = t & 63;
  const uint32_t ka = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)a & 15));
  const uint32_t kb = __builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)b & 15));

  if (blockIdx.x == 0) {
    if (t < head) {
      const int i = t - head;
      E ea = a_[i], eb = b_[i];
      c_[i] = Elem<E, OP>::apply(ea, eb, C_OLD ? c_[i] : ea);
    } else if (t >= 64 && t - 64 < tail) {
      const size_t i = nvec * N + (size_t)(t - 64);
      E ea = a_[i], eb = b_[i];
      c_[i] = Elem<E, OP>::apply(ea, eb, C_OLD ? c_[i] : ea);
    }
  }

  const size_t ntiles = (nvec + TILE - 1) / TILE;
  size_t first = blockIdx.x;  // XCD-contiguous tiles, as the default
  if ((gridDim.x & 7) == 0) first = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  for (size_t tile = first; tile < ntiles; tile += gridDim.x) {
    const size_t off = (tile * TILE + t) * 16;
    if ((tile + 1) * TILE <= nvec) {  // full tile: every lane of every wave is live
      // every load issued before the first use: aligned slots, then lane 63's own windows
      u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a - ka + off));
      u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(b - kb + off));
      u32x4 ux = {0, 0, 0, 0}, uy = {0, 0, 0, 0};  // (not x/y: no wait on their loads)
      if (lane == 63 && ka) ux = ld_u(a + off);
      if (lane == 63 && kb) uy = ld_u(b + off);
      u32x4 z;
      if (C_OLD) z = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(c + off));
      x = shfl_window(x, ux, ka, lane);
      y = shfl_window(y, uy, kb, lane);
      if (!C_OLD) z = x;  // the f16 store quirk's old bits are a's in the in-place form
      const auto w = rsrc<kBuf | 16>(c + tile * TILE * 16, TILE * 16);
      st<kBuf | 16>(c, w, (uint32_t)t * 16, vapply<E, OP>(x, y, z));
    } else if (tile * TILE + t < nvec) {
      u32x4 x = ld_u(a + off), y = ld_u(b + off);
      st_a(c + off, vapply<E, OP>(x, y, C_OLD ? ld_u(c + off) : x));
    }
  }
}

#endif  // HYDRA_MEASURE

// -------------------------------------------------------------------------------------------
// bf16 bucket, fp32 accumulate (BASELINE config 5): acc[i] += float(b[i]); 10 B / element.
// acc 16-B aligned (we own it), b element-aligned.  8 elements per lane per step.
// -------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_acc_bf16(float* __restrict__ acc,
                                                     const uint16_t* __restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  const size_t n8 = n / 8;
  for (size_t v = (size_t)blockIdx.x * kBlock + threadIdx.x; v < n8; v += stride) {
    u32x4 bb = *reinterpret_cast<const u32x4_u*>(b + v * 8);
    u32x4 a0 = *reinterpret_cast<const u32x4*>(acc + v * 8);
    u32x4 a1 = *reinterpret_cast<const u32x4*>(acc + v * 8 + 4);
    Vec<float> x0, x1;
    x0.raw = a0;
    x1.raw = a1;
    x0.e[0] = fop<kSum>(x0.e[0], bitsf(bb[0] << 16));
    x0.e[1] = fop<kSum>(x0.e[1], bitsf(bb[0] & 0xffff0000u));
    x0.e[2] = fop<kSum>(x0.e[2], bitsf(bb[1] << 16));
    x0.e[3] = fop<kSum>(x0.e[3], bitsf(bb[1] & 0xffff0000u));
    x1.e[0] = fop<kSum>(x1.e[0], bitsf(bb[2] << 16));
    x1.e[1] = fop<kSum>(x1.e[1], bitsf(bb[2] & 0xffff0000u));
    x1.e[2] = fop<kSum>(x1.e[2], bitsf(bb[3] << 16));
    x1.e[3] = fop<kSum>(x1.e[3], bitsf(bb[3] & 0xffff0000u));
    *reinterpret_cast<u32x4*>(acc + v * 8) = x0.raw;
    *reinterpret_cast<u32x4*>(acc + v * 8 + 4) = x1.raw;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
    const size_t i = n8 * 8 + threadIdx.x;
    acc[i] = fop<kSum>(acc[i], bf2f(b[i]));
  }
}

__global__ __launch_bounds__(kBlock) void k_f32_to_bf16(uint16_t* __restrict__ out,
                                                        const float* __restrict__ acc, size_t n) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    out[i] = f2bf(acc[i]);
}

// P-way fold in the reference ring's order (reduce_ops.h fold_vec / fold_elem).
template <typename E, int OP, bool ACC32, bool NT, int MAP = 0>
__global__ __launch_bounds__(kBlock) void k_fold(E* dst, FoldSrcs S, int nsrc, size_t nvec,
                                                 int head, int tail) {
  constexpr int N = Vec<E>::N;
  const int t = threadIdx.x;
  if (blockIdx.x == 0) {
    if (t < head) {
      dst[t - head] = fold_elem<E, OP, ACC32>(S, nsrc, (ptrdiff_t)t - head);
    } else if (t >= 64 && t - 64 < tail) {
      const ptrdiff_t i = (ptrdiff_t)(nvec * N) + (t - 64);
      dst[i] = fold_elem<E, OP, ACC32>(S, nsrc, i);
    }
  }
  char* d = reinterpret_cast<char*>(dst);
  const size_t stride = (size_t)gridDim.x * kBlock;
  size_t first = blockIdx.x;  // MAP 1: XCD-contiguous blocks within each grid stride (k_reduce)
  if (MAP == 1 && (gridDim.x & 7) == 0) first = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  for (size_t vb = first * kBlock; vb < nvec; vb += stride) {  // wave-uniform
    const size_t v = vb + t;
    // write-through (sc1) store through a block-uniform descriptor, as the chunk-sum default
    const auto w = __builtin_amdgcn_make_buffer_rsrc(d + vb * 16, 0, kBlock * 16, 0x00020000);
    if (v < nvec)
      __builtin_amdgcn_raw_buffer_store_b128(fold_vec<E, OP, ACC32, NT>(S, nsrc, v * 16), w,
                                             (uint32_t)t * 16, 0, 16);
  }
}

#ifdef HYDRA_MEASURE  // k_reduce_pers: measurement variants 45-47
// -------------------------------------------------------------------------------------------
// Persistent, software-pipelined variant (measurement: variants 45-47).  A capped grid of
// CUs x W workgroups; each workgroup streams ONE contiguous range of tiles (XCD-contiguous
// logical ids), loading tile k+1 while it adds and stores tile k, so every wave keeps its loads
// in flight across tiles without the dispatcher launching a new workgroup per 4 KiB tile.
// -------------------------------------------------------------------------------------------
template <typename E, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_pers(E* c_, const E* a_, const E* b_,
                                                        size_t nvec, int head, int tail) {
  constexpr int N = Vec<E>::N;
  char* c = reinterpret_cast<char*>(c_);
  const char* a = reinterpret_cast<const char*>(a_);
  const char* b = reinterpret_cast<const char*>(b_);
  const int t = threadIdx.x;
  if (blockIdx.x == 0) {
    if (t < head) {
      const int i = t - head;
      c_[i] = Elem<E, OP>::apply(a_[i], b_[i], a_[i]);
    } else if (t >= 64 && t - 64 < tail) {
      const size_t i = nvec * N + (size_t)(t - 64);
      c_[i] = Elem<E, OP>::apply(a_[i], b_[i], a_[i]);
    }
  }
  const uint32_t G = gridDim.x;
  uint32_t L = blockIdx.x;
  if ((G & 7) == 0) L = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const size_t ntiles = nvec / kBlock;
  const size_t per = (ntiles + G - 1) / G;
  const size_t t0 = std::min(ntiles, (size_t)L * per), t1 = std::min(ntiles, t0 + per);
  if (t0 < t1) {
    size_t off = (t0 * kBlock + t) * 16;
    u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(a + off));
    u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(b + off));
    for (size_t tile = t0; tile < t1; tile++) {
      const size_t cur = off;
      u32x4 xn = x, yn = y;
      if (tile + 1 < t1) {  // block-uniform
        off += (size_t)kBlock * 16;
        xn = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(a + off));
        yn = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(b + off));
      }
      __builtin_nontemporal_store(vapply<E, OP>(x, y, x), reinterpret_cast<u32x4*>(c + cur));
      x = xn;
      y = yn;
    }
  }
  if (L == G - 1) {  // the ragged last tile (< kBlock vectors)
    const size_t v = ntiles * kBlock + t;
    if (v < nvec) {
      const size_t o = v * 16;
      st_a(c + o, vapply<E, OP>(ld_u(a + o), ld_u(b + o), ld_u(a + o)));
    }
  }
}

#endif  // HYDRA_MEASURE

// -------------------------------------------------------------------------------------------
// Batched chunk-sum: K independent segments c_k = op(a_k, b_k) in ONE launch.  A caller that
// holds several arrived segments (consecutive ring segments, both rails of bew_allreduce_a)
// pays one dispatch and one completion instead of K: below ~1 Mi elements a launch costs a
// dispatch plus one dependent HBM round trip (~3 us) whatever its size (DESIGN.md 4.2 sweep).
// Block b serves tile b - tile0[k] of the segment k whose tile range holds b (wave-uniform
// lookup over the kernarg table); tile 0 of each segment also does its ragged head and tail.
// -------------------------------------------------------------------------------------------
struct BatchSeg {
  char* c;             // at the vector body: c 16-B aligned
  const char* a;
  const char* b;
  uint64_t nvec;       // 16-B vectors in the body
  int32_t head, tail;  // ragged elements before / after the body
  uint32_t tile0;      // first block of this segment
  uint32_t c_old;      // float16 store quirk with c != a: load c's old bits
};
struct BatchArgs {
  BatchSeg s[kMaxBatch];
  int32_t count;
};

template <typename E, int OP>
__device__ __forceinline__ void batch_edges(const BatchSeg& g, int t) {
  constexpr int N = Vec<E>::N;
  E* c_ = reinterpret_cast<E*>(g.c);
  const E* a_ = reinterpret_cast<const E*>(g.a);
  const E* b_ = reinterpret_cast<const E*>(g.b);
  const bool head = t < g.head, tail = t >= 64 && t - 64 < g.tail;
  if (!head && !tail) return;
  const ptrdiff_t i = head ? (ptrdiff_t)t - g.head : (ptrdiff_t)(g.nvec * N) + (t - 64);
  const E ea = a_[i], eb = b_[i];
  const E ec = g.c_old ? c_[i] : ea;
  c_[i] = Elem<E, OP>::apply(ea, eb, ec);
}

template <typename E, int OP>
__global__ __launch_bounds__(kBlock) void k_reduce_batch(const BatchArgs args) {
  const uint32_t bid = blockIdx.x;
  int k = 0;  // wave-uniform: the last segment whose first tile is <= this block
#pragma unroll
  for (int j = 1; j < kMaxBatch; j++)
    if (j < args.count && args.s[j].tile0 <= bid) k = j;
  const BatchSeg& g = args.s[k];
  const int t = threadIdx.x;
  const uint32_t tile = bid - g.tile0;
  if (tile == 0 && (g.head | g.tail)) batch_edges<E, OP>(g, t);
  const size_t v0 = (size_t)tile * kBlock;
  if (v0 >= g.nvec) return;
  const uint32_t off = (uint32_t)t * 16;
  const char* at = g.a + v0 * 16;
  const char* bt = g.b + v0 * 16;
  char* ct = g.c + v0 * 16;
  if (v0 + (size_t)t < g.nvec) {
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(at + off));
    const u32x4 y = __builtin_nontemporal_load(reinterpret_cast<const u32x4_u*>(bt + off));
    const u32x4 z = g.c_old ? ld_u(ct + off) : x;
    // write-through (sc1) store through a block-uniform descriptor, as the tuned chunk-sum
    const auto w = rsrc<kBuf | 16>(ct, kBlock * 16);
    st<kBuf | 16>(ct, w, off, vapply<E, OP>(x, y, z));
  }
}

// -------------------------------------------------------------------------------------------
// launch
// -------------------------------------------------------------------------------------------
// CUs of the current device (the launches go to the current device's streams), looked up once
// per device; racing first calls store the same value (was one process-wide
// value for whichever device asked first)
constexpr int kCuDevices = 64;
std::atomic<int> g_cu_count[kCuDevices] = {};

int cu_count() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  if (dev >= kCuDevices) {
    int cus = 0;
    return hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess
               ? cus : 256;
  }
  int c = g_cu_count[dev].load(std::memory_order_relaxed);
  if (!c) {
    int cus = 0;
    c = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                cus > 0
            ? cus : 256;
    g_cu_count[dev].store(c, std::memory_order_relaxed);
  }
  return c;
}

struct Split {  // head / vector body / tail of one call, aligned on c
  int head, tail;
  size_t nvec;
};

template <typename E>
Split split_call(const void* c, size_t n) {
  constexpr int N = Vec<E>::N;
  const uintptr_t cp = reinterpret_cast<uintptr_t>(c);
  Split s;
  s.head = (int)(((16 - (cp & 15)) & 15) / sizeof(E));  // elements until c is 16-B aligned
  if ((size_t)s.head > n) s.head = (int)n;
  const size_t body = n - s.head;
  s.nvec = body / N;
  s.tail = (int)(body - s.nvec * N);
  return s;
}

template <typename E, int OP, int UNROLL, int LDP, int STP, int BS = kBlock, int MAP = 0>
hipError_t launch_t(void* c, const void* a, const void* b, size_t n, hipStream_t s,
                    int max_blocks) {
  const Split sp = split_call<E>(c, n);
  E* cb = reinterpret_cast<E*>(c) + sp.head;
  const E* ab = reinterpret_cast<const E*>(a) + sp.head;
  const E* bb = reinterpret_cast<const E*>(b) + sp.head;
  constexpr size_t TILE = (size_t)BS * UNROLL;
  size_t tiles = (sp.nvec + TILE - 1) / TILE;
  if (tiles == 0) tiles = 1;
  size_t grid = tiles;
  if (max_blocks > 0 && grid > (size_t)max_blocks) grid = (size_t)max_blocks;
  const bool c_old = Elem<E, OP>::kNeedsOld && c != a;
  if (c_old)
    hipLaunchKernelGGL((k_reduce<E, OP, UNROLL, LDP, STP, true, BS, MAP>), dim3((unsigned)grid),
                       dim3(BS), 0, s, cb, ab, bb, sp.nvec, sp.head, sp.tail);
  else
    hipLaunchKernelGGL((k_reduce<E, OP, UNROLL, LDP, STP, false, BS, MAP>), dim3((unsigned)grid),
                       dim3(BS), 0, s, cb, ab, bb, sp.nvec, sp.head, sp.tail);
  return hipGetLastError();
}

#ifdef HYDRA_MEASURE  // launchers of the measurement variants
template <typename E, int OP, int U>
hipError_t launch_lds(void* c, const void* a, const void* b, size_t n, hipStream_t s,
                      int blocks_per_cu) {
  const Split sp = split_call<E>(c, n);
  E* cb = reinterpret_cast<E*>(c) + sp.head;
  const E* ab = reinterpret_cast<const E*>(a) + sp.head;
  const E* bb = reinterpret_cast<const E*>(b) + sp.head;
  size_t wts = sp.nvec / (64 * U);
  size_t grid = (wts + 3) / 4;
  const size_t cap = (size_t)cu_count() * blocks_per_cu;
  if (grid > cap) grid = cap;
  if (grid == 0) grid = 1;
  const bool c_old = Elem<E, OP>::kNeedsOld && c != a;
  if (c_old)
    hipLaunchKernelGGL((k_reduce_lds<E, OP, U, true>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       cb, ab, bb, sp.nvec, sp.head, sp.tail);
  else
    hipLaunchKernelGGL((k_reduce_lds<E, OP, U, false>), dim3((unsigned)grid), dim3(kBlock), 0,
                       s, cb, ab, bb, sp.nvec, sp.head, sp.tail);
  return hipGetLastError();
}

template <typename E, int OP>
hipError_t launch_pers(void* c, const void* a, const void* b, size_t n, hipStream_t s, int per_cu) {
  const Split sp = split_call<E>(c, n);
  E* cb = reinterpret_cast<E*>(c) + sp.head;
  const E* ab = reinterpret_cast<const E*>(a) + sp.head;
  const E* bb = reinterpret_cast<const E*>(b) + sp.head;
  size_t grid = (size_t)cu_count() * per_cu;
  const size_t tiles = (sp.nvec + kBlock - 1) / kBlock;
  if (grid > tiles) grid = tiles ? tiles : 1;
  hipLaunchKernelGGL((k_reduce_pers<E, OP>), dim3((unsigned)grid), dim3(kBlock), 0, s, cb, ab, bb,
                     sp.nvec, sp.head, sp.tail);
  return hipGetLastError();
}

template <typename E, int OP>
hipError_t launch_shfl(void* c, const void* a, const void* b, size_t n, hipStream_t s) {
  const Split sp = split_call<E>(c, n);
  E* cb = reinterpret_cast<E*>(c) + sp.head;
  const E* ab = reinterpret_cast<const E*>(a) + sp.head;
  const E* bb = reinterpret_cast<const E*>(b) + sp.head;
  size_t grid = (sp.nvec + kBlock - 1) / kBlock;
  if (grid == 0) grid = 1;
  const bool c_old = Elem<E, OP>::kNeedsOld && c != a;
  if (c_old)
    hipLaunchKernelGGL((k_reduce_shfl<E, OP, true>), dim3((unsigned)grid), dim3(kBlock), 0, s, cb,
                       ab, bb, sp.nvec, sp.head, sp.tail);
  else
    hipLaunchKernelGGL((k_reduce_shfl<E, OP, false>), dim3((unsigned)grid), dim3(kBlock), 0, s,
                       cb, ab, bb, sp.nvec, sp.head, sp.tail);
  return hipGetLastError();
}

#endif  // HYDRA_MEASURE

// The tuned default: one 16-B vector per lane per operand, nontemporal loads,
// write-through sc1 stores, tiles mapped XCD-contiguously (variant 40).  Fully HBM-resident
// (bench.py's headline, 4 rotating buffer pairs; profiles/r02_tune_rotate*.json) nontemporal
// stores (variant 42) are 1 % faster at 64 Mi; but wherever the working set can live in the
// 256 MiB Infinity Cache -- ring chunks, 4-16 Mi buckets, a bucket reduced again soon -- the sc1
// store keeps it there and wins by 16-38 % (profiles/r02_sweep_kernel_trace.txt vs
// r01_sweep_kernel_trace.txt; one pair back to back 7.5 vs 6.2 TB/s).
template <typename E, int OP>
hipError_t launch_default(void* c, const void* a, const void* b, size_t n, hipStream_t s) {
  return launch_t<E, OP, 1, kNT, kBuf | 16, kBlock, 1>(c, a, b, n, s, 0);
}

#ifdef HYDRA_MEASURE  // hydra_set_variant 1..52
template <typename E, int OP>
hipError_t launch_tuning(int variant, void* c, const void* a, const void* b, size_t n,
                          hipStream_t s) {
  const int cus = cu_count();
  constexpr int B = kBuf;
  switch (variant) {
    case 1: return launch_t<E, OP, 1, kPlain, kPlain>(c, a, b, n, s, 0);
    case 2: return launch_t<E, OP, 4, kPlain, kPlain>(c, a, b, n, s, 0);
    case 3: return launch_t<E, OP, 4, kPlain, kPlain>(c, a, b, n, s, cus * 8);
    case 4: return launch_t<E, OP, 4, kNT, kNT>(c, a, b, n, s, 0);
    case 5: return launch_t<E, OP, 2, kPlain, kPlain>(c, a, b, n, s, 0);
    case 6: return launch_t<E, OP, 8, kPlain, kPlain>(c, a, b, n, s, 0);
    case 7: return launch_t<E, OP, 4, kPlain, kPlain>(c, a, b, n, s, cus * 4);
    case 8: return launch_t<E, OP, 8, kNT, kNT>(c, a, b, n, s, 0);
    case 9: return launch_t<E, OP, 2, kNT, kNT>(c, a, b, n, s, 0);
    case 10: return launch_t<E, OP, 4, kNT, kNT>(c, a, b, n, s, cus * 8);
    case 11: return launch_t<E, OP, 4, kNT, kPlain>(c, a, b, n, s, 0);
    case 12: return launch_t<E, OP, 4, kPlain, kNT>(c, a, b, n, s, 0);
    case 13: return launch_lds<E, OP, 2>(c, a, b, n, s, 5);
    case 14: return launch_t<E, OP, 4, B | 19, B | 2>(c, a, b, n, s, 0);   // ld sc0 sc1 nt
    case 15: return launch_t<E, OP, 4, B | 2, B | 18>(c, a, b, n, s, 0);   // st sc1 nt
    case 16: return launch_t<E, OP, 4, B | 3, B | 3>(c, a, b, n, s, 0);    // sc0 nt both
    case 17: return launch_t<E, OP, 1, kNT, kNT>(c, a, b, n, s, 0);
    case 18: return launch_lds<E, OP, 4>(c, a, b, n, s, 2);
    case 19: return launch_t<E, OP, 4, kNT, kNT>(c, a, b, n, s, cus * 16);
    case 20: return launch_t<E, OP, 1, kNT, kPlain>(c, a, b, n, s, 0);
    case 21: return launch_t<E, OP, 2, kNT, kPlain>(c, a, b, n, s, 0);
    case 22: return launch_t<E, OP, 8, kNT, kPlain>(c, a, b, n, s, 0);
    case 23: return launch_t<E, OP, 4, kNT, B | 1>(c, a, b, n, s, 0);     // st sc0
    case 24: return launch_t<E, OP, 4, kNT, B | 16>(c, a, b, n, s, 0);    // st sc1
    case 25: return launch_t<E, OP, 4, kNT, B | 17>(c, a, b, n, s, 0);    // st sc0 sc1
    case 26: return launch_t<E, OP, 4, B | 2, kPlain>(c, a, b, n, s, 0);  // buffer ld nt
    case 27: return launch_t<E, OP, 4, kNT, kPlain>(c, a, b, n, s, cus * 8);
    case 28: return launch_t<E, OP, 4, kNT, kPlain>(c, a, b, n, s, cus * 32);
    case 29: return launch_t<E, OP, 2, kNT, kPlain, 512>(c, a, b, n, s, 0);
    case 30: return launch_t<E, OP, 1, kNT, kPlain, 1024>(c, a, b, n, s, 0);
    case 31: return launch_t<E, OP, 4, B | 18, kPlain>(c, a, b, n, s, 0); // ld sc1 nt
    case 32: return launch_t<E, OP, 4, B | 3, kPlain>(c, a, b, n, s, 0);  // ld sc0 nt
    case 33: return launch_t<E, OP, 1, kNT, B | 16>(c, a, b, n, s, 0);
    case 34: return launch_t<E, OP, 2, kNT, B | 16>(c, a, b, n, s, 0);
    case 35: return launch_t<E, OP, 8, kNT, B | 16>(c, a, b, n, s, 0);
    case 36: return launch_t<E, OP, 1, kNT, B | 18>(c, a, b, n, s, 0);
    case 37: return launch_t<E, OP, 4, kNT, B | 18>(c, a, b, n, s, 0);
    case 38: return launch_t<E, OP, 4, B | 18, B | 16>(c, a, b, n, s, 0);
    case 39: return launch_t<E, OP, 2, kNT, B | 16, 512>(c, a, b, n, s, 0);
    case 40: return launch_t<E, OP, 1, kNT, B | 16, kBlock, 1>(c, a, b, n, s, 0);  // 33, XCD map
    case 41: return launch_t<E, OP, 1, kNT, B | 18, kBlock, 1>(c, a, b, n, s, 0);  // 36, XCD map
    case 42: return launch_t<E, OP, 1, kNT, kNT, kBlock, 1>(c, a, b, n, s, 0);     // 17, XCD map
    case 43: return launch_t<E, OP, 2, kNT, B | 16, kBlock, 1>(c, a, b, n, s, 0);  // 34, XCD map
    case 44: return launch_shfl<E, OP>(c, a, b, n, s);  // 40 + aligned loads, DPP realignment
    case 45: return launch_pers<E, OP>(c, a, b, n, s, 4);   // persistent, pipelined, 4 WG/CU
    case 46: return launch_pers<E, OP>(c, a, b, n, s, 8);   // 8 WG/CU
    case 47: return launch_pers<E, OP>(c, a, b, n, s, 16);  // 16 WG/CU
    case 48: return launch_t<E, OP, 1, kNT, B | 17, kBlock, 1>(c, a, b, n, s, 0);  // st sc0 sc1
    case 49: return launch_t<E, OP, 1, kNT, B | 19, kBlock, 1>(c, a, b, n, s, 0);  // st sc0 sc1 nt
    case 50: return launch_t<E, OP, 1, kNT, B | 16, 128, 1>(c, a, b, n, s, 0);     // 40, 128 thr
    case 52: return launch_t<E, OP, 1, B | 2, B | 16, kBlock, 1>(c, a, b, n, s, 0); // buffer nt ld
    default: return launch_default<E, OP>(c, a, b, n, s);
  }
}

#endif  // HYDRA_MEASURE

// Measurement variants exist only for the fp32/int32 sum (the benchmarked path); every other
// dtype/op combination always runs the tuned default.
template <typename E, int OP>
hipError_t launch_variant(int variant, void* c, const void* a, const void* b, size_t n,
                          hipStream_t s) {
  constexpr bool kTunable = OP == kSum && (std::is_same<E, float>::value ||
                                          std::is_same<E, int32_t>::value);
#ifdef HYDRA_MEASURE
  if constexpr (kTunable) {
    if (variant != 0) return launch_tuning<E, OP>(variant, c, a, b, n, s);
  }
#else
  (void)variant;
  (void)kTunable;
#endif
  return launch_default<E, OP>(c, a, b, n, s);
}

template <int OP>
hipError_t dispatch_dtype(int variant, int dtype, void* c, const void* a, const void* b, size_t n,
                          hipStream_t s) {
  switch (dtype) {
    case kI8: return launch_variant<int8_t, OP>(variant, c, a, b, n, s);
    case kU8: return launch_variant<uint8_t, OP>(variant, c, a, b, n, s);
    case kI32: return launch_variant<int32_t, OP>(variant, c, a, b, n, s);
    case kU32: return launch_variant<uint32_t, OP>(variant, c, a, b, n, s);
    case kI64: return launch_variant<int64_t, OP>(variant, c, a, b, n, s);
    case kU64: return launch_variant<uint64_t, OP>(variant, c, a, b, n, s);
    case kF32: return launch_variant<float, OP>(variant, c, a, b, n, s);
    case kF64: return launch_variant<double, OP>(variant, c, a, b, n, s);
    case kF16: return launch_variant<f16_t, OP>(variant, c, a, b, n, s);
    case kBF16: return launch_variant<bf16_t, OP>(variant, c, a, b, n, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_reduce(int variant, int op, int dtype, void* c, const void* a, const void* b,
                         size_t n, hipStream_t s) {
  switch (op) {
    case kSum: return dispatch_dtype<kSum>(variant, dtype, c, a, b, n, s);
    case kProduct: return dispatch_dtype<kProduct>(variant, dtype, c, a, b, n, s);
    case kMax: return dispatch_dtype<kMax>(variant, dtype, c, a, b, n, s);
    case kMin: return dispatch_dtype<kMin>(variant, dtype, c, a, b, n, s);
  }
  return hipErrorInvalidValue;
}

namespace {
template <typename E, int OP, bool ACC32, bool NT, int MAP = 0>
hipError_t launch_fold_v(void* dst, const void* const* srcs, int nsrc, size_t n, hipStream_t s,
                         size_t cap_per_cu) {
  const Split sp = split_call<E>(dst, n);
  FoldSrcs S;
  for (int j = 0; j < kMaxRanks; j++)
    S.p[j] = j < nsrc ? reinterpret_cast<const char*>(srcs[j]) + (size_t)sp.head * sizeof(E)
                      : nullptr;
  E* d = reinterpret_cast<E*>(dst) + sp.head;
  size_t blocks = (sp.nvec + kBlock - 1) / kBlock;
  const size_t cap = (size_t)cu_count() * cap_per_cu;
  if (cap_per_cu && blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL((k_fold<E, OP, ACC32, NT, MAP>), dim3((unsigned)blocks), dim3(kBlock), 0, s, d,
                     S, nsrc, sp.nvec, sp.head, sp.tail);
  return hipGetLastError();
}

// Fold variants (hydra_set_variant, measurement only; 0 = default): 1 plain loads, grid capped
// at 8 blocks/CU; 2 nontemporal loads, capped; 3 nontemporal, one block per 256 vectors;
// 4-7 = 1, plain full grid, 3, 2 with XCD-contiguous blocks.
template <typename E, int OP, bool ACC32>
hipError_t launch_fold_t(void* dst, const void* const* srcs, int nsrc, size_t n, hipStream_t s) {
  switch (current_variant()) {
#ifdef HYDRA_MEASURE
    case 1: return launch_fold_v<E, OP, ACC32, false>(dst, srcs, nsrc, n, s, 8);
    case 2: return launch_fold_v<E, OP, ACC32, true>(dst, srcs, nsrc, n, s, 8);
    case 3: return launch_fold_v<E, OP, ACC32, true>(dst, srcs, nsrc, n, s, 0);
    case 4: return launch_fold_v<E, OP, ACC32, false, 1>(dst, srcs, nsrc, n, s, 8);  // 1, XCD map
    case 5: return launch_fold_v<E, OP, ACC32, false, 1>(dst, srcs, nsrc, n, s, 0);  // full grid
    case 6: return launch_fold_v<E, OP, ACC32, true, 1>(dst, srcs, nsrc, n, s, 0);   // 3, XCD map
    case 7: return launch_fold_v<E, OP, ACC32, true, 1>(dst, srcs, nsrc, n, s, 8);   // 2, XCD map
#endif
    default:  // tuned HBM-resident (profiles/r02_tune_fold_rot.json, 3 rotating source sets):
              // same-type folds nontemporal loads, full grid, XCD-contiguous (variant 6: P=8
              // fp32 46.5 us = 6.49 TB/s, vs 55.3 us for round 1's plain-load choice, which had
              // won the MALL-assisted steady state); bf16->fp32 nontemporal, full grid (6.53)
      if constexpr (ACC32) return launch_fold_v<E, OP, ACC32, true>(dst, srcs, nsrc, n, s, 0);
      else return launch_fold_v<E, OP, ACC32, true, 1>(dst, srcs, nsrc, n, s, 0);
  }
}

template <int OP>
hipError_t fold_dtype(int dtype, bool acc32, void* dst, const void* const* srcs, int nsrc,
                      size_t n, hipStream_t s) {
  if (acc32) {
    if (dtype != kBF16) return hipErrorInvalidValue;
    return launch_fold_t<bf16_t, OP, true>(dst, srcs, nsrc, n, s);
  }
  switch (dtype) {
    case kI8: return launch_fold_t<int8_t, OP, false>(dst, srcs, nsrc, n, s);
    case kU8: return launch_fold_t<uint8_t, OP, false>(dst, srcs, nsrc, n, s);
    case kI32: return launch_fold_t<int32_t, OP, false>(dst, srcs, nsrc, n, s);
    case kU32: return launch_fold_t<uint32_t, OP, false>(dst, srcs, nsrc, n, s);
    case kI64: return launch_fold_t<int64_t, OP, false>(dst, srcs, nsrc, n, s);
    case kU64: return launch_fold_t<uint64_t, OP, false>(dst, srcs, nsrc, n, s);
    case kF32: return launch_fold_t<float, OP, false>(dst, srcs, nsrc, n, s);
    case kF64: return launch_fold_t<double, OP, false>(dst, srcs, nsrc, n, s);
    case kF16: return launch_fold_t<f16_t, OP, false>(dst, srcs, nsrc, n, s);
    case kBF16: return launch_fold_t<bf16_t, OP, false>(dst, srcs, nsrc, n, s);
  }
  return hipErrorInvalidValue;
}
}  // namespace

hipError_t launch_fold(int op, int dtype, bool acc32, void* dst, const void* const* srcs,
                       int nsrc, size_t n, hipStream_t s) {
  if (nsrc < 1 || nsrc > kMaxRanks) return hipErrorInvalidValue;
  switch (op) {
    case kSum: return fold_dtype<kSum>(dtype, acc32, dst, srcs, nsrc, n, s);
    case kProduct: return fold_dtype<kProduct>(dtype, acc32, dst, srcs, nsrc, n, s);
    case kMax: return fold_dtype<kMax>(dtype, acc32, dst, srcs, nsrc, n, s);
    case kMin: return fold_dtype<kMin>(dtype, acc32, dst, srcs, nsrc, n, s);
  }
  return hipErrorInvalidValue;
}

namespace {
template <typename E, int OP>
hipError_t launch_batch_t(const BatchSegDesc* segs, size_t count, hipStream_t st) {
  size_t i = 0;
  while (i < count) {  // up to kMaxBatch segments (and < 2^31 blocks) per launch
    BatchArgs args{};
    uint64_t blocks = 0;
    int k = 0;
    for (; i < count && k < kMaxBatch; i++) {
      const BatchSegDesc& d = segs[i];
      if (d.n == 0) continue;
      const Split sp = split_call<E>(d.c, d.n);
      const uint64_t tiles = std::max<uint64_t>(1, (sp.nvec + kBlock - 1) / kBlock);
      if (tiles > 0x7fffffffull) return hipErrorInvalidValue;  // > 2^39 elements: no such bucket
      if (blocks + tiles > 0x7fffffffull) break;  // next launch
      BatchSeg& g = args.s[k++];
      g.c = static_cast<char*>(d.c) + (size_t)sp.head * sizeof(E);
      g.a = static_cast<const char*>(d.a) + (size_t)sp.head * sizeof(E);
      g.b = static_cast<const char*>(d.b) + (size_t)sp.head * sizeof(E);
      g.nvec = sp.nvec;
      g.head = sp.head;
      g.tail = sp.tail;
      g.tile0 = (uint32_t)blocks;
      g.c_old = (Elem<E, OP>::kNeedsOld && d.c != d.a) ? 1u : 0u;
      blocks += tiles;
    }
    if (k == 0) continue;
    args.count = k;
    hipLaunchKernelGGL((k_reduce_batch<E, OP>), dim3((unsigned)blocks), dim3(kBlock), 0, st, args);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int OP>
hipError_t batch_dtype(int dtype, const BatchSegDesc* segs, size_t count, hipStream_t st) {
  switch (dtype) {
    case kI8: return launch_batch_t<int8_t, OP>(segs, count, st);
    case kU8: return launch_batch_t<uint8_t, OP>(segs, count, st);
    case kI32: return launch_batch_t<int32_t, OP>(segs, count, st);
    case kU32: return launch_batch_t<uint32_t, OP>(segs, count, st);
    case kI64: return launch_batch_t<int64_t, OP>(segs, count, st);
    case kU64: return launch_batch_t<uint64_t, OP>(segs, count, st);
    case kF32: return launch_batch_t<float, OP>(segs, count, st);
    case kF64: return launch_batch_t<double, OP>(segs, count, st);
    case kF16: return launch_batch_t<f16_t, OP>(segs, count, st);
    case kBF16: return launch_batch_t<bf16_t, OP>(segs, count, st);
  }
  return hipErrorInvalidValue;
}
}  // namespace

hipError_t launch_reduce_batch(int op, int dtype, const BatchSegDesc* segs, size_t count,
                               hipStream_t st) {
  switch (op) {
    case kSum: return batch_dtype<kSum>(dtype, segs, count, st);
    case kProduct: return batch_dtype<kProduct>(dtype, segs, count, st);
    case kMax: return batch_dtype<kMax>(dtype, segs, count, st);
    case kMin: return batch_dtype<kMin>(dtype, segs, count, st);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_acc_bf16_f32(float* acc, const void* b, size_t n, hipStream_t s) {
  size_t blocks = (n / 8 + kBlock - 1) / kBlock;
  const size_t cap = (size_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_acc_bf16, dim3((unsigned)blocks), dim3(kBlock), 0, s, acc,
                     reinterpret_cast<const uint16_t*>(b), n);
  return hipGetLastError();
}

hipError_t launch_f32_to_bf16(void* out, const float* acc, size_t n, hipStream_t s) {
  size_t blocks = (n + kBlock - 1) / kBlock;
  const size_t cap = (size_t)cu_count() * 16;
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(k_f32_to_bf16, dim3((unsigned)blocks), dim3(kBlock), 0, s,
                     reinterpret_cast<uint16_t*>(out), acc, n);
  return hipGetLastError();
}

}  // namespace hydra
