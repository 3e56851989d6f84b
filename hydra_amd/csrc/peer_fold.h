// peer_fold.h -- the peer-access allreduce's device code (fold, copy, the two schedules), as
// templates.  Included by the per-op translation units only (peer_kernels_{sum,product,max,
// min}.hip and, for the measurement variants, peer_kernels.hip): each compiles one reduction
// op's kernels, so the ~100 instantiations build in parallel instead of one 5-minute file.
// The schedules and their protocol are described in peer_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "errors.h"
#include "peer_kernels.h"
#include "peer_sync.h"
#include "reduce_kernels.h"
#include "reduce_ops.h"

namespace hydra {
namespace {

// Measurement variants (libhydra_measure.so only: hydra_set_variant 2001..2007 and the phase
// clocks of hydra_measure_peer_stamps, f32 sum; 0 = the shipped kernel): bit 0 nontemporal
// loads, bit 1 nontemporal stores, bit 2 twice the loads in flight, bit 3 phase clocks, bit 4
// the 1-3-source folds as deep as the others, bit 5 the push's slabs handed out by a ticket
// counter instead of k = b mod G, bit 6 barrier 1 WITH a release fence (the kernel before
// r06u), bit 7 barrier 1 with an agent-scope acquire, bit 8 the entry check reading the
// host-mapped error word too (the kernel before r06w), bit 9 plain stores and a release at
// every barrier after the first (the kernels before r06zc / r06zh).
template <int V>
__device__ __forceinline__ u32x4 pld(const char* p) {
  if constexpr ((V & 1) != 0) return ld<kNT>(p, rsrc<kNT>(nullptr, 0), 0);
  else return ld_u(p);
}
template <int V>
__device__ __forceinline__ void pst(char* p, u32x4 v) {
  if constexpr ((V & 2) != 0) st<kNT>(p, rsrc<kNT>(nullptr, 0), 0, v);
  else st_a(p, v);
}

// SYS: system-coherent stores (sc0 sc1: written through to memory, the line dropped from L2) --
// the push's, so its barrier 2 needs no L2 writeback before the flag: the stores are complete
// once `s_waitcnt vmcnt(0)` returns (profiles/r06zc: barrier 2 21 -> 11 us at P = 2, the push
// 11-30 % faster there, 2-10 % at P = 8).  The element form:
template <bool SYS, typename E>
__device__ __forceinline__ void est(E* p, E v) {
  if constexpr (SYS) {
    using U = std::conditional_t<sizeof(E) == 1, uint8_t,
              std::conditional_t<sizeof(E) == 2, uint16_t,
              std::conditional_t<sizeof(E) == 4, uint32_t, uint64_t>>>;
    U b;
    __builtin_memcpy(&b, &v, sizeof(E));
    __hip_atomic_store(reinterpret_cast<U*>(p), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    *p = v;
  }
}

// dst = fold of NP 16-B sources in the reference order: v[NP-1] innermost,
// acc = v[j] op acc for j = NP-2 .. 0 (c = local + received, in place on local).  NP is a
// compile-time count: with a runtime count every load sat behind a scalar branch, and the
// compiler waited for each load before issuing the next (one load in flight per wave).
template <typename E, int OP, bool ACC32, int NP>
__device__ __forceinline__ u32x4 fold_n(const u32x4 (&v)[NP]) {
  if constexpr (ACC32) {
    float a[8];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      a[2 * k] = bitsf(v[NP - 1][k] << 16);
      a[2 * k + 1] = bitsf(v[NP - 1][k] & 0xffff0000u);
    }
#pragma unroll
    for (int j = NP - 2; j >= 0; j--) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        a[2 * k] = fop<OP>(bitsf(v[j][k] << 16), a[2 * k]);
        a[2 * k + 1] = fop<OP>(bitsf(v[j][k] & 0xffff0000u), a[2 * k + 1]);
      }
    }
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; k++)
      o[k] = (uint32_t)f2bf(a[2 * k]) | ((uint32_t)f2bf(a[2 * k + 1]) << 16);
    return o;
  } else {
    u32x4 acc = v[NP - 1];
#pragma unroll
    for (int j = NP - 2; j >= 0; j--) acc = vapply<E, OP>(v[j], acc, v[j]);
    return acc;
  }
}

struct PeerSrcs {
  const char* p[kPeerMaxRanks];
};
struct PeerDsts {  // where a folded slab is stored: the local bucket, and (push) every peer's
  char* p[kPeerMaxRanks];
};

// one element, same order as fold_n (static source indices: no scratch spills)
template <typename E, int OP, bool ACC32>
__device__ __forceinline__ E fold_one(const PeerSrcs& S, int nsrc, size_t i) {
  if constexpr (ACC32) {
    float a = 0.f;
#pragma unroll
    for (int j = kPeerMaxRanks - 1; j >= 0; j--) {
      if (j < nsrc) {
        const float x = bf2f(reinterpret_cast<const uint16_t*>(S.p[j])[i]);
        a = (j == nsrc - 1) ? x : fop<OP>(x, a);
      }
    }
    E r;
    const uint16_t h = f2bf(a);
    __builtin_memcpy(&r, &h, 2);
    return r;
  } else {
    E acc = reinterpret_cast<const E*>(S.p[0])[i];
#pragma unroll
    for (int j = kPeerMaxRanks - 1; j >= 0; j--) {
      if (j < nsrc) {
        const E x = reinterpret_cast<const E*>(S.p[j])[i];
        acc = (j == nsrc - 1) ? x : Elem<E, OP>::apply(x, acc, x);
      }
    }
    return acc;
  }
}

// One workgroup folds `count` elements: D.p[d][i] = fold(S.p[0][i], ..., S.p[NP-1][i]) for each
// of the ND destinations (1: in place on the local bucket; NP: push -- the same result stored
// into every rank's bucket).  Aligned on D.p[0] (16 B; push requires every destination at the
// same alignment, checked by the launcher); sources may sit at any element alignment (gfx950
// unaligned mode).
// The main loop issues PU x NP unpredicated 16-B loads per lane before its first store (15-32
// in flight: the grid is small -- every workgroup pays barriers -- so the depth has to come from
// each wave; round 5's A/B on one GPU, profiles/r05k_*: twice the r05j depth was as fast or
// faster at every size >= 16 Mi); the last partial round is predicated.
template <typename E, int OP, bool ACC32, int V, int NP, int ND, bool SYS>
__device__ __forceinline__ void slab_fold_n(const PeerDsts& D, const PeerSrcs& S, size_t count) {
  // (1-byte elements: half the depth -- their per-byte max / min unpack needs the registers)
  // (V & 16: the small-NP cases as deep as NP >= 4's 32 vectors -- free in registers, which the
  // NP = 8 case sets for the whole kernel)
  constexpr int PU = ((V & 4) ? 2 : 1) * (NP >= 4 ? 4 : ((V & 16) ? 32 : 16) / NP) /
                     (sizeof(E) == 1 ? 2 : 1);
  constexpr int N = Vec<E>::N;
  const int t = threadIdx.x;
  size_t head = ((16 - (reinterpret_cast<uintptr_t>(D.p[0]) & 15)) & 15) / sizeof(E);
  if (head > count) head = count;
  const size_t nvec = (count - head) / N;
  const size_t tail = count - head - nvec * N;
  if ((size_t)t < head) {
    const E v = fold_one<E, OP, ACC32>(S, NP, t);
#pragma unroll
    for (int d = 0; d < ND; d++) est<SYS>(reinterpret_cast<E*>(D.p[d]) + t, v);
  }
  if ((size_t)t < tail) {
    const size_t i = head + nvec * N + t;
    const E v = fold_one<E, OP, ACC32>(S, NP, i);
#pragma unroll
    for (int d = 0; d < ND; d++) est<SYS>(reinterpret_cast<E*>(D.p[d]) + i, v);
  }
  const char* src[NP];
#pragma unroll
  for (int j = 0; j < NP; j++) src[j] = S.p[j] + head * sizeof(E);
  char* out[ND];
#pragma unroll
  for (int d = 0; d < ND; d++) out[d] = D.p[d] + head * sizeof(E);
  // (SYS) buffer stores with sc0 sc1 (aux 17), one resource per destination
  __amdgpu_buffer_rsrc_t R[ND];
#pragma unroll
  for (int d = 0; d < ND; d++)
    R[d] = SYS ? __builtin_amdgcn_make_buffer_rsrc(out[d], 0, (int)(nvec * 16), 0x00020000)
               : __builtin_amdgcn_make_buffer_rsrc(nullptr, 0, 0, 0);
  auto vst = [&](int d, size_t vi, u32x4 o) {
    if constexpr (SYS)
      __builtin_amdgcn_raw_buffer_store_b128(o, R[d], (uint32_t)(vi * 16), 0, 17);
    else
      pst<V>(out[d] + vi * 16, o);
  };
  constexpr size_t kStep = (size_t)kBlock * PU;
  const size_t full = nvec / kStep * kStep;
  for (size_t v0 = 0; v0 < full; v0 += kStep) {
    u32x4 r[PU][NP];
#pragma unroll
    for (int u = 0; u < PU; u++) {
      const size_t o = (v0 + (size_t)u * kBlock + t) * 16;
#pragma unroll
      for (int j = 0; j < NP; j++) r[u][j] = pld<V>(src[j] + o);
    }
#pragma unroll
    for (int u = 0; u < PU; u++) {
      const u32x4 o = fold_n<E, OP, ACC32, NP>(r[u]);
#pragma unroll
      for (int d = 0; d < ND; d++) vst(d, v0 + (size_t)u * kBlock + t, o);
    }
  }
  for (size_t v = full + t; v < nvec; v += kBlock) {  // the last partial round
    u32x4 r[NP];
#pragma unroll
    for (int j = 0; j < NP; j++) r[j] = pld<V>(src[j] + v * 16);
    const u32x4 o = fold_n<E, OP, ACC32, NP>(r);
#pragma unroll
    for (int d = 0; d < ND; d++) vst(d, v, o);
  }
}

// PUSH: every source is also a destination (the result is stored into all P buckets)
// SYS: system-coherent stores (est / vst above) -- for results a peer reads (push, and the
// pull's phase 1)
template <typename E, int OP, bool ACC32, int V = 0, bool PUSH = false, bool SYS = PUSH>
__device__ __forceinline__ void slab_fold(const PeerDsts& D, const PeerSrcs& S, int nsrc,
                                          size_t count) {
  switch (nsrc) {  // uniform over the grid: one branch per slab, none in the loop
#define HYDRA_SLAB_FOLD_CASE(k) \
  case k: slab_fold_n<E, OP, ACC32, V, k, PUSH ? k : 1, SYS && (V & 512) == 0>(D, S, count); break;
    HYDRA_SLAB_FOLD_CASE(1)
    HYDRA_SLAB_FOLD_CASE(2)
    HYDRA_SLAB_FOLD_CASE(3)
    HYDRA_SLAB_FOLD_CASE(4)
    HYDRA_SLAB_FOLD_CASE(5)
    HYDRA_SLAB_FOLD_CASE(6)
    HYDRA_SLAB_FOLD_CASE(7)
    HYDRA_SLAB_FOLD_CASE(8)
#undef HYDRA_SLAB_FOLD_CASE
  }
}

// One workgroup copies `count` elements src -> dst (phase 2 / copy-back): raw 16-B vectors,
// kCU of them per lane in flight (one source only, so deeper than the fold's kPU).
constexpr int kCU = 16;
template <typename E, int V = 0>
__device__ __forceinline__ void slab_copy(char* dst, const char* src, size_t count) {
  constexpr int CU = (V & 4) ? 2 * kCU : kCU;
  constexpr int N = Vec<E>::N;
  const int t = threadIdx.x;
  size_t head = ((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15) / sizeof(E);
  if (head > count) head = count;
  const size_t nvec = (count - head) / N;
  const size_t tail = count - head - nvec * N;
  E* de = reinterpret_cast<E*>(dst);
  const E* se = reinterpret_cast<const E*>(src);
  if ((size_t)t < head) de[t] = se[t];
  if ((size_t)t < tail) de[head + nvec * N + t] = se[head + nvec * N + t];
  const size_t base = head * sizeof(E);
  for (size_t v0 = 0; v0 < nvec; v0 += (size_t)kBlock * CU) {
    u32x4 r[CU];
#pragma unroll
    for (int u = 0; u < CU; u++) {
      const size_t v = v0 + (size_t)u * kBlock + t;
      if (v < nvec) r[u] = pld<V>(src + base + v * 16);
    }
#pragma unroll
    for (int u = 0; u < CU; u++) {
      const size_t v = v0 + (size_t)u * kBlock + t;
      if (v < nvec) pst<V>(dst + base + v * 16, r[u]);
    }
  }
}

// Barrier 1 (every rank's bucket is ready) publishes nothing this kernel wrote: the buckets
// were produced before the kernel started, by stream-ordered work whose completion already put
// them in memory (a kernel's end-of-kernel release writes its XCD L2s back -- the L2s of one
// GPU are not coherent with each other, so that writeback is what makes any kernel's output
// readable by the next kernel's other XCDs, and by a peer GPU reading this HBM over xGMI; a
// copy engine writes memory directly).  So its signal carries no release fence: 512 workgroups
// each writing their XCD's L2 back cost 13 us of the 36 us barrier at P = 2 (profiles/r06u).
// The acquire stays (a peer's bucket may sit stale in this GPU's caches).  Barriers 2 and 3
// publish this kernel's stores and keep the release.
template <int V>
constexpr bool kStartRelease = (V & 64) != 0;

// The group already failed (an earlier timeout here or on a peer): leave at once.
template <int V>
__device__ __forceinline__ bool group_broken(const PeerSync& S) {
  int bad = 0;
  if (threadIdx.x == 0 && peer_aborted(S, (V & 256) != 0)) {
    if (peer_ld(S.err) == 0) peer_st(S.err, kPeerErrAborted);
    bad = 1;
  }
  return __syncthreads_or(bad) != 0;
}

// (V & 8) workgroup's phase clock k (kPeerStamps per workgroup), after its own stores are done
template <int V>
__device__ __forceinline__ void stamp(const PeerLaunch& A, int k) {
  if constexpr ((V & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) A.stamps[(size_t)blockIdx.x * kPeerStamps + k] = peer_clock();
  }
}

template <typename E, int OP, bool ACC32, int V = 0>
__global__ __launch_bounds__(kBlock) void k_peer_two_shot(PeerLaunch A) {
  const size_t SL = A.slab_bytes / sizeof(E);
  const PeerSync& Y = A.sync;
  const int P = Y.P, r = Y.rank;
  const uint32_t G = gridDim.x;
  stamp<V>(A, 0);
  if (group_broken<V>(Y)) return;
  if (!peer_barrier(Y, 1, kStartRelease<V>, (V & 128) == 0)) return;  // every bucket is ready
  stamp<V>(A, 1);
  PeerSrcs S;
  // phase 1: own block r, slabs k = b, b+G, ...; all P sources, in place
  {
    const size_t lo = A.lo[r], hi = A.lo[r + 1];
    for (size_t k = blockIdx.x; lo + k * SL < hi; k += G) {
      const size_t s = lo + k * SL;
      PeerDsts D;
      D.p[0] = A.x[r] + s * sizeof(E);
#pragma unroll
      for (int j = 0; j < kPeerMaxRanks; j++)
        if (j < P) S.p[j] = A.x[(r + j) % P] + s * sizeof(E);
      slab_fold<E, OP, ACC32, V, false, true>(D, S, P, hi - s < SL ? hi - s : SL);
    }
  }
  // workgroup b of every rank has finished ITS slabs (k = b mod G) of its own block (stored
  // system-coherent: no L2 writeback before the flag)
  stamp<V>(A, 2);
  if (!peer_barrier(Y, 2, (V & 512) != 0)) return;
  stamp<V>(A, 3);
  // phase 2: the same slab indices of every other block, pulled from their owners; the start
  // peer rotates with b so the workgroups of one rank read from all P-1 links at once
  for (int i = 0; i < P - 1; i++) {
    const int q = (r + 1 + (int)((blockIdx.x + i) % (uint32_t)(P - 1))) % P;
    const size_t lo = A.lo[q], hi = A.lo[q + 1];
    for (size_t k = blockIdx.x; lo + k * SL < hi; k += G) {
      const size_t s = lo + k * SL;
      slab_copy<E, V>(A.x[r] + s * sizeof(E), A.x[q] + s * sizeof(E), hi - s < SL ? hi - s : SL);
    }
  }
  // nobody leaves (and lets its caller overwrite the bucket) while a peer may still read it
  stamp<V>(A, 4);
  peer_barrier(Y, 3, (V & 512) != 0);  // publishes no store (its own bucket only): no release
  stamp<V>(A, 5);
}

// TWO_SHOT_PUSH: rank r folds its own block r pulling slab k from all P buckets (as TWO_SHOT's
// phase 1) and stores the result into EVERY rank's bucket -- in place locally, over xGMI into
// the P-1 peers' -- so TWO_SHOT's phase 2 (pulling the other blocks back) and its barrier are
// gone: per rank n E read and n E written instead of (3P-1)/P n E, link bytes unchanged
// (2(P-1)/P n E: (P-1)/P n read, (P-1)/P n written).  Safe without more synchronisation: block
// r of any bucket is read only by rank r (its fold), and each slab is read and then written by
// the same workgroup; a peer's push into my bucket touches only ITS block.  Barrier 2: every
// peer's workgroup b has pushed its slabs k = b mod G into my bucket and read my slabs of its
// block -- after it my bucket is final and nobody reads it.
template <typename E, int OP, bool ACC32, int V = 0>
__global__ __launch_bounds__(kBlock) void k_peer_push(PeerLaunch A) {
  const size_t SL = A.slab_bytes / sizeof(E);
  const PeerSync& Y = A.sync;
  const int P = Y.P, r = Y.rank;
  const uint32_t G = gridDim.x;
  stamp<V>(A, 0);
  if (group_broken<V>(Y)) return;
  if (!peer_barrier(Y, 1, kStartRelease<V>, (V & 128) == 0)) return;  // every bucket is ready
  stamp<V>(A, 1);
  const size_t lo = A.lo[r], hi = A.lo[r + 1];
  auto fold_slab = [&](size_t k) {
    const size_t s = lo + k * SL;
    PeerSrcs S;
    PeerDsts D;
#pragma unroll
    for (int j = 0; j < kPeerMaxRanks; j++)
      if (j < P) {
        S.p[j] = A.x[(r + j) % P] + s * sizeof(E);
        D.p[j] = A.x[(r + j) % P] + s * sizeof(E);  // D.p[0]: the local bucket
      }
    slab_fold<E, OP, ACC32, V, true>(D, S, P, hi - s < SL ? hi - s : SL);
  };
  if constexpr ((V & 32) != 0) {
    // Dynamic slabs: workgroup b takes slab b, then tickets G, G+1, ... from this rank's
    // counter (drawn one slab ahead, so the atomic's round trip hides behind the fold), so a
    // slow workgroup takes fewer slabs.  Barrier 2 stays per workgroup index: a rank's kernel
    // ends only when every workgroup of it has met workgroup b of every peer there, i.e. after
    // every peer workgroup finished whatever slabs it took.
    __shared__ uint32_t next_s;
    PeerSignals* own = Y.sig.p[r];
    const size_t nsl = (hi - lo + SL - 1) / SL;
    for (size_t k = blockIdx.x; k < nsl;) {
      uint32_t nk = 0;
      if (threadIdx.x == 0)
        nk = G + __hip_atomic_fetch_add(&own->ticket, 1u, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM);
      fold_slab(k);
      if (threadIdx.x == 0) next_s = nk;
      __syncthreads();
      k = next_s;
      __syncthreads();
    }
    if (threadIdx.x == 0 &&  // the last workgroup out: every ticket of this call is drawn
        __hip_atomic_fetch_add(&own->done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ==
            G - 1) {
      __hip_atomic_store(&own->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&own->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  } else {
    for (size_t k = blockIdx.x; lo + k * SL < hi; k += G) fold_slab(k);
  }
  stamp<V>(A, 2);
  peer_barrier(Y, 2, (V & 512) != 0);  // no L2 writeback: the stores were system-coherent
  stamp<V>(A, 3);
  stamp<V>(A, 4);
  stamp<V>(A, 5);
}

template <typename E, int OP, bool ACC32, int V = 0>
__global__ __launch_bounds__(kBlock) void k_peer_one_shot(PeerLaunch A) {
  const size_t SL = A.slab_bytes / sizeof(E);
  const PeerSync& Y = A.sync;
  const int P = Y.P, r = Y.rank;
  const uint32_t G = gridDim.x;
  stamp<V>(A, 0);
  if (group_broken<V>(Y)) return;
  if (!peer_barrier(Y, 1, kStartRelease<V>, (V & 128) == 0)) return;
  stamp<V>(A, 1);
  PeerSrcs S;
  // slab list over all owner blocks: (q, k) enumerated block by block; slab w -> workgroup w%G
  size_t w = 0;
  for (int q = 0; q < P; q++) {
    const size_t lo = A.lo[q], hi = A.lo[q + 1];
    const size_t nsl = (hi - lo + SL - 1) / SL;
    for (size_t k = 0; k < nsl; k++, w++) {
      if (w % G != blockIdx.x) continue;
      const size_t s = lo + k * SL;
      PeerDsts D;
      D.p[0] = A.scratch + s * sizeof(E);
#pragma unroll
      for (int j = 0; j < kPeerMaxRanks; j++)
        if (j < P) S.p[j] = A.x[(q + j) % P] + s * sizeof(E);
      slab_fold<E, OP, ACC32, V>(D, S, P, hi - s < SL ? hi - s : SL);
    }
  }
  // every rank's workgroup b has read its slabs of every bucket -> safe to overwrite ours.  It
  // publishes no store (the scratch slabs are copied back by the workgroup that wrote them):
  // no release
  stamp<V>(A, 2);
  if (!peer_barrier(Y, 2, (V & 512) != 0)) return;
  stamp<V>(A, 3);
  w = 0;
  for (int q = 0; q < P; q++) {
    const size_t lo = A.lo[q], hi = A.lo[q + 1];
    const size_t nsl = (hi - lo + SL - 1) / SL;
    for (size_t k = 0; k < nsl; k++, w++) {
      if (w % G != blockIdx.x) continue;
      const size_t s = lo + k * SL;
      slab_copy<E, V>(A.x[r] + s * sizeof(E), A.scratch + s * sizeof(E), hi - s < SL ? hi - s : SL);
    }
  }
  stamp<V>(A, 4);
  stamp<V>(A, 5);
}

template <typename E, int OP, bool ACC32, int V = 0>
hipError_t launch_t(int algo, const PeerLaunch& A, unsigned grid, hipStream_t s,
                    int* occ = nullptr) {
  if (occ)  // workgroups per CU of the kernel this call would launch
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(
        occ,
        algo == kPeerOneShot ? reinterpret_cast<const void*>(&k_peer_one_shot<E, OP, ACC32, V>)
        : algo == kPeerTwoShotPush ? reinterpret_cast<const void*>(&k_peer_push<E, OP, ACC32, V>)
                                   : reinterpret_cast<const void*>(&k_peer_two_shot<E, OP, ACC32, V>),
        kBlock, 0);
  if (algo == kPeerOneShot)
    hipLaunchKernelGGL((k_peer_one_shot<E, OP, ACC32, V>), dim3(grid), dim3(kBlock), 0, s, A);
  else if (algo == kPeerTwoShotPush)
    hipLaunchKernelGGL((k_peer_push<E, OP, ACC32, V>), dim3(grid), dim3(kBlock), 0, s, A);
  else
    hipLaunchKernelGGL((k_peer_two_shot<E, OP, ACC32, V>), dim3(grid), dim3(kBlock), 0, s, A);
  return hipGetLastError();
}

// every dtype of one op (the per-op translation units' whole content)
template <int OP>
hipError_t dispatch(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                    hipStream_t s, int* occ) {
  if (acc32) {
    if (dtype != kBF16) return hipErrorInvalidValue;
    return launch_t<bf16_t, OP, true>(algo, A, grid, s, occ);
  }
  switch (dtype) {
    case kI8: return launch_t<int8_t, OP, false>(algo, A, grid, s, occ);
    case kU8: return launch_t<uint8_t, OP, false>(algo, A, grid, s, occ);
    case kI32: return launch_t<int32_t, OP, false>(algo, A, grid, s, occ);
    case kU32: return launch_t<uint32_t, OP, false>(algo, A, grid, s, occ);
    case kI64: return launch_t<int64_t, OP, false>(algo, A, grid, s, occ);
    case kU64: return launch_t<uint64_t, OP, false>(algo, A, grid, s, occ);
    case kF32: return launch_t<float, OP, false>(algo, A, grid, s, occ);
    case kF64: return launch_t<double, OP, false>(algo, A, grid, s, occ);
    case kF16: return launch_t<f16_t, OP, false>(algo, A, grid, s, occ);
    case kBF16: return launch_t<bf16_t, OP, false>(algo, A, grid, s, occ);
  }
  return hipErrorInvalidValue;
}

}  // namespace
}  // namespace hydra
