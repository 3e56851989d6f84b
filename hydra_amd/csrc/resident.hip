// resident.hip -- the resident reducer's kernel (see resident.h for the protocol).
#include "resident.h"

#include <algorithm>
#include <type_traits>

#include "reduce_kernels.h"
#include "reduce_ops.h"

namespace hydra {
namespace {

// The device word workgroup 0 publishes a job in: the instance's generation tag in the top 16
// bits, the job's workgroup count in the next 12, the job number in the low 36.  The host zeroes
// the device record before every launch (resident_host.cpp ensure_running), so no word another
// instance left behind reaches this one's workers even when the 16-bit tag has wrapped; the tag
// is a second guard on top of that.  A worker learns
// from ONE load both which job is current and whether it takes part: it never pairs a job
// number with another job's record (a worker delayed between two loads once could).
constexpr int kTagShift = 48;
constexpr int kNwgShift = 36;
constexpr uint64_t kSeqMask = (uint64_t(1) << kNwgShift) - 1;
constexpr uint64_t kNwgMask = (uint64_t(1) << (kTagShift - kNwgShift)) - 1;
static_assert(kResidentMaxBlocks <= kNwgMask, "nwg fits its field");
__device__ __forceinline__ uint64_t pub_word(uint64_t tag, uint64_t nwg, uint64_t seq) {
  return (tag << kTagShift) | ((nwg & kNwgMask) << kNwgShift) | (seq & kSeqMask);
}
__device__ __forceinline__ uint64_t fin_word(uint64_t tag, uint64_t seq) {  // `finished`
  return pub_word(tag, 0, seq);
}

// The ragged head / tail of a segment, one element per lane (waves 0 and 1), with its tile 0.
template <typename E, int OP>
__device__ __forceinline__ void res_edges(const ResSeg& g, int t) {
  constexpr int N = Vec<E>::N;
  E* c_ = reinterpret_cast<E*>(g.c);
  const E* a_ = reinterpret_cast<const E*>(g.a);
  const E* b_ = reinterpret_cast<const E*>(g.b);
  const bool head = t < g.head, tail = t >= 64 && t - 64 < g.tail;
  if (head || tail) {
    const ptrdiff_t i = head ? (ptrdiff_t)t - g.head : (ptrdiff_t)(g.nvec * N) + (t - 64);
    const E ea = a_[i], eb = b_[i];
    const E ec = g.c_old ? c_[i] : ea;
    c_[i] = Elem<E, OP>::apply(ea, eb, ec);
  }
}

// Global-address-space 16-B accesses: the descriptor's pointers come from LDS, so plain
// dereferences compile to FLAT instructions, which count on lgkmcnt as well -- and every LDS
// read of the next tile's descriptor then waited for the previous tile's loads (round 4's kernel
// kept one tile in flight per wave).  Host-mapped and device operands are both global memory.
typedef __attribute__((address_space(1))) const u32x4_u* gld_t;
typedef __attribute__((address_space(1))) u32x4* gst_t;
__device__ __forceinline__ u32x4 ld_g(const char* p) { return *(gld_t)(p); }
__device__ __forceinline__ void st_g(char* p, u32x4 v) { *(gst_t)(p) = v; }

// This workgroup's tiles first, first + stride, ... of the call, B at a time: every tile's
// pointers first (the LDS descriptor reads), then all of the batch's loads, then the stores, so
// a workgroup with several tiles pays one PCIe round trip per batch rather than per tile (host
// operands are latency-bound).  The loads are unconditional -- a lane with nothing to do in a
// tile reads `dummy` (16 B of device memory) and stores nothing -- so no register merge at a
// branch join waits for them either.
template <int B, typename E, int OP>
__device__ __forceinline__ void res_run(const ResDesc& D, uint32_t first, uint32_t stride, int t,
                                        const char* dummy) {
  constexpr bool kF16 = std::is_same_v<E, f16_t>;  // only float16 reads c's old bits (c_old)
  for (uint32_t base = first; base < D.tiles; base += stride * B) {
    const char* pa[B];
    const char* pb[B];
    const char* pc[B];
    char* cp[B];
    bool old_c[B];
#pragma unroll
    for (int u = 0; u < B; u++) {
      pa[u] = pb[u] = pc[u] = dummy;
      cp[u] = nullptr;
      old_c[u] = false;
      const uint32_t tile = base + u * stride;
      if (tile < D.tiles) {
        int k = 0;  // the last segment whose first tile is <= this tile (uniform)
        for (int j = 1; j < D.count; j++)
          if (D.s[j].tile0 <= tile) k = j;
        const ResSeg& g = D.s[k];
        const uint32_t lt = tile - g.tile0;
        if (lt == 0 && (g.head | g.tail)) res_edges<E, OP>(g, t);
        const size_t v = (size_t)lt * kBlock + t;
        if (v < g.nvec) {
          const size_t o = v * 16;
          pa[u] = g.a + o;
          pb[u] = g.b + o;
          cp[u] = g.c + o;
          if (kF16 && g.c_old) {
            pc[u] = g.c + o;
            old_c[u] = true;
          }
        }
      }
    }
    u32x4 x[B], y[B], z[B];
#pragma unroll
    for (int u = 0; u < B; u++) {
      x[u] = ld_g(pa[u]);
      y[u] = ld_g(pb[u]);
      if constexpr (kF16) z[u] = ld_g(pc[u]);
    }
#pragma unroll
    for (int u = 0; u < B; u++) {
      // the float16 store quirk compares with c's old bits: c's own when c != a (c_old), else a's
      if (cp[u]) st_g(cp[u], vapply<E, OP>(x[u], y[u], (kF16 && old_c[u]) ? z[u] : x[u]));
    }
  }
}

template <int B, typename E>
__device__ __forceinline__ void res_op(const ResDesc& D, uint32_t first, uint32_t stride, int t,
                                       const char* dummy) {
  switch (D.op) {
    case kSum: res_run<B, E, kSum>(D, first, stride, t, dummy); break;
    case kProduct: res_run<B, E, kProduct>(D, first, stride, t, dummy); break;
    case kMax: res_run<B, E, kMax>(D, first, stride, t, dummy); break;
    case kMin: res_run<B, E, kMin>(D, first, stride, t, dummy); break;
  }
}

template <int B>
__device__ __forceinline__ void res_tiles(const ResDesc& D, uint32_t first, uint32_t stride,
                                          int t, const char* dummy) {
  switch (D.dtype) {
    case kI8: res_op<B, int8_t>(D, first, stride, t, dummy); break;
    case kU8: res_op<B, uint8_t>(D, first, stride, t, dummy); break;
    case kI32: res_op<B, int32_t>(D, first, stride, t, dummy); break;
    case kU32: res_op<B, uint32_t>(D, first, stride, t, dummy); break;
    case kI64: res_op<B, int64_t>(D, first, stride, t, dummy); break;
    case kU64: res_op<B, uint64_t>(D, first, stride, t, dummy); break;
    case kF32: res_op<B, float>(D, first, stride, t, dummy); break;
    case kF64: res_op<B, double>(D, first, stride, t, dummy); break;
    case kF16: res_op<B, f16_t>(D, first, stride, t, dummy); break;
    case kBF16: res_op<B, bf16_t>(D, first, stride, t, dummy); break;
  }
}

template <typename T>
__device__ __forceinline__ T ld_sys(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_agent(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kDescWords = (int)(sizeof(ResDesc) / 8);
static_assert(sizeof(ResDesc) % 8 == 0 && kDescWords <= 2 * 64, "descriptor copy: 2 words/lane");


// Workgroup 0 (wave 0) picks the next call: the first pending slot after the one served last.
__device__ __forceinline__ int pick_slot(uint64_t pending, int last) {
  const uint64_t after = pending & ~((uint64_t(2) << last) - 1);
  return (int)__builtin_ctzll(after ? after : pending);
}

// Bounded agent-scope wait for every workgroup to finish job `want` (workgroup 0 reuses the
// device job record only after that).  false: the wait expired (err set).
__device__ __forceinline__ bool wait_finished(ResCtl* h, ResDev* d, uint64_t want,
                                              uint64_t grace_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_agent(&d->finished) != want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > grace_ticks) {
      __hip_atomic_store(&h->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// B: tiles whose loads a workgroup issues together; a call of at most `solo` tiles is served by
// workgroup 0 alone (no device hop to the others, no arrival counter); a job wakes
// ceil(tiles / tpb) workgroups.
//
// Liveness: workgroup 0 bumps the device heartbeat `beat` on every call it serves (solo calls
// publish no job), and a worker restarts its grace period whenever the job word or the heartbeat
// moves.  A worker gives up (err) only when neither moved for idle + grace -- i.e. only if
// workgroup 0 itself is gone without publishing the exit, which a correct grid never does.
template <int B>
__global__ __launch_bounds__(kBlock) void k_resident(ResCtl* h, ResDev* d, uint64_t gen,
                                                     uint64_t idle_ticks, uint64_t grace_ticks,
                                                     uint32_t solo, uint32_t tpb) {
  __shared__ uint64_t s_seq;
  __shared__ int s_slot;
  __shared__ int s_mode;  // 0 a published job, 1 workgroup 0 alone, 2 leave, 3 not in this job
  __shared__ uint32_t s_nwg;  // workgroups in the published job
  __shared__ ResDesc s_desc;
  const int t = threadIdx.x;
  const uint64_t gtag = gen & ((uint64_t(1) << (64 - kTagShift)) - 1);
  // 16 readable bytes of device memory for the loads of lanes without an element (res_run)
  const char* dummy = reinterpret_cast<const char*>(&d->job);
  uint64_t job = 0;  // the last job published (workgroup 0) / seen (the others)
  uint64_t beat = 0;  // workgroup 0: calls served by this instance
  // workgroup 0, wave 0: lane i < kResidentSlots tracks slot i's last served sequence number
  uint64_t served = 0;
  int last_slot = kResidentSlots - 1;
  if (blockIdx.x == 0 && t < kResidentSlots) served = ld_sys(&h->slot[t].done);
  for (;;) {
    if (blockIdx.x == 0) {
      if (t < 64) {  // wave 0: every slot's doorbell and the quit word in one load instruction
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t s = 0;
        int k = 0, mode = 0;
        for (;;) {
          const uint64_t db = t < kResidentSlots ? ld_sys(&h->slot[t].doorbell)
                              : t == 63        ? (uint64_t)ld_sys(&h->quit)
                                               : 0;
          // quit first: a host that stops the instance (a drain, a timeout, exit) must not wait
          // behind other threads' calls; a call rung meanwhile is served by the next instance
          if (__shfl((unsigned long long)db, 63) != 0) {
            mode = 2;
            break;
          }
          const uint64_t pending = __ballot(t < kResidentSlots && db != served);
          if (pending) {
            k = pick_slot(pending, last_slot);
            s = __shfl((unsigned long long)db, k);
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            mode = 2;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (mode != 2) {
          if (t == k) served = s;
          last_slot = k;
          beat++;
          if (t == 0)  // liveness for the workers (solo calls publish nothing)
            __hip_atomic_store(&d->beat, beat, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          // the descriptor was written before the doorbell: acquire, then read it (two words
          // per lane, one host round trip)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          const uint64_t* src = reinterpret_cast<const uint64_t*>(&h->slot[k].desc);
          uint64_t w0 = 0, w1 = 0;
          if (t < kDescWords) w0 = src[t];
          if (t + 64 < kDescWords) w1 = src[t + 64];
          // word 1 holds {count, tiles}: a small call stays in this workgroup
          const uint32_t tiles = (uint32_t)(__shfl((unsigned long long)w0, 1) >> 32);
          if (tiles <= solo) {
            uint64_t* dst = reinterpret_cast<uint64_t*>(&s_desc);
            if (t < kDescWords) dst[t] = w0;
            if (t + 64 < kDescWords) dst[t + 64] = w1;
            mode = 1;
          } else if (job != 0 && !wait_finished(h, d, fin_word(gtag, job), grace_ticks)) {
            mode = 2;  // a workgroup never finished the last job: leave (err is set)
          } else {  // the job record, write-through, then publish it
            const uint32_t nwg = min(gridDim.x, max(2u, (tiles + tpb - 1) / tpb));
            if (t == 0) s_nwg = nwg;
            uint64_t* dst = reinterpret_cast<uint64_t*>(&d->job.desc);
            if (t < kDescWords)
              __hip_atomic_store(dst + t, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t + 64 < kDescWords)
              __hip_atomic_store(dst + t + 64, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t == 0) {
              __hip_atomic_store(&d->job.seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(&d->job.slot, (uint32_t)k, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
              __hip_atomic_store(&d->job.nwg, nwg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            job++;
            if (t == 0)
              __hip_atomic_store(&d->pub, pub_word(gtag, nwg, job), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
          }
        } else {
          // leave: once every workgroup finished the last job (so none is still to wake for
          // it), publish the exit
          if (job != 0) (void)wait_finished(h, d, fin_word(gtag, job), grace_ticks);
          if (t == 0)
            __hip_atomic_store(&d->exit_gen, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (t == 0) {
          s_seq = s;
          s_slot = k;
          s_mode = mode;
        }
      }
    } else if (t == 0) {  // the other workgroups: the job word workgroup 0 publishes
      uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t seen_beat = ld_agent(&d->beat);
      uint32_t nwg = 0;
      int mode = 0;
      for (;;) {
        const uint64_t p = ld_agent(&d->pub);
        if ((p >> kTagShift) == gtag && (p & kSeqMask) != job) {
          job = p & kSeqMask;
          nwg = (uint32_t)((p >> kNwgShift) & kNwgMask);  // from the same word: this job's
          break;
        }
        if (ld_agent(&d->exit_gen) == gen) {
          mode = 2;
          break;
        }
        const uint64_t b = ld_agent(&d->beat);
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (b != seen_beat) {  // workgroup 0 is serving (solo) calls: alive
          seen_beat = b;
          t0 = now;
        } else if (now - t0 > idle_ticks + grace_ticks) {
          __hip_atomic_store(&h->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          mode = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (mode == 0) {
        s_nwg = nwg;
        if (blockIdx.x >= nwg) mode = 3;  // not in this job: its record is never read
      }
      s_mode = mode;
    }
    if (t == 0 && s_mode != 3) {
      // the job record (device, agent) and the operands / staging the host wrote (system)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    const int mode = s_mode;
    if (mode == 2) break;
    if (mode == 3) {  // not needed for this job: wait for the next
      __syncthreads();
      continue;
    }
    if (mode == 1) {  // workgroup 0 alone: every tile here, then the slot's completion word
      // (<= solo tiles, B of them in flight at once: one PCIe round trip for a 4-tile call)
      res_tiles<B>(s_desc, 0, 1, t, dummy);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&h->slot[s_slot].done, s_seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();
      continue;
    }
    {  // a published job: its record into LDS
      const uint64_t* src = reinterpret_cast<const uint64_t*>(&d->job);
      uint64_t* dst = reinterpret_cast<uint64_t*>(&s_desc);
      constexpr int kHead = (int)(offsetof(ResJob, desc) / 8);
      for (int q = t; q < kDescWords; q += kBlock) dst[q] = ld_agent(src + kHead + q);
    }
    __syncthreads();
    // a published job: one tile at a time per wave -- its store then overlaps the next tile's
    // loads on the full-duplex link; batching B tiles' loads ahead of their stores measured
    // 2-9 % slower for jobs of 16 tiles and up (profiles/r05o_resident_batch_ab.json)
    res_tiles<1>(s_desc, blockIdx.x, s_nwg, t, dummy);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this workgroup's stores reach the host
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t old =
          __hip_atomic_fetch_add(&d->arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old == s_nwg - 1) {
        const uint64_t seq = ld_agent(&d->job.seq);
        const uint32_t slot = ld_agent(&d->job.slot);
        __hip_atomic_store(&d->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&d->finished, fin_word(gtag, job), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&h->slot[slot].done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();  // s_desc is rewritten next round
  }
  if (blockIdx.x == 0 && t == 0)
    __hip_atomic_store(&h->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t launch_resident(ResCtl* h, ResDev* d, uint64_t gen, uint64_t idle_ticks,
                           uint64_t grace_ticks, const ResidentShape& shape, hipStream_t s) {
  const uint32_t solo = shape.solo, tpb = std::max(1u, shape.tiles_per_block);
  if (shape.batch >= 4)
    hipLaunchKernelGGL(k_resident<4>, dim3(shape.blocks), dim3(kBlock), 0, s, h, d, gen,
                       idle_ticks, grace_ticks, solo, tpb);
  else if (shape.batch == 2)
    hipLaunchKernelGGL(k_resident<2>, dim3(shape.blocks), dim3(kBlock), 0, s, h, d, gen,
                       idle_ticks, grace_ticks, solo, tpb);
  else
    hipLaunchKernelGGL(k_resident<1>, dim3(shape.blocks), dim3(kBlock), 0, s, h, d, gen,
                       idle_ticks, grace_ticks, solo, tpb);
  return hipGetLastError();
}

}  // namespace hydra
