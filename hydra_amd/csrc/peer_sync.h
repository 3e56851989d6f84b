// peer_sync.h -- cross-process / cross-GPU workgroup barrier over peer-mapped flags (xGMI).
//
// Used by the peer-access allreduce (peer_kernels.hip): every rank's kernel has the same grid,
// and workgroup b of each rank synchronises only with workgroup b of every other rank, so no
// grid-wide barrier (and no co-residency requirement across workgroups) is needed.
//
// Memory model (LLVM AMDGPU, gfx950; MI355X_MICROARCH.md "inter-workgroup visibility"):
//   producer: the results a peer reads are stored system-coherent (sc0 sc1: written through
//             to memory, peer_fold.h est / vst) -> every storing wave `s_waitcnt vmcnt(0)` (the
//             stores are complete) -> workgroup barrier -> relaxed system-scope flag stores
//             into every rank's signal area.  (release = true adds a system-scope fence --
//             buffer_wbl2 sc0 sc1: this XCD's dirty L2 lines reach memory -- and a second
//             explicit wait before the flags: the form plain stores need, kept for the
//             measurement variants of the pre-round-6 kernels; a barrier that publishes no
//             store needs neither);
//   consumer: relaxed polls of its own (uncached) signal area -> system-scope acquire fence
//             (buffer_inv sc0 sc1: drops stale L1 / non-coherent L2 copies of peer lines) ->
//             `s_waitcnt vmcnt(0)` -> workgroup barrier -> plain loads.
// Failure: a wait that exceeds its timeout records a code in the rank's host-mapped error
// word and in every peer's `abort` word; every spin loop watches its own `abort`, so the whole
// group drains within one timeout and every later kernel on the group exits at once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hydra {

constexpr int kPeerMaxRanks = 8;  // one xGMI-connected node
constexpr int kPeerMaxBlocks = 1024;
// error codes in the host-mapped word: 1-3 = timeout at barrier 1-3 of a call on this rank,
// kPeerErrAborted = another rank gave up first
constexpr uint32_t kPeerErrAborted = 5;

struct PeerSignals {
  uint32_t flag[kPeerMaxBlocks][kPeerMaxRanks];  // flag[block][source rank] = last epoch seen
  uint32_t abort;                                // non-zero: some rank gave up (its code)
  // (push with dynamic slabs) this rank's slab tickets and finished workgroups of the running
  // call; the last workgroup out zeroes both for the next call
  uint32_t ticket, done;
};

struct PeerSigPtrs {
  PeerSignals* p[kPeerMaxRanks];  // rank q's signal area, mapped into this process
};

struct PeerSync {
  PeerSigPtrs sig;
  uint32_t* err;           // this rank's host-mapped error word
  uint64_t timeout_ticks;  // s_memrealtime ticks (100 MHz)
  int P, rank;
};

// s_memrealtime runs at a constant 100 MHz on gfx9
__device__ __forceinline__ uint64_t peer_clock() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint32_t peer_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void peer_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Is the group already broken?  (one lane.)  The own abort word alone answers it: every failure
// writes it -- peer_fail stores the code into every rank's abort word, this rank's included --
// and it is never cleared, so the host-mapped error word adds nothing but a read over PCIe,
// which 512 workgroups issuing at once at kernel entry cost ~20 us per call (profiles/r06w).
// (host = true: that read too -- the measurement variant of the kernel before r06w.)
__device__ __forceinline__ bool peer_aborted(const PeerSync& S, bool host = false) {
  return peer_ld(&S.sig.p[S.rank]->abort) != 0 || (host && peer_ld(S.err) != 0);
}

// Give up: record `code` here and tell every peer.
__device__ __forceinline__ void peer_fail(const PeerSync& S, uint32_t code) {
  peer_st(S.err, code);
  for (int q = 0; q < S.P; q++) peer_st(&S.sig.p[q]->abort, code);
}

// Epochs live on the device: workgroup b's next epoch is one past the value it last published
// for itself (flag[b][rank] of its own area, written only by it).  Workgroup b of every rank
// runs the same sequence of barriers, so the counters agree without any host bookkeeping --
// which is what makes a captured hipGraph replayable (kernel arguments never change).
__device__ __forceinline__ uint32_t peer_next_epoch(const PeerSync& S) {
  return peer_ld(&S.sig.p[S.rank]->flag[blockIdx.x][S.rank]) + 1u;
}

// Release this workgroup's finished stores and publish `epoch` as flag[blockIdx.x][rank] in
// every rank's signal area.  Call from all threads.
// (release = false: this workgroup has stored nothing a peer will read since the kernel
// started -- the start barrier, peer_fold.h kStartRelease)
__device__ __forceinline__ void peer_signal(const PeerSync& S, uint32_t epoch,
                                            bool release = true) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {  // wave 0
    if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if ((int)threadIdx.x < S.P) peer_st(&S.sig.p[threadIdx.x]->flag[blockIdx.x][S.rank], epoch);
  }
}

// Wait until every rank's workgroup blockIdx.x has published `epoch`, then acquire.  Returns
// false (group broken) on timeout or abort; every wave still leaves, so the grid drains.
__device__ __forceinline__ bool peer_wait(const PeerSync& S, uint32_t epoch, uint32_t code,
                                          bool sys_acquire = true) {
  int ok = 1;
  if (threadIdx.x < 64) {  // wave 0: lane q polls rank q's arrival
    const int q = threadIdx.x;
    const uint64_t t0 = peer_clock();
    uint32_t spins = 0;
    if (q < S.P) {
      const uint32_t* mine = &S.sig.p[S.rank]->flag[blockIdx.x][q];
      while ((int32_t)(peer_ld(mine) - epoch) < 0) {
        __builtin_amdgcn_s_sleep(2);
        if ((++spins & 63) == 0) {
          if (peer_aborted(S)) {
            if (peer_ld(S.err) == 0) peer_st(S.err, kPeerErrAborted);
            ok = 0;
            break;
          }
          if (peer_clock() - t0 > S.timeout_ticks) {
            peer_fail(S, code);
            ok = 0;
            break;
          }
        }
      }
    }
    if (sys_acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (measurement variant only)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  return __syncthreads_and(ok) != 0;
}

// Workgroup-level barrier with the same workgroup index on every rank.
// release / sys_acquire: see peer_signal / peer_wait (both true but in measurement variants)
__device__ __forceinline__ bool peer_barrier(const PeerSync& S, uint32_t code,
                                             bool release = true, bool sys_acquire = true) {
  __shared__ uint32_t epoch_s;
  if (threadIdx.x == 0) epoch_s = peer_next_epoch(S);
  __syncthreads();
  const uint32_t epoch = epoch_s;
  peer_signal(S, epoch, release);
  return peer_wait(S, epoch, code, sys_acquire);
}

}  // namespace hydra
