// peer_sync.h -- cross-process / cross-GPU workgroup barrier over peer-mapped flags (xGMI).
//
// Used by the peer-access allreduce (peer_kernels.hip): every rank's kernel has the same grid,
// and workgroup b of each rank synchronises only with workgroup b of every other rank, so no
// grid-wide barrier (and no co-residency requirement beyond one workgroup per rank) is needed.
//
// Memory model (LLVM AMDGPU, gfx950): the flag store is a system-scope release (buffer_wbl2 sc0
// sc1 + wait: this XCD's dirty L2 lines -- the block's phase results -- reach memory before the
// flag does); the waiter's system-scope acquire (buffer_inv sc0 sc1) drops stale copies of
// remote lines (peer HBM is cached non-coherently in the local L2) before the next phase reads
// them.  The flags live in uncached device memory shared by IPC.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hydra {

constexpr int kPeerMaxRanks = 8;  // one xGMI-connected node
constexpr int kPeerMaxBlocks = 1024;

struct PeerSignals {
  uint32_t flag[kPeerMaxBlocks][kPeerMaxRanks];  // flag[block][source rank] = last epoch seen
};

struct PeerSigPtrs {
  PeerSignals* p[kPeerMaxRanks];  // rank q's signal area, mapped into this process
};

// s_memrealtime runs at a constant 100 MHz on gfx9
__device__ __forceinline__ uint64_t peer_clock() { return __builtin_amdgcn_s_memrealtime(); }

// Workgroup-level barrier with the same workgroup index on every rank.  Returns false (and
// records `code` in *err, a host-mapped word) if a peer did not arrive within timeout_ticks;
// every wave still leaves the barrier, so the grid always drains.
__device__ __forceinline__ bool peer_barrier(const PeerSigPtrs& sig, int P, int rank,
                                             uint32_t epoch, uint64_t timeout_ticks,
                                             uint32_t* err, uint32_t code) {
  // Every wave waits for its own stores to be acknowledged by L2 (hipcc's __syncthreads does
  // not wait on vmcnt), so wave 0's buffer_wbl2 below writes back the whole block's results.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int t = threadIdx.x;
  int ok = 1;
  if (t < P) {
    __hip_atomic_store(&sig.p[t]->flag[blockIdx.x][rank], epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = &sig.p[rank]->flag[blockIdx.x][t];
    const uint64_t t0 = peer_clock();
    while ((int32_t)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                     epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (peer_clock() - t0 > timeout_ticks) {
        __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = 0;
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
  }
  return __syncthreads_and(ok) != 0;
}

}  // namespace hydra
