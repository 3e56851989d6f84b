// peer_kernels.h -- launcher of the peer-access (IPC over xGMI) bucket allreduce kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "peer_sync.h"

namespace hydra {

enum PeerAlgo { kPeerAuto = 0, kPeerTwoShot = 1, kPeerOneShot = 2 };
constexpr size_t kPeerSlabBytes = 64 << 10;  // work unit: 64 KiB of one owner block

struct PeerLaunch {
  char* x[kPeerMaxRanks];        // rank q's bucket, mapped into this process (x[rank] = local)
  PeerSigPtrs sig;               // rank q's signal area, mapped
  size_t lo[kPeerMaxRanks + 1];  // owner block q = elements [lo[q], lo[q+1])
  char* scratch;                 // ONE_SHOT: n elements of local staging
  uint32_t* err;                 // host-mapped error word (barrier timeouts)
  uint64_t timeout_ticks;        // 100 MHz s_memrealtime ticks
  uint32_t epoch;                // first epoch of this call (TWO_SHOT uses 3, ONE_SHOT 2)
  int P, rank;
};

hipError_t launch_peer(int algo, int op, int dtype, bool acc32, const PeerLaunch& A,
                       unsigned grid, hipStream_t s);

}  // namespace hydra
