// peer_kernels.h -- launcher of the peer-access (IPC over xGMI) bucket allreduce kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "peer_sync.h"

namespace hydra {

enum PeerAlgo { kPeerAuto = 0, kPeerTwoShot = 1, kPeerOneShot = 2, kPeerTwoShotPush = 3 };
constexpr size_t kPeerSlabBytes = 64 << 10;  // largest work unit: 64 KiB of one owner block
constexpr size_t kPeerMinSlabBytes = 4 << 10;

struct PeerLaunch {
  char* x[kPeerMaxRanks];        // rank q's bucket, mapped into this process (x[rank] = local)
  PeerSync sync;                 // signal areas, error word, timeout, P, rank
  size_t lo[kPeerMaxRanks + 1];  // owner block q = elements [lo[q], lo[q+1])
  size_t slab_bytes;             // work unit (multiple of 16 and of the element size)
  char* scratch;                 // ONE_SHOT: n elements of local staging
  uint64_t* stamps;              // (measurement build only) per-workgroup phase clocks, or null
};

hipError_t launch_peer(int algo, int op, int dtype, bool acc32, const PeerLaunch& A,
                       unsigned grid, hipStream_t s);
// *per_cu = workgroups of the kernel launch_peer would run that one CU holds at once
hipError_t peer_occupancy(int algo, int op, int dtype, bool acc32, int* per_cu);

// (measurement build) clocks per workgroup in PeerLaunch::stamps: s_memrealtime (100 MHz) at
// kernel entry, after barrier 1, at the end of phase 1 (fold), after barrier 2, at the end of
// phase 2 (copy), after barrier 3 (two-shot; one-shot: the last two equal the fourth)
constexpr int kPeerStamps = 6;

// one reduction op's kernels, every dtype (peer_kernels_<op>.hip; launch_peer dispatches);
// occ non-null: report the kernel's workgroups per CU instead of launching it
hipError_t launch_peer_sum(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                           hipStream_t s, int* occ);
hipError_t launch_peer_product(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                               hipStream_t s, int* occ);
hipError_t launch_peer_max(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                           hipStream_t s, int* occ);
hipError_t launch_peer_min(int algo, int dtype, bool acc32, const PeerLaunch& A, unsigned grid,
                           hipStream_t s, int* occ);

}  // namespace hydra
