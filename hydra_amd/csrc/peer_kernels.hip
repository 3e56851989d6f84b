// peer_kernels.hip -- launcher of the gfx950 peer-access bucket allreduce (device code in
// peer_fold.h, compiled per op in peer_kernels_<op>.hip): the reduction reads the peers'
// buckets straight over xGMI (IPC-mapped HBM), so the sum IS the hop -- no RCCL proxy, no
// scratch landing zone, one kernel per allreduce.
//
// Ownership and fold order are the reference ring's (gloo/gloo/allreduce.cc:199-221, :253-258,
// :301-305): owner block q = segments [qS, (q+1)S) of the bucket, reduced as
// x_q + (x_{q+1} + (... + (x_{q-2} + x_{q-1}))), so every result is bit-identical to RING /
// DIRECT (xgmi_plan.h) and to the reference.
//
//   TWO_SHOT  phase 1: rank r folds ITS block r, pulling slab k of block r from all P buckets
//             (P-1 of them remote) and writing the result in place; phase 2: rank r pulls the
//             finished slabs of every other block q from their owners into its own bucket.
//             Link bytes per rank 2(P-1)/P * n * E, the same as the ring, spread over P-1 links.
//   ONE_SHOT  every rank folds the WHOLE bucket (each block in its owner's order) into local
//             scratch, then copies it back; (P-1) * n * E link bytes, 2 barriers -- for small
//             buckets, where the ring's 2(P-1) latencies dominate.
//
// Work unit: a slab (4-64 KiB, fixed per call from (P, n, dtype)) of one owner block.  Slab k of
// every block is handled by workgroup k mod G on every rank (G identical on every rank), so
// workgroup b only ever synchronises with workgroup b of the other ranks (peer_sync.h):
//   start barrier: every rank's bucket is ready (no release fence: nothing this kernel stored
//                  is published by it -- peer_fold.h kStartRelease);
//   phase 1 -> 2 barrier: workgroup b's phase-1 slabs are final on every rank;
//   end barrier (two-shot): nobody leaves while a peer may still read its bucket.
// Every wait is bounded (timeout -> error word + abort broadcast), so the grid always drains.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "peer_fold.h"

namespace hydra {
namespace {

#ifdef HYDRA_MEASURE
constexpr int kPeerVariantBase = 2000;  // hydra_set_variant 2001..2007: peer kernel A/B

// (measurement only) the f32-sum kernels with nontemporal loads / stores / deeper pipelining
hipError_t launch_variant(int v, int algo, const PeerLaunch& A, unsigned grid, hipStream_t s,
                          int* occ = nullptr) {
  switch (v) {
    case 1: return launch_t<float, kSum, false, 1>(algo, A, grid, s, occ);
    case 2: return launch_t<float, kSum, false, 2>(algo, A, grid, s, occ);
    case 3: return launch_t<float, kSum, false, 3>(algo, A, grid, s, occ);
    case 4: return launch_t<float, kSum, false, 4>(algo, A, grid, s, occ);
    case 5: return launch_t<float, kSum, false, 5>(algo, A, grid, s, occ);
    case 6: return launch_t<float, kSum, false, 6>(algo, A, grid, s, occ);
    case 7: return launch_t<float, kSum, false, 7>(algo, A, grid, s, occ);
    case 16: return launch_t<float, kSum, false, 16>(algo, A, grid, s, occ);
    case 32: return launch_t<float, kSum, false, 32>(algo, A, grid, s, occ);
    case 64: return launch_t<float, kSum, false, 64>(algo, A, grid, s, occ);
    case 128: return launch_t<float, kSum, false, 128>(algo, A, grid, s, occ);
    case 192: return launch_t<float, kSum, false, 192>(algo, A, grid, s, occ);
    case 256: return launch_t<float, kSum, false, 256>(algo, A, grid, s, occ);
    case 512: return launch_t<float, kSum, false, 512>(algo, A, grid, s, occ);
  }
  return hipErrorInvalidValue;
}
#endif  // HYDRA_MEASURE

}  // namespace

hipError_t launch_peer(int algo, int op, int dtype, bool acc32, const PeerLaunch& A,
                       unsigned grid, hipStream_t s) {
  if (A.sync.P < 1 || A.sync.P > kPeerMaxRanks || grid < 1 || grid > (unsigned)kPeerMaxBlocks ||
      A.slab_bytes < 16 || A.slab_bytes % 16)
    return hipErrorInvalidValue;
#ifdef HYDRA_MEASURE
  const int v = current_variant() - kPeerVariantBase;  // (measurement only)
  if (A.stamps) {  // hydra_measure_peer_stamps: the shipped kernel (or 32) plus phase clocks
    if (op != kSum || dtype != kF32 || acc32) return hipErrorInvalidValue;
    if (v == 32) return launch_t<float, kSum, false, 40>(algo, A, grid, s);
    if (v == 64) return launch_t<float, kSum, false, 72>(algo, A, grid, s);
    if (v == 128) return launch_t<float, kSum, false, 136>(algo, A, grid, s);
    if (v == 192) return launch_t<float, kSum, false, 200>(algo, A, grid, s);
    if (v == 256) return launch_t<float, kSum, false, 264>(algo, A, grid, s);
    if (v == 512) return launch_t<float, kSum, false, 520>(algo, A, grid, s);
    return launch_t<float, kSum, false, 8>(algo, A, grid, s);
  }
  if (((v >= 1 && v <= 7) || v == 16 || v == 32 || v == 64 || v == 128 || v == 192 || v == 256 || v == 512) && op == kSum && dtype == kF32 && !acc32)
    return launch_variant(v, algo, A, grid, s);
#endif
  switch (op) {  // one translation unit per op (peer_kernels_<op>.hip)
    case kSum: return launch_peer_sum(algo, dtype, acc32, A, grid, s, nullptr);
    case kProduct: return launch_peer_product(algo, dtype, acc32, A, grid, s, nullptr);
    case kMax: return launch_peer_max(algo, dtype, acc32, A, grid, s, nullptr);
    case kMin: return launch_peer_min(algo, dtype, acc32, A, grid, s, nullptr);
  }
  return hipErrorInvalidValue;
}

hipError_t peer_occupancy(int algo, int op, int dtype, bool acc32, int* per_cu) {
  const PeerLaunch A{};
#ifdef HYDRA_MEASURE  // a variant's own register count (the deeper ones hold fewer per CU)
  const int v = current_variant() - kPeerVariantBase;
  if (((v >= 1 && v <= 7) || v == 16 || v == 32 || v == 64 || v == 128 || v == 192 || v == 256 || v == 512) && op == kSum && dtype == kF32 && !acc32)
    return launch_variant(v, algo, A, 1, nullptr, per_cu);
#endif
  switch (op) {
    case kSum: return launch_peer_sum(algo, dtype, acc32, A, 1, nullptr, per_cu);
    case kProduct: return launch_peer_product(algo, dtype, acc32, A, 1, nullptr, per_cu);
    case kMax: return launch_peer_max(algo, dtype, acc32, A, 1, nullptr, per_cu);
    case kMin: return launch_peer_min(algo, dtype, acc32, A, 1, nullptr, per_cu);
  }
  return hipErrorInvalidValue;
}

}  // namespace hydra
