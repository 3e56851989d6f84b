// copy_pool.h -- host memcpy fan-out for hydra_reduce_host's staging.
//
// A pageable operand reaches the kernel only through the context's pinned staging, copied by
// the CPU (host_map.h: hydra never pins a caller's pageable range).  One core copies ~25 GB/s,
// so at the reference ring's 1 MiB segment the three copies (a and b in, c out) cost more than
// the GPU's PCIe pass.  copy_all() splits a list of copies into 64 KiB pieces and runs them on
// a small process-wide pool of helper threads plus the calling thread; copies under
// kFanoutMin bytes in total stay on the caller (waking a helper costs microseconds).
// HYDRA_COPY_THREADS sets the helper count (default 4; 0 = the caller copies alone).
#pragma once

#include <cstddef>

namespace hydra {

struct CopyJob {
  void* dst;
  const void* src;
  size_t bytes;
};

constexpr size_t kFanoutMin = 256u << 10;  // below this total, the caller copies alone
constexpr size_t kCopyPiece = 64u << 10;

// Copies every job (disjoint destinations); returns when all bytes are in place.  Thread-safe:
// concurrent callers (the two rails of bew_allreduce_a) share the helpers.
void copy_all(const CopyJob* jobs, size_t count);

}  // namespace hydra
