// bcube_geometry.h -- the group walk of gloo's BCUBE allreduce (allreduce.cc:423-535), shared by
// the host runtime (bcube() over TCP) and the device plan (plan_bcube over RCCL).
//
// One step per factor of P (2s first, then the remainder, computeGroupSizePerStep :426-437).
// In step s, rank r and the ranks base + i*dist (i < g) share a buffer range; it is cut into g
// chunks of ceil(len/g) elements and r keeps chunk (r/dist) % g, folding the group's partials
// into it in place: own value first, then the peers in group order (:592-603).  The all-gather
// walks the steps backwards.  A group shares its range, so both ends of every transfer derive
// the same length (zero-length chunks can be skipped on both sides).
#pragma once

#include <algorithm>
#include <cstddef>
#include <vector>

namespace hydra {

struct BcubeStep {
  size_t dist, g, grank, base;  // group geometry
  size_t off, len, chunk;       // the group's range (elements) and chunk length
  size_t moff, mlen;            // this rank's chunk
  size_t chunk_len(size_t i) const { return len > i * chunk ? std::min(chunk, len - i * chunk) : 0; }
};

inline std::vector<BcubeStep> bcube_steps(int P, int r, size_t n) {
  std::vector<size_t> sizes;
  size_t left = (size_t)P;
  while (left % 2 == 0) {
    sizes.push_back(2);
    left /= 2;
  }
  if (left > 1) sizes.push_back(left);
  std::vector<BcubeStep> steps;
  size_t dist = 1, off = 0, len = n;
  for (size_t g : sizes) {
    BcubeStep s;
    s.dist = dist;
    s.g = g;
    s.grank = ((size_t)r / dist) % g;
    s.base = (size_t)r - s.grank * dist;
    s.off = off;
    s.len = len;
    s.chunk = (len + g - 1) / g;
    s.moff = off + s.grank * s.chunk;
    s.mlen = s.chunk_len(s.grank);
    steps.push_back(s);
    dist *= g;
    off = s.moff;
    len = s.mlen;
  }
  return steps;
}

}  // namespace hydra
