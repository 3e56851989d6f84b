// include/hydra/halving_doubling_geometry.h -- per-rank geometry of gloo's
// AllreduceHalvingDoubling<T> (gloo/gloo/allreduce_halving_doubling.h:37-222), shared by the
// host class (hydra::AllreduceHalvingDoubling<T>, allreduce.h) and the device plan
// (HYDRA_ALGO_HALVING_DOUBLING, hydra_amd/csrc/xgmi_plan.h) so both walk the same schedule.
// Header-only, no dependencies beyond the standard library.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace hydra {
namespace detail {

struct HalvingDoublingGeometry {
  struct Step {
    size_t send_off = 0, send_cnt = 0, recv_off = 0, recv_cnt = 0;
  };
  int block_off = 0, block = 0, rank_in_block = 0, smaller = 0, larger = 0;
  std::vector<Step> steps;         // one per step inside the block
  size_t piece_to_larger = 0;      // sendCountToLargerBlock_ (:195-196)
  size_t kept_off = 0, kept = 0;   // the chunk this rank owns after the block's halving

  static int ilog2(uint64_t x) { return x ? 63 - __builtin_clzll(x) : 0; }
  static uint32_t reverse_bits(uint32_t v, int nbits) {  // reverseLastNBits (:23-34)
    uint32_t r = 0;
    for (int b = 0; b < nbits; b++, v >>= 1) r = (r << 1) | (v & 1u);
    return r;
  }

  HalvingDoublingGeometry(int P, int rank, size_t count) {
    // Blocks are the set bits of P, the smallest at the top ranks (initBinaryBlocks, :39-64).
    int top = P, prev = 0;
    for (int bit = 1; top > 0; bit <<= 1) {
      if (!(P & bit)) continue;
      top -= bit;
      if (block) { larger = bit; break; }
      if (rank >= top) { block_off = top; block = bit; smaller = prev; }
      prev = bit;
    }
    rank_in_block = rank - block_off;
    const int total_steps = ilog2((uint64_t)P);
    const size_t chunk = (count + (size_t(1) << total_steps) - 1) >> total_steps;
    size_t span = total_steps ? chunk << (total_steps - 1) : 0, base = 0;
    for (int bit = 1; bit < block; bit <<= 1, span >>= 1) {  // :113-157
      Step s;
      s.send_off = base + ((rank ^ bit) & bit ? span : 0);
      s.recv_off = base + (rank & bit ? span : 0);
      s.send_cnt = s.send_off < count ? std::min(span, count - s.send_off) : 0;
      s.recv_cnt = s.recv_off < count ? std::min(span, count - s.recv_off) : 0;
      if (rank & bit) base += span;
      steps.push_back(s);
    }
    if (larger) piece_to_larger = span >> (ilog2((uint64_t)(larger / block)) - 1);
    kept_off = steps.empty() ? 0 : steps.back().recv_off;
    kept = steps.empty() ? count : steps.back().recv_cnt;
  }
  // Ranks of the next larger block this rank scatters its kept chunk to, piece by piece.
  int larger_peer(int piece) const {
    const int k = larger / block;
    const uint32_t ordinal = reverse_bits((uint32_t)rank_in_block, ilog2((uint64_t)block)) * k;
    return block_off - larger + (int)reverse_bits(ordinal + piece, ilog2((uint64_t)larger));
  }
  size_t piece_len(int piece) const {
    const size_t at = piece_to_larger * (size_t)piece;
    return at < kept ? std::min(piece_to_larger, kept - at) : 0;
  }
  int smaller_peer() const { return block_off + block + rank_in_block % smaller; }
  // Receive box for the halving steps and the smaller block's piece (elements).
  size_t inbox_elems() const {
    size_t m = smaller ? kept : 0;
    for (const auto& s : steps) m = std::max(m, s.recv_cnt);
    return m;
  }
};

}  // namespace detail
}  // namespace hydra
