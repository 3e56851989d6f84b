// reduce.cpp -- new-style reduce to a root (gloo/gloo/reduce.cc:21-262): the other new-style
// collective that calls the reduce function (reduce.cc:195), here with whatever Func the caller
// set -- in hydra the gfx950 kernel behind hydra_reduce_host (include/hydra/gloo_reduce.h).
//
// Behaviour kept from the reference, so results are bit-identical with the same reduce
// function (tests/test_host_ring.py, fixtures from the reference itself):
//   * its own segment geometry (reduce.cc:87-135), not the allreduce ring's: segmentBytes =
//     roundUp(min(ceil(B / 2P), maxSegmentSize rounded down to E), E), numSegments =
//     roundUp(max(ceil(B / segmentBytes), 2P), P);
//   * the ring reduce-scatter runs all numSegments iterations (reduce.cc:182-223), sending from
//     `in` for the first S segments and from `out` afterwards, and reducing out-of-place,
//     reduce(out + off, in + off, tmp + slot, n);
//   * then every non-root rank sends its chunk [rank * S * segmentBytes, +chunkBytes) to the
//     root (reduce.cc:229-261).  Only the root's output is defined.

#include <algorithm>
#include <cstring>

#include "../../../include/hydra/allreduce.h"

namespace hydra {

namespace {

constexpr uint8_t kReduceSlotPrefix = 0x03;  // gloo/gloo/types.h:59
uint64_t reduce_slot(uint32_t tag) {        // Slot::build (types.cc:15-19)
  return (uint64_t(kReduceSlotPrefix) << 56) | ((uint64_t(tag) & 0xffffffffu) << 24);
}

size_t round_up(size_t v, size_t m) {
  const size_t r = v % m;
  return r ? v + m - r : v;
}

}  // namespace

void reduce(ReduceOptions& o) {
  if (o.elements == 0) return;  // reduce.cc:22-24, before any check
  if (!o.context) throw EnforceNotMet("reduce: null context");
  Context& ctx = *o.context;
  if (o.elementSize == 0) throw EnforceNotMet("reduce: elementSize == 0");
  if (o.root < 0 || o.root >= ctx.size) throw EnforceNotMet("reduce: root out of range");
  if (!o.reduce) throw EnforceNotMet("reduce: no reduce function");
  if (!o.out) throw EnforceNotMet("reduce: no output buffer");
  const int P = ctx.size, r = ctx.rank;
  const int recvRank = (P + r + 1) % P, sendRank = (P + r - 1) % P;
  if (recvRank != r) ctx.getPair(recvRank);
  if (sendRank != r) ctx.getPair(sendRank);

  UnboundBuffer* out = o.out.get();
  UnboundBuffer* in = o.in ? o.in.get() : out;  // no input: the output is also the input
  const size_t total = o.elements * o.elementSize;
  if (in->size != total) throw EnforceNotMet("reduce: input size mismatch");
  if (out->size != total) throw EnforceNotMet("reduce: output size mismatch");

  if (P == 1) {
    if (in != out) std::memcpy(out->ptr, in->ptr, total);
    return;
  }

  const size_t es = o.elementSize;
  const size_t maxSegBytes = es * (o.maxSegmentSize / es);
  const size_t segBytes =
      round_up(std::min((total + (size_t)P * 2 - 1) / ((size_t)P * 2), maxSegBytes), es);
  if (segBytes == 0)  // the reference would divide by zero here
    throw EnforceNotMet("reduce: maxSegmentSize smaller than one element");
  const size_t numSegments =
      round_up(std::max((total + segBytes - 1) / segBytes, (size_t)P * 2), (size_t)P);
  const size_t S = numSegments / P;
  const size_t chunkBytes = S * segBytes;
  const uint64_t slot = reduce_slot(o.tag);

  auto tmp = ctx.createUnboundBuffer(ctx.scratch(segBytes * 2), segBytes * 2);
  const size_t slotOff[2] = {0, segBytes};
  struct Seg {
    size_t send_off, recv_off;
    ssize_t send_len, recv_len;
  };
  auto rs = [&](size_t i) {
    Seg s;
    s.send_off = (((r + 1) * S + i) * segBytes) % (numSegments * segBytes);
    s.recv_off = (((r + 2) * S + i) * segBytes) % (numSegments * segBytes);
    s.send_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.send_off);
    s.recv_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.recv_off);
    return s;
  };

  for (size_t i = 0; i < numSegments; i++) {
    if (i >= 2) {
      const Seg prev = rs(i - 2);
      if (prev.recv_len > 0) {
        tmp->waitRecv(o.timeout);
        o.reduce(static_cast<char*>(out->ptr) + prev.recv_off,
                 static_cast<const char*>(in->ptr) + prev.recv_off,
                 static_cast<const char*>(tmp->ptr) + slotOff[i & 1], prev.recv_len / es);
      }
      if (prev.send_len > 0) ((i - 2) < S ? in : out)->waitSend(o.timeout);
    }
    if (i + 2 < numSegments) {
      const Seg cur = rs(i);
      if (cur.recv_len > 0) tmp->recv(recvRank, slot, slotOff[i & 1], cur.recv_len);
      if (cur.send_len > 0) (i < S ? in : out)->send(sendRank, slot, cur.send_off, cur.send_len);
    }
  }

  // gather the owners' chunks to the root (reduce.cc:229-261)
  if (r == o.root) {
    size_t numRecv = 0;
    for (int q = 0; q < P; q++) {
      if (q == r) continue;
      const size_t off = (size_t)q * chunkBytes;
      const ssize_t len = std::min((ssize_t)chunkBytes, (ssize_t)total - (ssize_t)off);
      if (len > 0) {
        out->recv(q, slot, off, len);
        numRecv++;
      }
    }
    for (size_t i = 0; i < numRecv; i++) out->waitRecv(o.timeout);
  } else {
    const size_t off = (size_t)r * chunkBytes;
    const ssize_t len = std::min((ssize_t)chunkBytes, (ssize_t)total - (ssize_t)off);
    if (len > 0) {
      out->send(o.root, slot, off, len);
      out->waitSend(o.timeout);
    }
  }
}

}  // namespace hydra
