// allreduce.cpp -- host ring allreduce (new_allreduce_ring) and the two-rail split
// (bew_allreduce_a), behaviour of gloo/gloo/allreduce.cc:99-422 and pipeallreduce-a.{h,cc}.
//
// The per-segment reduction is whatever Func the caller set; in hydra it is the gfx950 kernel
// behind hydra_reduce_host (include/hydra/gloo_reduce.h).  The schedule, the segment geometry,
// the two-in-flight scratch and the fold order (c = local + received, in place) are the
// reference's, so results are bit-identical to gloo::allreduce with the same reduce function.

#include <cstring>
#include <thread>

#include "../../../include/hydra/allreduce.h"
#include "../bcube_geometry.h"
#include "../split_table.h"

namespace hydra {

namespace {

using BufVec = std::vector<std::unique_ptr<UnboundBuffer>>;
using RangeFn = std::function<void(size_t, size_t)>;

size_t round_up(size_t v, size_t m) {
  const size_t r = v % m;
  return r ? v + m - r : v;
}

constexpr uint8_t kAllreduceSlotPrefix = 0x04;  // gloo/gloo/types.h:60
uint64_t make_slot(uint32_t tag) {             // Slot::build (types.cc:15-19)
  return (uint64_t(kAllreduceSlotPrefix) << 56) | ((uint64_t(tag) & 0xffffffffu) << 24);
}

// Local pre-reduction of several inputs (or outputs) into out[0] for a byte range.
RangeFn local_reduce(const BufVec& in, const BufVec& out, size_t es,
                     const AllreduceOptions::Func& fn) {
  if (!in.empty()) {
    if (in.size() == 1)
      return [&in, &out](size_t off, size_t len) {
        std::memcpy(static_cast<char*>(out[0]->ptr) + off,
                    static_cast<const char*>(in[0]->ptr) + off, len);
      };
    return [&in, &out, es, fn](size_t off, size_t len) {
      char* o = static_cast<char*>(out[0]->ptr) + off;
      fn(o, static_cast<const char*>(in[0]->ptr) + off, static_cast<const char*>(in[1]->ptr) + off,
         len / es);
      for (size_t i = 2; i < in.size(); i++)
        fn(o, o, static_cast<const char*>(in[i]->ptr) + off, len / es);
    };
  }
  return [&out, es, fn](size_t off, size_t len) {
    char* o = static_cast<char*>(out[0]->ptr) + off;
    for (size_t i = 1; i < out.size(); i++)
      fn(o, o, static_cast<const char*>(out[i]->ptr) + off, len / es);
  };
}

RangeFn local_broadcast(const BufVec& out) {
  return [&out](size_t off, size_t len) {
    for (size_t i = 1; i < out.size(); i++)
      std::memcpy(static_cast<char*>(out[i]->ptr) + off,
                  static_cast<const char*>(out[0]->ptr) + off, len);
  };
}

struct SegRange {
  size_t send_off, recv_off;
  ssize_t send_len, recv_len;
};

void ring(const AllreduceOptions& o, const RangeFn& reduceInputs,
          const RangeFn& broadcastOutputs) {
  Context& ctx = *o.context;
  const BufVec& out = o.out;
  const uint64_t slot = make_slot(o.tag);
  const size_t total = o.elements * o.elementSize;
  const int P = ctx.size, r = ctx.rank;
  const int recvRank = (P + r + 1) % P, sendRank = (P + r - 1) % P;
  ctx.getPair(recvRank);
  ctx.getPair(sendRank);

  const size_t maxSegBytes = o.elementSize * std::max<size_t>(1, o.maxSegmentSize / o.elementSize);
  const size_t numSegments =
      round_up(std::max((total + maxSegBytes - 1) / maxSegBytes, (size_t)P * 2), (size_t)P);
  const size_t S = numSegments / P;
  const size_t segBytes = round_up((total + numSegments - 1) / numSegments, o.elementSize);

  // two segments in flight: scratch holds both (the context's cached, optionally pinned, slots)
  auto tmp = ctx.createUnboundBuffer(ctx.scratch(segBytes * 2), segBytes * 2);
  const size_t slotOff[2] = {0, segBytes};

  auto rs = [&](size_t i) {
    SegRange s;
    s.send_off = (((r + 1) * S + i) * segBytes) % (numSegments * segBytes);
    s.recv_off = (((r + 2) * S + i) * segBytes) % (numSegments * segBytes);
    s.send_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.send_off);
    s.recv_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.recv_off);
    return s;
  };
  const size_t iters = numSegments - S + 2;
  for (size_t i = 0; i < iters; i++) {
    if (i >= 2) {
      const SegRange prev = rs(i - 2);
      if (prev.recv_len > 0) {
        reduceInputs(prev.recv_off, prev.recv_len);
        tmp->waitRecv(o.timeout);
        char* dst = static_cast<char*>(out[0]->ptr) + prev.recv_off;
        o.reduce(dst, dst, static_cast<const char*>(tmp->ptr) + slotOff[i & 1],
                 prev.recv_len / o.elementSize);
      }
      if (prev.send_len > 0) out[0]->waitSend(o.timeout);
    }
    if (i < numSegments - S) {
      const SegRange cur = rs(i);
      if (cur.recv_len > 0) tmp->recv(recvRank, slot, slotOff[i & 1], cur.recv_len);
      if (cur.send_len > 0) {
        if (i < S) reduceInputs(cur.send_off, cur.send_len);
        out[0]->send(sendRank, slot, cur.send_off, cur.send_len);
      }
    }
  }

  auto ag = [&](size_t i) {
    SegRange s;
    s.send_off = (((r)*S + i) * segBytes) % (numSegments * segBytes);
    s.recv_off = (((r + 1) * S + i) * segBytes) % (numSegments * segBytes);
    s.send_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.send_off);
    s.recv_len = std::min((ssize_t)segBytes, (ssize_t)total - (ssize_t)s.recv_off);
    return s;
  };
  for (size_t i = 0; i < iters; i++) {
    if (i >= 2) {
      const SegRange prev = ag(i - 2);
      if (prev.recv_len > 0) {
        out[0]->waitRecv(o.timeout);
        broadcastOutputs(prev.recv_off, prev.recv_len);
      }
      if (prev.send_len > 0) out[0]->waitSend(o.timeout);
    }
    if (i < numSegments - S) {
      const SegRange cur = ag(i);
      if (cur.recv_len > 0) out[0]->recv(recvRank, slot, cur.recv_off, cur.recv_len);
      if (cur.send_len > 0) {
        out[0]->send(sendRank, slot, cur.send_off, cur.send_len);
        if (i < S) broadcastOutputs(cur.send_off, cur.send_len);
      }
    }
  }
}

// ---- BCUBE (allreduce.cc:423-700), geometry in bcube_geometry.h ------------------------------
void bcube(const AllreduceOptions& o, const RangeFn& reduceInputs,
           const RangeFn& broadcastOutputs) {
  Context& ctx = *o.context;
  const BufVec& out = o.out;
  const uint64_t slot = make_slot(o.tag);
  const size_t es = o.elementSize;
  const std::vector<BcubeStep> steps = bcube_steps(ctx.size, ctx.rank, o.elements);
  size_t scratchElems = o.elements;  // chunk lengths round up (:540-547)
  for (const auto& s : steps) scratchElems = std::max(scratchElems, s.g * s.chunk);
  auto tmp = ctx.createUnboundBuffer(ctx.scratch(scratchElems * es), scratchElems * es);
  char* const obase = static_cast<char*>(out[0]->ptr);
  const char* const tbase = static_cast<const char*>(tmp->ptr);

  for (size_t k = 0; k < steps.size(); k++) {  // reduce-scatter
    const BcubeStep& s = steps[k];
    int nrecv = 0, nsend = 0;
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      if (peer == ctx.rank || s.mlen == 0) continue;
      tmp->recv(peer, slot, i * s.chunk * es, s.mlen * es);
      nrecv++;
    }
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      if (peer == ctx.rank) continue;
      const size_t coff = s.off + i * s.chunk, clen = s.chunk_len(i);
      if (k == 0) reduceInputs(coff * es, clen * es);
      if (clen == 0) continue;
      out[0]->send(peer, slot, coff * es, clen * es);
      nsend++;
    }
    for (int i = 0; i < nrecv; i++) tmp->waitRecv(o.timeout);
    for (int i = 0; i < nsend; i++) out[0]->waitSend(o.timeout);
    if (k == 0) reduceInputs(s.moff * es, s.mlen * es);
    for (size_t i = 0; i < s.g && s.mlen; i++) {
      if ((int)(s.base + i * s.dist) == ctx.rank) continue;
      char* mine = obase + s.moff * es;
      o.reduce(mine, mine, tbase + i * s.chunk * es, s.mlen);
    }
  }
  broadcastOutputs(steps.back().moff * es, steps.back().mlen * es);

  for (auto it = steps.rbegin(); it != steps.rend(); ++it) {  // all-gather
    const BcubeStep& s = *it;
    int nrecv = 0, nsend = 0;
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      const size_t clen = s.chunk_len(i);
      if (peer == ctx.rank || clen == 0) continue;
      out[0]->recv(peer, slot, (s.off + i * s.chunk) * es, clen * es);
      nrecv++;
    }
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      if (peer == ctx.rank || s.mlen == 0) continue;
      out[0]->send(peer, slot, s.moff * es, s.mlen * es);
      nsend++;
    }
    for (int i = 0; i < nrecv; i++) out[0]->waitRecv(o.timeout);
    for (int i = 0; i < nsend; i++) out[0]->waitSend(o.timeout);
    for (size_t i = 0; i < s.g; i++) {
      if ((int)(s.base + i * s.dist) == ctx.rank) continue;
      broadcastOutputs((s.off + i * s.chunk) * es, s.chunk_len(i) * es);
    }
  }
}

}  // namespace

void allreduce(const AllreduceOptions& o) {
  if (o.out.empty()) throw EnforceNotMet("allreduce: no output buffer");
  if (o.elements == 0) throw EnforceNotMet("allreduce: elements == 0");
  if (o.elementSize == 0) throw EnforceNotMet("allreduce: elementSize == 0");
  if (!o.reduce) throw EnforceNotMet("allreduce: no reduce function");
  const size_t total = o.elements * o.elementSize;
  for (const auto& b : o.out)
    if (b->size != total) throw EnforceNotMet("allreduce: output size mismatch");
  for (const auto& b : o.in)
    if (b->size != total) throw EnforceNotMet("allreduce: input size mismatch");
  const RangeFn reduceInputs = local_reduce(o.in, o.out, o.elementSize, o.reduce);
  const RangeFn broadcastOutputs = local_broadcast(o.out);
  if (o.context->size == 1) {  // allreduce.cc:129-133
    reduceInputs(0, total);
    broadcastOutputs(0, total);
    return;
  }
  switch (o.algorithm) {
    case AllreduceOptions::UNSPECIFIED:
    case AllreduceOptions::RING:
      ring(o, reduceInputs, broadcastOutputs);
      break;
    case AllreduceOptions::BCUBE:
      bcube(o, reduceInputs, broadcastOutputs);
      break;
    default:
      throw EnforceNotMet("Algorithm not handled.");
  }
}

// ---- bew_allreduce_a split (pipeallreduce-a.h:137-376) --------------------------------------
void calculateElements(SplitTable t, int P, size_t n, size_t* e1, size_t* e2) {
  split_elements(t == SplitTable::AG ? 1 : 0, P, n, e1, e2);
}

void APipeAllreduceOptions::setSplit(char* p, size_t n, size_t es, bool input) {
  size_t e1, e2;
  calculateElements(table_, size_, n, &e1, &e2);
  char* p1 = p;
  char* p2 = p + e1 * es;
  opts3.elements = e1;
  opts2.elements = e2;
  auto set = [&](AllreduceOptions& o, char* q, size_t e) {
    void* ptr = q;
    if (input) o.setInputsRaw(&ptr, 1, e, es);
    else o.setOutputsRaw(&ptr, 1, e, es);
  };
  if (e2 == 0) set(opts3, p1, e1);
  else if (e1 == 0) set(opts2, p2, e2);
  else {
    set(opts3, p1, e1);
    set(opts2, p2, e2);
  }
}

void apipe_allreduce(APipeAllreduceOptions& o) {  // pipeallreduce-a.cc:27-61
  if (o.opts3.elements != 0 && o.opts2.elements != 0) {
    std::exception_ptr err1, err2;
    std::thread a([&] {
      try { allreduce(o.opts3); } catch (...) { err1 = std::current_exception(); }
    });
    std::thread b([&] {
      try { allreduce(o.opts2); } catch (...) { err2 = std::current_exception(); }
    });
    b.join();
    a.join();
    if (err1) std::rethrow_exception(err1);
    if (err2) std::rethrow_exception(err2);
  } else if (o.opts2.elements != 0) {
    allreduce(o.opts2);
  } else {
    allreduce(o.opts3);
  }
}

}  // namespace hydra
