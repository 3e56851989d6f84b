// xgmi_plan.h -- data-only schedules of the multi-GPU bucket allreduce.
//
// A plan is the op list ONE rank executes.  Executors interpret it: the RCCL executor
// (xgmi_allreduce.cpp) maps SEND/RECV/GROUP onto ncclSend/ncclRecv/ncclGroup* on a comm stream
// and REDUCE/FOLD onto the HIP kernels on a compute stream; the one-GPU simulator runs every
// rank's plan in lock-step with device copies standing in for xGMI; tests/ interpret plans on
// the CPU with numpy.  All three see exactly the same schedule.
//
// Block ownership and fold order are the reference's (gloo/gloo/allreduce.cc:147-422):
//   numSegments / segmentBytes / S from allreduce.cc:199-221 (hydra_ring_plan), block q =
//   segments [qS, (q+1)S) clipped to the bucket, owned by rank q; its reduced value is
//   x_q + (x_{q+1} + (... + (x_{q-2} + x_{q-1})))   (indices mod P).
//
// Algorithms
//   RING   the reference's schedule on device: reduce-scatter hop s (s = 0..P-2) sends block
//          (r+1+s) to r-1 and receives block (r+2+s) from r+1, folding c = local + received
//          with the HIP sum (allreduce.cc:284-344); all-gather hop s sends block (r+s) to r-1,
//          receives block (r+1+s) from r+1 (:385-421).  Blocks are cut into chunks so hop s of
//          chunk c overlaps the sum of chunk c-1.  Uses one xGMI link per direction.
//   DIRECT MI355X-first: the node is fully connected (7 xGMI links per GPU), so every rank
//          sends each owner its block in ONE p2p group (all links busy), and the owner folds the
//          P contributions in the reference's order in ONE kernel (FOLD), then sends its block to
//          every peer (direct all-gather).  Same per-element arithmetic as RING, so bit-exact.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "bcube_geometry.h"
#include "hydra/halving_doubling_geometry.h"

namespace hydra {

enum PlanKind : int32_t {
  kOpSend = 1,    // send `bytes` from buffer `buf` at `off` to `peer`
  kOpRecv = 2,    // receive `bytes` from `peer` into buffer `buf` at `off`
  kOpGroup = 3,   // end of a p2p group: every SEND/RECV since the previous GROUP is one group
  kOpReduce = 4,  // user[off .. +bytes] = op(user[off..], scratch[src_off..])          (ring hop)
  kOpFold = 5,    // user[off..] = fold(user[off..], contributions in scratch, see slot_of)
  kOpAllToAll = 6,   // collective: user[off + q*bytes, bytes] -> rank q's scratch[src_off + r*bytes]
  kOpAllGather = 7,  // collective, in place: user[off + r*bytes, bytes] -> every rank's same range
};
enum PlanBuf : int32_t { kBufUser = 0, kBufScratch = 1 };
enum Algo : int32_t {
  kAlgoAuto = 0, kAlgoRing = 1, kAlgoDirect = 2, kAlgoRccl = 3, kAlgoA2A = 4, kAlgoRingOld = 5,
  kAlgoRingChunked = 6, kAlgoBcube = 7, kAlgoHalvingDoubling = 8,
  kAlgoReduce = 64  // internal: gloo::reduce to PlanGeom::root (hydra_reduce_root), not an allreduce
};

// AllreduceRingChunked<T> geometry (allreduce_ring_chunked.h:32-36): 2P chunks of
// max(256, ceil(n / 2P)) elements; trailing chunks may be short or empty.
inline size_t chunked_ring_elems(int P, size_t n) {
  const size_t chunks = 2 * (size_t)P;
  return std::max<size_t>(256, (n + chunks - 1) / chunks);
}

// Mirrored by hydra_plan_op_t in include/hydra_xgmi.h (same layout).
struct PlanOp {
  int32_t kind;
  int32_t peer;         // SEND/RECV: peer rank; FOLD: -1 = slots in contributor order
                        // (slot j-1 holds rank r+j), >= 0 = slots in rank order rotated by peer
  int32_t buf;
  int32_t nsrc;         // FOLD: number of contributions incl. the local one
  int64_t off;          // user/scratch byte offset (SEND/RECV: in `buf`; REDUCE/FOLD: user dst)
  int64_t bytes;
  int64_t src_off;      // REDUCE/FOLD: scratch byte offset of the (first) received operand
  int64_t slot_stride;  // FOLD: bytes between consecutive contributions in scratch
  int32_t wait0;        // indices of earlier ops this op must wait for (cross-stream), -1 none
  int32_t wait1;
};

struct PlanGeom {
  int P = 1;
  size_t n = 0, esize = 4, total = 0;
  size_t num_segments = 0, segment_bytes = 0, S = 0;
  size_t chunk = 0;  // pipelining chunk (bytes, multiple of esize and 16)
  int root = -1;     // kAlgoReduce: the rank that ends with the reduction
  size_t block_begin(int q) const { return std::min(total, (size_t)q * S * segment_bytes); }
  size_t block_end(int q) const { return std::min(total, (size_t)(q + 1) * S * segment_bytes); }
  size_t block_bytes(int q) const { return block_end(q) - block_begin(q); }
  size_t max_block() const {
    size_t m = 0;
    for (int q = 0; q < P; q++) m = std::max(m, block_bytes(q));
    return m;
  }
  size_t nchunks() const {  // chunks of the largest block (every block uses this count)
    const size_t mb = max_block();
    return mb ? (mb + chunk - 1) / chunk : 0;
  }
  // chunk c of block q: [begin, begin+len) relative to the bucket; len may be 0
  void chunk_of(int q, size_t c, size_t* begin, size_t* len) const {
    const size_t b = block_begin(q), e = block_end(q);
    const size_t lo = std::min(e, b + c * chunk), hi = std::min(e, lo + chunk);
    *begin = lo;
    *len = hi - lo;
  }
};

inline size_t round_up_sz(size_t v, size_t m) {
  const size_t r = v % m;
  return r ? v + m - r : v;
}

// allreduce.cc:199-221
inline void ring_geometry(int P, size_t n, size_t esize, size_t max_segment, size_t* ns,
                          size_t* sb, size_t* S) {
  const size_t total = n * esize;
  const size_t max_seg_bytes = esize * std::max<size_t>(1, max_segment / esize);
  *ns = round_up_sz(std::max((total + max_seg_bytes - 1) / max_seg_bytes, (size_t)P * 2),
                    (size_t)P);
  *S = *ns / (size_t)P;
  *sb = round_up_sz((total + *ns - 1) / *ns, esize);
}

// gloo::reduce's own geometry (reduce.cc:87-135): segmentBytes = roundUp(min(ceil(B / 2P),
// maxSegmentSize rounded down to E), E); numSegments = roundUp(max(ceil(B / segmentBytes), 2P), P).
// *sb == 0 when max_segment < esize (the reference would divide by zero).
inline void reduce_geometry(int P, size_t n, size_t esize, size_t max_segment, size_t* ns,
                            size_t* sb, size_t* S) {
  const size_t total = n * esize;
  const size_t max_seg_bytes = esize * (max_segment / esize);
  *sb = round_up_sz(std::min((total + (size_t)P * 2 - 1) / ((size_t)P * 2), max_seg_bytes), esize);
  *ns = *sb ? round_up_sz(std::max((total + *sb - 1) / *sb, (size_t)P * 2), (size_t)P) : 0;
  *S = *ns / (size_t)P;
}

// Pipelining chunk when the caller passes 0.  16 MiB keeps the host's enqueue of a DIRECT
// allreduce of BASELINE config 4 (P = 8, 64 Mi fp32: 62 plan ops, ~0.19 ms) well under its
// ~0.9 ms of xGMI time; 4 MiB (248 ops, ~0.82 ms of ncclSend/ncclRecv calls) sat at the
// CPU-bound edge (scripts/executor_overhead.py).
constexpr size_t kDefaultChunk = 16u << 20;

inline PlanGeom make_geom(int P, size_t n, size_t esize, size_t max_segment, size_t chunk) {
  PlanGeom g;
  g.P = P;
  g.n = n;
  g.esize = esize;
  g.total = n * esize;
  ring_geometry(P, n, esize, max_segment ? max_segment : (1u << 20), &g.num_segments,
                &g.segment_bytes, &g.S);
  const size_t unit = 16;  // every element size (1, 2, 4, 8) divides 16
  g.chunk = round_up_sz(std::max<size_t>(chunk ? chunk : kDefaultChunk, unit), unit);
  // never pipeline in chunks larger than a block (small buckets keep a small scratch)
  g.chunk = std::min(g.chunk, round_up_sz(std::max<size_t>(g.max_block(), 1), unit));
  return g;
}

inline PlanGeom make_geom_reduce(int P, size_t n, size_t esize, size_t max_segment,
                                 size_t chunk, int root) {
  PlanGeom g = make_geom(P, n, esize, max_segment, chunk);
  reduce_geometry(P, n, esize, max_segment ? max_segment : (1u << 20), &g.num_segments,
                  &g.segment_bytes, &g.S);
  const size_t unit = 16;
  g.chunk = round_up_sz(std::max<size_t>(chunk ? chunk : kDefaultChunk, unit), unit);
  g.chunk = std::min(g.chunk, round_up_sz(std::max<size_t>(g.max_block(), 1), unit));
  g.root = root;
  return g;
}

// Byte offset in scratch of contribution j (1..nsrc-1) of a FOLD op.
inline int64_t fold_slot(const PlanOp& o, int j) {
  if (o.peer < 0) return o.src_off + (int64_t)(j - 1) * o.slot_stride;
  return o.src_off + (int64_t)((o.peer + j) % o.nsrc) * o.slot_stride;
}

// A2A needs the reference's blocks to be equal and to tile the bucket (true for every
// BASELINE bucket: 64 Mi fp32 / 256 Mi bf16 at P = 2..8).
inline bool blocks_equal(const PlanGeom& g) {
  const size_t b = g.block_bytes(0);
  if (b == 0 || (size_t)g.P * b != g.total) return false;
  for (int q = 1; q < g.P; q++)
    if (g.block_bytes(q) != b) return false;
  return true;
}

// Scratch bytes one rank needs for `algo` (wire element size = esize).
inline size_t plan_scratch_bytes(int algo, const PlanGeom& g) {
  if (g.P <= 1) return 0;
  if (algo == kAlgoRing) return 2 * g.chunk;
  if (algo == kAlgoDirect || algo == kAlgoReduce) return 2 * (size_t)(g.P - 1) * g.chunk;
  if (algo == kAlgoA2A) return g.total;
  if (algo == kAlgoRingOld) return 2 * round_up_sz(g.total, 16);
  if (algo == kAlgoRingChunked) return 2 * round_up_sz(chunked_ring_elems(g.P, g.n) * g.esize, 16);
  if (algo == kAlgoHalvingDoubling) {  // the largest halving receive: step 0's half
    const int steps = detail::HalvingDoublingGeometry::ilog2((uint64_t)g.P);
    const size_t chunk = (g.n + (size_t(1) << steps) - 1) >> steps;
    return round_up_sz((chunk << (steps - 1)) * g.esize, 16);
  }
  if (algo == kAlgoBcube) {  // allreduce.cc:540-547: chunk lengths round up
    size_t e = g.n;
    for (const auto& s : bcube_steps(g.P, 0, g.n)) e = std::max(e, s.g * s.chunk);
    return round_up_sz(e * g.esize, 16);
  }
  return 0;
}

class PlanBuilder {
 public:
  std::vector<PlanOp> ops;
  int add(int32_t kind, int32_t peer, int32_t buf, int64_t off, int64_t bytes, int64_t src_off = 0,
          int64_t slot_stride = 0, int32_t nsrc = 0, int32_t w0 = -1, int32_t w1 = -1) {
    PlanOp o{kind, peer, buf, nsrc, off, bytes, src_off, slot_stride, w0, w1};
    ops.push_back(o);
    return (int)ops.size() - 1;
  }
};

// ---- RING ----------------------------------------------------------------------------------
inline std::vector<PlanOp> plan_ring(const PlanGeom& g, int r) {
  PlanBuilder pb;
  const int P = g.P;
  if (P <= 1 || g.total == 0) return pb.ops;
  const int send_to = (r + P - 1) % P, recv_from = (r + 1) % P;
  const size_t C = g.nchunks();
  // last compute op that wrote chunk c of any block (the block sent next hop), per chunk
  std::vector<int> wrote(C, -1);
  int reader[2] = {-1, -1};  // last REDUCE that read scratch slot 0/1
  size_t k = 0;              // global chunk counter (scratch slot = k & 1)
  for (int s = 0; s < P - 1; s++) {
    const int sq = (r + 1 + s) % P, rq = (r + 2 + s) % P;
    for (size_t c = 0; c < C; c++, k++) {
      size_t sb, sl, rb, rl;
      g.chunk_of(sq, c, &sb, &sl);
      g.chunk_of(rq, c, &rb, &rl);
      const int slot = (int)(k & 1);
      const int64_t soff = (int64_t)slot * (int64_t)g.chunk;
      if (sl == 0 && rl == 0) continue;
      if (sl) pb.add(kOpSend, send_to, kBufUser, sb, sl);
      if (rl) pb.add(kOpRecv, recv_from, kBufScratch, soff, rl);
      // the group sends a chunk the previous hop reduced, and overwrites a scratch slot that an
      // earlier REDUCE read: wait for both
      const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, s > 0 ? wrote[c] : -1,
                             reader[slot]);
      if (rl) {
        const int red = pb.add(kOpReduce, -1, kBufUser, rb, rl, soff, 0, 2, grp);
        wrote[c] = red;
        reader[slot] = red;
      } else {
        wrote[c] = -1;
      }
    }
  }
  // all-gather: pure copies on the comm stream; hop 0 sends the block this rank just folded
  for (int s = 0; s < P - 1; s++) {
    const int sq = (r + s) % P, rq = (r + 1 + s) % P;
    for (size_t c = 0; c < C; c++) {
      size_t sb, sl, rb, rl;
      g.chunk_of(sq, c, &sb, &sl);
      g.chunk_of(rq, c, &rb, &rl);
      if (sl == 0 && rl == 0) continue;
      if (sl) pb.add(kOpSend, send_to, kBufUser, sb, sl);
      if (rl) pb.add(kOpRecv, recv_from, kBufUser, rb, rl);
      pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, s == 0 ? wrote[c] : -1);
    }
  }
  return pb.ops;
}

// ---- DIRECT --------------------------------------------------------------------------------
// Scratch layout per chunk parity p: slot j (j = 1..P-1) at (p*(P-1) + (j-1)) * chunk holds the
// contribution of rank (r+j)%P to this rank's block, so FOLD reads them in the reference's order.
inline std::vector<PlanOp> plan_direct(const PlanGeom& g, int r) {
  PlanBuilder pb;
  const int P = g.P;
  if (P <= 1 || g.total == 0) return pb.ops;
  const size_t C = g.nchunks();
  int reader[2] = {-1, -1};
  std::vector<int> folded(C, -1);
  for (size_t c = 0; c < C; c++) {
    const int par = (int)(c & 1);
    const int64_t base = (int64_t)par * (P - 1) * (int64_t)g.chunk;
    bool any = false;
    // send my contribution to every other owner q (it lands in q's slot j = (r - q) mod P)
    for (int d = 1; d < P; d++) {
      const int q = (r + d) % P;
      size_t b, l;
      g.chunk_of(q, c, &b, &l);
      if (l) { pb.add(kOpSend, q, kBufUser, b, l); any = true; }
    }
    size_t mb, ml;
    g.chunk_of(r, c, &mb, &ml);
    if (ml) {
      for (int j = 1; j < P; j++) {
        const int p = (r + j) % P;
        pb.add(kOpRecv, p, kBufScratch, base + (int64_t)(j - 1) * (int64_t)g.chunk, ml);
        any = true;
      }
    }
    if (!any) continue;
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, reader[par]);
    if (ml) {
      const int f = pb.add(kOpFold, -1, kBufUser, mb, ml, base, (int64_t)g.chunk, P, grp);
      reader[par] = f;
      folded[c] = f;
    }
  }
  // direct all-gather, per chunk, as soon as that chunk is folded
  for (size_t c = 0; c < C; c++) {
    bool any = false;
    size_t mb, ml;
    g.chunk_of(r, c, &mb, &ml);
    if (ml)
      for (int d = 1; d < P; d++) { pb.add(kOpSend, (r + d) % P, kBufUser, mb, ml); any = true; }
    for (int d = 1; d < P; d++) {
      const int q = (r + d) % P;
      size_t b, l;
      g.chunk_of(q, c, &b, &l);
      if (l) { pb.add(kOpRecv, q, kBufUser, b, l); any = true; }
    }
    if (any) pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, folded[c]);
  }
  return pb.ops;
}

// ---- A2A -----------------------------------------------------------------------------------
// Equal blocks of B bytes: the reduce-scatter exchange IS an all-to-all (block q of every rank
// to rank q, landing in rank order), the owner folds the P contributions in the reference order
// (FOLD with rank-ordered slots rotated by r), and the all-gather is RCCL's in-place all-gather.
// Three launches per allreduce; RCCL picks the link schedule for both collectives.
inline std::vector<PlanOp> plan_a2a(const PlanGeom& g, int r) {
  PlanBuilder pb;
  if (g.P <= 1 || g.total == 0) return pb.ops;
  const int64_t B = (int64_t)g.block_bytes(0);
  const int x = pb.add(kOpAllToAll, -1, kBufUser, 0, B, 0);
  const int f = pb.add(kOpFold, r, kBufUser, (int64_t)r * B, B, 0, B, g.P, x);
  pb.add(kOpAllGather, -1, kBufUser, 0, B, 0, 0, 0, f);
  return pb.ops;
}

// ---- RING_OLD: old-style gloo::AllreduceRing<T> (allreduce_ring.h:71-106) -------------------
// P-1 rounds over the WHOLE bucket: round k sends rank+1 what this rank received in round k-1
// (round 0: its own bucket), receives rank-1's into scratch slot k%2 and folds it in place
// (x = x op inbox).  Rank r ends with x_r op x_{r-1} op ... op x_{r-P+1} -- its own order, as
// in the reference.  Chunked so round k of chunk c overlaps the fold of chunk c-1.
inline std::vector<PlanOp> plan_ring_old(const PlanGeom& g, int r) {
  PlanBuilder pb;
  const int P = g.P;
  if (P <= 1 || g.total == 0) return pb.ops;
  const int right = (r + 1) % P, left = (r + P - 1) % P;
  const int64_t slot_bytes = (int64_t)round_up_sz(g.total, 16);
  const size_t C = (g.total + g.chunk - 1) / g.chunk;
  std::vector<int> reader[2] = {std::vector<int>(C, -1), std::vector<int>(C, -1)};
  for (int k = 0; k < P - 1; k++) {
    const int in_slot = k & 1;
    for (size_t c = 0; c < C; c++) {
      const int64_t off = (int64_t)(c * g.chunk);
      const int64_t len = (int64_t)std::min(g.chunk, g.total - c * g.chunk);
      if (k == 0) pb.add(kOpSend, right, kBufUser, off, len);
      else pb.add(kOpSend, right, kBufScratch, (int64_t)((k - 1) & 1) * slot_bytes + off, len);
      pb.add(kOpRecv, left, kBufScratch, (int64_t)in_slot * slot_bytes + off, len);
      const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, reader[in_slot][c]);
      reader[in_slot][c] =
          pb.add(kOpReduce, -1, kBufUser, off, len, (int64_t)in_slot * slot_bytes + off, 0, 2,
                 grp);
    }
  }
  return pb.ops;
}

// ---- RING_CHUNKED: gloo::AllreduceRingChunked<T> (allreduce_ring_chunked.h:77-200) ---------
// 2P chunks; rank r starts chunks 2r and 2r+1 and each later round i (a uniform index over the
// reduce pass, rounds 2..2P-1, then the broadcast pass, rounds 0..2P-3) receives chunk
// co(i) from rank-1, folds it (x = x op inbox) or -- in the broadcast pass -- takes it, and
// forwards it to rank+1.  Send i and receive i form group i; rank r's send i is rank r+1's
// receive i, so every group is one ring step.  Chunk c, started by s = c/2, ends as
// x_{s-1} op (x_{s-2} op (... op (x_{s+1} op x_s))) on every rank, as in the reference.
// Empty chunks move nothing on either side (the reference's 1-element placeholder send,
// :218-225, carries no data the receiver uses).
inline int chunked_ring_chunk(int r, int P, int i) {
  const int C = 2 * P;
  const int round = i < C - 2 ? i + 2 : i - (C - 2);
  return ((2 * r) - (round & ~1) + (round & 1) + C) % C;
}

inline std::vector<PlanOp> plan_ring_chunked(const PlanGeom& g, int r) {
  PlanBuilder pb;
  const int P = g.P;
  if (P <= 1 || g.total == 0) return pb.ops;
  const int C = 2 * P, right = (r + 1) % P, left = (r + P - 1) % P;
  const size_t ce = chunked_ring_elems(P, g.n);
  const int64_t slot_bytes = (int64_t)round_up_sz(ce * g.esize, 16);
  auto span = [&](int co, int64_t* off, int64_t* len) {
    const size_t o = (size_t)co * ce;
    const size_t l = o >= g.n ? 0 : std::min(ce, g.n - o);
    *off = (int64_t)(o * g.esize);
    *len = (int64_t)(l * g.esize);
  };
  const int nsteps = 2 * C - 4;              // sends == receives == 4P-4
  std::vector<int> compute(nsteps, -1);      // REDUCE issued at step i (reduce pass only)
  std::vector<int> wrote(C, -1);             // last REDUCE that wrote user chunk c
  for (int i = 0; i < nsteps; i++) {
    // send i: the prelude chunks 2r, 2r+1, then what step i-2 produced
    const int sco = i < 2 ? 2 * r + i : chunked_ring_chunk(r, P, i - 2);
    const int rco = chunked_ring_chunk(r, P, i);
    const bool reduce_pass = i < C - 2;
    int64_t so, sl, ro, rl;
    span(sco, &so, &sl);
    span(rco, &ro, &rl);
    const int w0 = i >= 2 ? compute[i - 2] : -1;  // produced the sent chunk / read this slot
    const int w1 = reduce_pass ? -1 : wrote[rco];  // broadcast receives land in the user chunk
    if (sl == 0 && rl == 0) continue;
    if (sl) pb.add(kOpSend, right, kBufUser, so, sl);
    const int64_t slot_off = (int64_t)(i & 1) * slot_bytes;
    if (rl) {
      if (reduce_pass) pb.add(kOpRecv, left, kBufScratch, slot_off, rl);
      else pb.add(kOpRecv, left, kBufUser, ro, rl);
    }
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, w0, w1);
    if (reduce_pass && rl) {
      compute[i] = pb.add(kOpReduce, -1, kBufUser, ro, rl, slot_off, 0, 2, grp);
      wrote[rco] = compute[i];
    }
  }
  return pb.ops;
}

// ---- BCUBE: gloo's hypercube allreduce (allreduce.cc:423-700) on device ----------------------
// Per step one p2p group with every group peer (its chunk out of the user bucket, their
// partials of this rank's chunk into scratch slot i), then REDUCEs folding the partials into
// the chunk in group order, own value first -- the reference's order, so results are its bits.
// The all-gather walks the steps backwards, receiving straight into the user bucket.
inline std::vector<PlanOp> plan_bcube(const PlanGeom& g, int r) {
  PlanBuilder pb;
  if (g.P <= 1 || g.n == 0) return pb.ops;
  const int64_t es = (int64_t)g.esize;
  const std::vector<BcubeStep> steps = bcube_steps(g.P, r, g.n);
  int last = -1;  // last REDUCE: wrote this rank's chunk, read scratch
  for (const BcubeStep& s : steps) {
    const size_t first = pb.ops.size();
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      if (peer == r) continue;
      const size_t cl = s.chunk_len(i);
      if (cl) pb.add(kOpSend, peer, kBufUser, (int64_t)(s.off + i * s.chunk) * es, (int64_t)cl * es);
      if (s.mlen) pb.add(kOpRecv, peer, kBufScratch, (int64_t)(i * s.chunk) * es, (int64_t)s.mlen * es);
    }
    if (pb.ops.size() == first) continue;
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
    for (size_t i = 0; i < s.g && s.mlen; i++) {
      if ((int)(s.base + i * s.dist) == r) continue;
      last = pb.add(kOpReduce, -1, kBufUser, (int64_t)s.moff * es, (int64_t)s.mlen * es,
                    (int64_t)(i * s.chunk) * es, 0, 2, grp);
    }
  }
  bool first_ag = true;
  for (auto it = steps.rbegin(); it != steps.rend(); ++it) {
    const BcubeStep& s = *it;
    const size_t first = pb.ops.size();
    for (size_t i = 0; i < s.g; i++) {
      const int peer = (int)(s.base + i * s.dist);
      if (peer == r) continue;
      if (s.mlen) pb.add(kOpSend, peer, kBufUser, (int64_t)s.moff * es, (int64_t)s.mlen * es);
      const size_t cl = s.chunk_len(i);
      if (cl) pb.add(kOpRecv, peer, kBufUser, (int64_t)(s.off + i * s.chunk) * es, (int64_t)cl * es);
    }
    if (pb.ops.size() == first) continue;
    pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, first_ag ? last : -1);
    first_ag = false;
  }
  return pb.ops;
}

// ---- REDUCE to a root: gloo::reduce (reduce.cc:21-262) on device ---------------------------
// The reduce-scatter is DIRECT's (every rank sends each owner its block chunk in one p2p group,
// the owner folds the P contributions in the reference's order) over gloo::reduce's own block
// geometry, so owner q's block is x_q + (x_{q+1} + (... + x_{q-1})) exactly as the reference's
// ring leaves it; then every owner sends its block to the root (reduce.cc:229-261) chunk by
// chunk, as soon as that chunk is folded.  The root's bucket ends with the reduction; another
// rank's bucket holds its own folded block and its input elsewhere (only the root is defined).
inline std::vector<PlanOp> plan_reduce(const PlanGeom& g, int r) {
  PlanBuilder pb;
  const int P = g.P;
  if (P <= 1 || g.total == 0 || g.root < 0) return pb.ops;
  const size_t C = g.nchunks();
  int reader[2] = {-1, -1};
  std::vector<int> folded(C, -1);
  for (size_t c = 0; c < C; c++) {  // reduce-scatter: plan_direct's first half
    const int par = (int)(c & 1);
    const int64_t base = (int64_t)par * (P - 1) * (int64_t)g.chunk;
    bool any = false;
    for (int d = 1; d < P; d++) {
      const int q = (r + d) % P;
      size_t b, l;
      g.chunk_of(q, c, &b, &l);
      if (l) { pb.add(kOpSend, q, kBufUser, b, l); any = true; }
    }
    size_t mb, ml;
    g.chunk_of(r, c, &mb, &ml);
    if (ml)
      for (int j = 1; j < P; j++) {
        pb.add(kOpRecv, (r + j) % P, kBufScratch, base + (int64_t)(j - 1) * (int64_t)g.chunk, ml);
        any = true;
      }
    if (!any) continue;
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, reader[par]);
    if (ml) {
      const int f = pb.add(kOpFold, -1, kBufUser, mb, ml, base, (int64_t)g.chunk, P, grp);
      reader[par] = f;
      folded[c] = f;
    }
  }
  for (size_t c = 0; c < C; c++) {  // gather the owners' blocks to the root
    bool any = false;
    if (r == g.root) {
      for (int d = 1; d < P; d++) {
        const int q = (r + d) % P;
        size_t b, l;
        g.chunk_of(q, c, &b, &l);
        if (l) { pb.add(kOpRecv, q, kBufUser, b, l); any = true; }
      }
      if (any) pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, -1);
    } else {
      size_t mb, ml;
      g.chunk_of(r, c, &mb, &ml);
      if (ml) {
        pb.add(kOpSend, g.root, kBufUser, mb, ml);
        pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, folded[c]);
      }
    }
  }
  return pb.ops;
}

// ---- HALVING_DOUBLING: gloo::AllreduceHalvingDoubling<T> (allreduce_halving_doubling.h) ----
// One p2p group per step of the reference's schedule (shared geometry, halving_doubling_
// geometry.h): recursive halving inside the binary block (send the other half out of the
// bucket, receive the partner's half into scratch, REDUCE x = x op scratch), the smaller
// block's piece folded into the kept chunk, the kept chunk scattered to the next larger block
// and its finished pieces received back in place, the finished chunk forwarded to the smaller
// block, then recursive doubling straight into the bucket.  Same operands in the same order as
// the reference, so every rank ends with its bits.
inline std::vector<PlanOp> plan_halving_doubling(const PlanGeom& g, int r) {
  PlanBuilder pb;
  if (g.P <= 1 || g.n == 0) return pb.ops;
  const detail::HalvingDoublingGeometry h(g.P, r, g.n);
  const int64_t es = (int64_t)g.esize;
  int last = -1;  // last REDUCE: wrote the bucket, read scratch
  for (size_t i = 0; i < h.steps.size(); i++) {
    const auto& s = h.steps[i];
    const int peer = r ^ (1 << i);
    if (!s.send_cnt && !s.recv_cnt) continue;
    if (s.send_cnt) pb.add(kOpSend, peer, kBufUser, (int64_t)s.send_off * es, (int64_t)s.send_cnt * es);
    if (s.recv_cnt) pb.add(kOpRecv, peer, kBufScratch, 0, (int64_t)s.recv_cnt * es);
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
    if (s.recv_cnt)
      last = pb.add(kOpReduce, -1, kBufUser, (int64_t)s.recv_off * es, (int64_t)s.recv_cnt * es, 0,
                    0, 2, grp);
  }
  const int64_t kept_off = (int64_t)h.kept_off * es, kept = (int64_t)h.kept * es;
  if (h.smaller && kept) {  // :263-269
    pb.add(kOpRecv, h.smaller_peer(), kBufScratch, 0, kept);
    const int grp = pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
    last = pb.add(kOpReduce, -1, kBufUser, kept_off, kept, 0, 0, 2, grp);
  }
  if (h.larger && kept) {  // :273-301
    const int k = h.larger / h.block;
    for (int i = 0; i < k; i++)
      if (const size_t l = h.piece_len(i))
        pb.add(kOpSend, h.larger_peer(i), kBufUser, kept_off + (int64_t)(h.piece_to_larger * i) * es,
               (int64_t)l * es);
    pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
    for (int i = 0; i < k; i++)
      if (const size_t l = h.piece_len(i))
        pb.add(kOpRecv, h.larger_peer(i), kBufUser, kept_off + (int64_t)(h.piece_to_larger * i) * es,
               (int64_t)l * es);
    pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, -1);
  }
  if (h.smaller && kept) {  // :306-313
    pb.add(kOpSend, h.smaller_peer(), kBufUser, kept_off, kept);
    pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
  }
  for (size_t i = h.steps.size(); i-- > 0;) {  // :316-338
    const auto& s = h.steps[i];
    const int peer = r ^ (1 << i);
    if (!s.send_cnt && !s.recv_cnt) continue;
    if (s.recv_cnt) pb.add(kOpSend, peer, kBufUser, (int64_t)s.recv_off * es, (int64_t)s.recv_cnt * es);
    if (s.send_cnt) pb.add(kOpRecv, peer, kBufUser, (int64_t)s.send_off * es, (int64_t)s.send_cnt * es);
    pb.add(kOpGroup, -1, 0, 0, 0, 0, 0, 0, last);
  }
  return pb.ops;
}

inline std::vector<PlanOp> make_plan(int algo, const PlanGeom& g, int r) {
  if (algo == kAlgoHalvingDoubling) return plan_halving_doubling(g, r);
  if (algo == kAlgoReduce) return plan_reduce(g, r);
  if (algo == kAlgoBcube) return plan_bcube(g, r);
  if (algo == kAlgoRingChunked) return plan_ring_chunked(g, r);
  if (algo == kAlgoRingOld) return plan_ring_old(g, r);
  if (algo == kAlgoRing) return plan_ring(g, r);
  if (algo == kAlgoA2A) return plan_a2a(g, r);
  return plan_direct(g, r);
}

}  // namespace hydra
