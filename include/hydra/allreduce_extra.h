// include/hydra/allreduce_extra.h -- OUT OF SCOPE, opt-in: the other old-style Gloo
// Algorithm-API allreduce classes.
//
// SURVEY.md §2 lists these under "Other Gloo collectives" (out of scope for the bucket-reduction
// hot path); they were built in round 2 on the same ReductionFunction<T> plug-point and stay
// available -- with their reference-built fixtures and tests (pytest marker `extra`, run with
// HYDRA_EXTRA_TESTS=1) -- but nothing in the default build, test run or bench includes them:
//   AllreduceHalvingDoubling<T>  gloo/gloo/allreduce_halving_doubling.h:37-358
//   AllreduceLocal<T>            gloo/gloo/allreduce_local.cc:28-38
//   AllreduceBcube<T> (old-style) gloo/gloo/allreduce_bcube.h:255-691
#pragma once

#include <cstring>
#include <memory>
#include <vector>

#include "allreduce.h"
#include "halving_doubling_geometry.h"

namespace hydra {

// gloo::AllreduceHalvingDoubling<T> (allreduce_halving_doubling.h:37-358).  P splits into
// binary blocks (largest at rank 0, :39-64).  Inside a block, step i exchanges with
// rank ^ 2^i: recursive halving folds the kept half (x = x op received, :241-256), then
// recursive doubling copies the other half back (:316-338).  Between blocks, a rank folds the
// piece from its smaller-block partner (:263-269), scatters its chunk to the next larger block
// in bit-reversed order (:273-287), copies the larger block's finished pieces back (:293-301),
// and forwards its finished chunk to the smaller block (:306-313).  Receives land straight in
// the bucket where the reference copies from its recvBuf_ (same bits); the notification
// handshake is implicit in the FIFO transport, as for the rings above.

namespace detail {
// AllreduceHalvingDoubling's schedule (allreduce_halving_doubling.h:224-358) over `count`
// elements of `es` bytes at `base` (host memory the transport sends from), for this rank's
// geometry `g`.  fold(dst, box, n) applies dst op= box for n elements; `inbox` holds
// g.inbox_elems() elements.  Shared by AllreduceHalvingDoubling<T> and
// HipAllreduceHalvingDoubling<T, W> (cuda_allreduce_halving_doubling.cc), which differ only in
// where the fold runs.
//
// Sends read the bucket asynchronously (the pair's writer thread), so every region a later
// receive writes is first released by waiting on the send that read it.  Each phase sends
// through its own view of the bucket, so one wait never blocks on an unrelated send.
template <typename Fold>
void halving_doubling(Context& ctx, const HalvingDoublingGeometry& g, char* base, size_t count,
                      size_t es, char* inbox, uint64_t slot, Fold fold) {
  const auto tmo = ctx.getTimeout();
  const int r = ctx.rank;
  const size_t E = es, n = count;
  const uint64_t slot_up = slot + 0x40, slot_down = slot + 0x41, slot_gather = slot + 0x80;
  const size_t S = g.steps.size();
  std::vector<std::unique_ptr<UnboundBuffer>> halve;  // one per step: its send is waited
  std::vector<char> halve_sent(S, 0);                 // before doubling writes that region
  for (size_t i = 0; i < S; i++) halve.push_back(ctx.createUnboundBuffer(base, n * E));
  auto up = ctx.createUnboundBuffer(base, n * E);    // scatter to the larger block
  auto down = ctx.createUnboundBuffer(base, n * E);  // larger block's pieces, chunk to smaller
  auto dbl = ctx.createUnboundBuffer(base, n * E);   // recursive doubling
  auto box = ctx.createUnboundBuffer(inbox, g.inbox_elems() * E);
  size_t up_sent = 0, down_sent = 0, dbl_sent = 0;
  // 1. recursive halving inside the block
  for (size_t i = 0; i < S; i++) {
    const auto& s = g.steps[i];
    const int peer = r ^ (1 << i);
    if (s.send_cnt) {
      halve[i]->send(peer, slot + i, s.send_off * E, s.send_cnt * E);
      halve_sent[i] = 1;
    }
    if (s.recv_cnt) {
      box->recv(peer, slot + i, 0, s.recv_cnt * E);
      box->waitRecv(tmo);
      fold(base + s.recv_off * E, inbox, s.recv_cnt);
    }
  }
  // 2. fold the smaller block's piece of my chunk
  if (g.smaller && g.kept) {
    box->recv(g.smaller_peer(), slot_up, 0, g.kept * E);
    box->waitRecv(tmo);
    fold(base + g.kept_off * E, inbox, g.kept);
  }
  // 3. scatter my chunk to the larger block, then take the finished pieces back in place
  if (g.larger && g.kept) {
    const int k = g.larger / g.block;
    for (int i = 0; i < k; i++)
      if (const size_t l = g.piece_len(i)) {
        up->send(g.larger_peer(i), slot_up, (g.kept_off + g.piece_to_larger * i) * E, l * E);
        up_sent++;
      }
    for (; up_sent; up_sent--) up->waitSend(tmo);
    int posted = 0;
    for (int i = 0; i < k; i++)
      if (const size_t l = g.piece_len(i)) {
        down->recv(g.larger_peer(i), slot_down, (g.kept_off + g.piece_to_larger * i) * E, l * E);
        posted++;
      }
    for (int i = 0; i < posted; i++) down->waitRecv(tmo);
  }
  // 4. my finished chunk to the smaller block
  if (g.smaller && g.kept) {
    down->send(g.smaller_peer(), slot_down, g.kept_off * E, g.kept * E);
    down_sent++;
  }
  // 5. recursive doubling inside the block
  for (size_t i = S; i-- > 0;) {
    const auto& s = g.steps[i];
    const int peer = r ^ (1 << i);
    if (s.recv_cnt) {
      dbl->send(peer, slot_gather + i, s.recv_off * E, s.recv_cnt * E);
      dbl_sent++;
    }
    if (s.send_cnt) {
      if (halve_sent[i]) halve[i]->waitSend(tmo), halve_sent[i] = 0;
      dbl->recv(peer, slot_gather + i, s.send_off * E, s.send_cnt * E);
      dbl->waitRecv(tmo);
    }
  }
  for (size_t i = 0; i < S; i++)
    if (halve_sent[i]) halve[i]->waitSend(tmo);
  for (; down_sent; down_sent--) down->waitSend(tmo);
  for (; dbl_sent; dbl_sent--) dbl->waitSend(tmo);
}
}  // namespace detail

template <typename T>
class AllreduceHalvingDoubling {
 public:
  AllreduceHalvingDoubling(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                           int count, const ReductionFunction<T>* fn)
      : ctx_(context), ptrs_(ptrs), count_(count), fn_(fn),
        geo_(context->size, context->rank, count < 0 ? 0 : (size_t)count) {
    if (!fn_) throw EnforceNotMet("AllreduceHalvingDoubling: null reduction function");
    if (ptrs_.empty()) throw EnforceNotMet("AllreduceHalvingDoubling: no pointers");
    if (count_ < 0) throw EnforceNotMet("AllreduceHalvingDoubling: negative count");
    inbox_.resize(geo_.inbox_elems());
  }

  void run() {
    const size_t n = (size_t)count_, E = sizeof(T);
    for (size_t i = 1; i < ptrs_.size(); i++) fn_->call(ptrs_[0], ptrs_[i], count_);
    if (ctx_->size > 1 && n > 0)
      detail::halving_doubling(*ctx_, geo_, reinterpret_cast<char*>(ptrs_[0]), n, E,
                               reinterpret_cast<char*>(inbox_.data()), kSlot,
                               [this](char* dst, const char* box, size_t l) {
                                 fn_->call(reinterpret_cast<T*>(dst),
                                           reinterpret_cast<const T*>(box), l);
                               });
    for (size_t i = 1; i < ptrs_.size(); i++) std::memcpy(ptrs_[i], ptrs_[0], n * E);
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x12) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  const ReductionFunction<T>* fn_;
  detail::HalvingDoublingGeometry geo_;
  std::vector<T> inbox_;
};

// gloo::AllreduceLocal<T> (allreduce_local.{h,cc}): no communication -- ptrs[0] op= ptrs[i] in
// pointer order (allreduce_local.cc:30-33), then every pointer gets ptrs[0] (:35-37).
template <typename T>
class AllreduceLocal {
 public:
  AllreduceLocal(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, int count,
                 const ReductionFunction<T>* fn)
      : ctx_(context), ptrs_(ptrs), count_(count), fn_(fn) {
    if (!fn_) throw EnforceNotMet("AllreduceLocal: null reduction function");
    if (count_ < 0) throw EnforceNotMet("AllreduceLocal: negative count");
  }

  void run() {
    for (size_t i = 1; i < ptrs_.size(); i++) fn_->call(ptrs_[0], ptrs_[i], count_);
    for (size_t i = 1; i < ptrs_.size(); i++)
      std::memcpy(ptrs_[i], ptrs_[0], (size_t)count_ * sizeof(T));
  }

 private:
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  const ReductionFunction<T>* fn_;
};

// Old-style gloo::AllreduceBcube<T> (allreduce_bcube.h:255-691) with the context's default base
// 2: the left-fold local reduce (:339-341), then the hypercube reduce-scatter / all-gather.  For
// P a power of two its result is the new-style BCUBE's bit for bit (checked against the
// reference's own class, tests/test_oracle.py), so the bucket runs through allreduce(BCUBE)
// with the ReductionFunction as the Func.  For other P the reference's ranks end with different
// values; this class refuses them instead (EnforceNotMet).
template <typename T>
class AllreduceBcube {
 public:
  AllreduceBcube(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, int count,
                 const ReductionFunction<T>* fn)
      : ctx_(context), ptrs_(ptrs), count_(count), fn_(fn) {
    if (!fn_) throw EnforceNotMet("AllreduceBcube: null reduction function");
    if (ptrs_.empty()) throw EnforceNotMet("AllreduceBcube: no pointers");
    if (count_ < 0) throw EnforceNotMet("AllreduceBcube: negative count");
    if (ctx_->size & (ctx_->size - 1))
      throw EnforceNotMet("AllreduceBcube: the number of ranks must be a power of the base (2)");
  }

  void run() {
    const size_t n = (size_t)count_, bytes = n * sizeof(T);
    for (size_t i = 1; i < ptrs_.size(); i++) fn_->call(ptrs_[0], ptrs_[i], count_);
    if (ctx_->size > 1 && n > 0) {
      AllreduceOptions opts(ctx_);
      opts.setAlgorithm(AllreduceOptions::BCUBE);
      opts.setOutput(ptrs_[0], n);
      const ReductionFunction<T>* fn = fn_;
      opts.setReduceFunction([fn](void* c, const void* a, const void* b, size_t l) {
        if (c != a) std::memcpy(c, a, l * sizeof(T));
        fn->call(static_cast<T*>(c), static_cast<const T*>(b), l);
      });
      allreduce(opts);
    }
    for (size_t i = 1; i < ptrs_.size(); i++) std::memcpy(ptrs_[i], ptrs_[0], bytes);
  }

 private:
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  const ReductionFunction<T>* fn_;
};

}  // namespace hydra
