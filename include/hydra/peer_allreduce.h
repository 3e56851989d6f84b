// hydra::PeerAllreduce<T> -- the peer-access bucket allreduce (hydra_hip.h, hydra_peer_*)
// behind the reference's Algorithm shape: a constructor that does all setup, then run()
// (gloo/gloo/algorithm.h:27-38; cf. CudaAllreduceRing's (context, ptrs, count, streams) ctor,
// cuda_allreduce_ring.cc:17-76).  The 128-byte IPC handle blobs travel over the host
// runtime's own TCP full mesh (an all-gather on `context`), so a C++ caller of
// include/hydra/allreduce.h needs no other channel.
//
// One process per GPU, one device bucket per rank, identical `count` on every rank.  run()
// is ONE gfx950 kernel that reads the other ranks' blocks over xGMI and folds them in the
// reference ring's order, so every rank ends with gloo::allreduce RING's bits
// (allreduce.cc:147-422, maxSegmentSize fixing block ownership).  Without a caller stream
// run() is synchronous, like the reference's algorithms; with one it is enqueued on it.
#pragma once

#include <chrono>
#include <cstring>
#include <memory>
#include <vector>

#include "allreduce.h"
#include "gloo_reduce.h"
#include "../hydra_hip.h"

namespace hydra {

namespace detail {
// All-gather of one `len`-byte blob per rank over the context's pairs, rank order.
inline std::vector<char> allgather_blob(Context& ctx, const void* mine, size_t len,
                                        uint64_t slot) {
  const int P = ctx.size, r = ctx.rank;
  std::vector<char> all((size_t)P * len);
  std::memcpy(all.data() + (size_t)r * len, mine, len);
  std::vector<char> own(static_cast<const char*>(mine), static_cast<const char*>(mine) + len);
  auto out = ctx.createUnboundBuffer(own.data(), len);
  auto in = ctx.createUnboundBuffer(all.data(), all.size());
  for (int q = 0; q < P; q++)
    if (q != r) in->recv(q, slot, (size_t)q * len, len);
  for (int q = 0; q < P; q++)
    if (q != r) out->send(q, slot, 0, len);
  for (int q = 0; q < P; q++)
    if (q != r) in->waitRecv(ctx.getTimeout());
  for (int q = 0; q < P; q++)
    if (q != r) out->waitSend(ctx.getTimeout());
  return all;
}
}  // namespace detail

template <typename T>
class PeerAllreduce {
 public:
  PeerAllreduce(const std::shared_ptr<Context>& context, T* ptr, size_t count,
                hydra_stream_t stream = nullptr, int algo = HYDRA_PEER_AUTO,
                size_t maxSegmentSize = 0)
      : ctx_(context), ptr_(ptr), count_(count), algo_(algo), max_segment_(maxSegmentSize),
        stream_(stream), synchronous_(stream == nullptr) {
    using gloo_compat::enforce;
    if (!ctx_) throw EnforceNotMet("PeerAllreduce: null context");
    if (count_ && !ptr_) throw EnforceNotMet("PeerAllreduce: null pointer");
    enforce(hydra_pointer_device(ptr_, &device_));
    if (device_ < 0) throw EnforceNotMet("PeerAllreduce: ptr must be device memory");
    if (synchronous_) enforce(hydra_stream_create(device_, &stream_));
    char sig[HYDRA_PEER_HANDLE_BYTES], h[HYDRA_PEER_HANDLE_BYTES];
    enforce(hydra_peer_create(ctx_->size, ctx_->rank, device_, &peer_, sig));
    const auto sigs = detail::allgather_blob(*ctx_, sig, sizeof(sig), slot(0));
    enforce(hydra_peer_connect(peer_, sigs.data()));
    enforce(hydra_peer_register(peer_, ptr_, bytes(), h));
    const auto hs = detail::allgather_blob(*ctx_, h, sizeof(h), slot(1));
    enforce(hydra_peer_open(peer_, ptr_, bytes(), hs.data()));
  }

  // Collective, like the constructor: every rank closes its mappings of the others' memory,
  // meets the others, and only then frees its own signal area -- so once the destructor
  // returns on any rank, no rank maps that rank's bucket any more and the caller may free it
  // (hydra_hip.h, teardown rule).
  ~PeerAllreduce() {
    if (peer_) {
      hydra_peer_detach(peer_);
      try {
        const char c = 0;
        (void)detail::allgather_blob(*ctx_, &c, 1, slot(2));
      } catch (...) {  // a dead peer: nothing left to wait for
      }
      hydra_peer_destroy(peer_);
    }
    if (synchronous_ && stream_) hydra_stream_destroy(stream_);
  }
  PeerAllreduce(const PeerAllreduce&) = delete;
  PeerAllreduce& operator=(const PeerAllreduce&) = delete;

  void run() {
    using gloo_compat::enforce;
    enforce(hydra_peer_allreduce(peer_, algo_, HYDRA_SUM, gloo_compat::dtype_of<T>(), 0, ptr_,
                                 count_, max_segment_, stream_));
    if (synchronous_) {
      enforce(hydra_stream_synchronize(stream_));
      int err = 0;
      enforce(hydra_peer_error(peer_, &err));
      if (err)  // a peer never arrived: the reference's IoException on a timed-out op
        throw IoException("Timed out waiting for a peer in the peer-access allreduce (code " +
                          std::to_string(err) + ")");
    }
  }

 private:
  size_t bytes() const { return count_ * sizeof(T); }
  static uint64_t slot(int i) { return (uint64_t(0x13) << 56) | (uint64_t)i; }

  std::shared_ptr<Context> ctx_;
  T* ptr_;
  size_t count_;
  int algo_;
  size_t max_segment_;
  hydra_stream_t stream_;
  bool synchronous_;
  int device_ = -1;
  hydra_peer_t peer_ = nullptr;
};

}  // namespace hydra
