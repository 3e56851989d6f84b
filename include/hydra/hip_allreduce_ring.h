// hydra::HipAllreduceRing<T, W> -- the HIP analog of gloo::CudaAllreduceRing<T, W>
// (gloo/gloo/cuda_allreduce_ring.{h,cc}) for device-resident buffers on the host runtime's TCP
// ring.  Same constructor (context, device ptrs, count, optional streams) and run(); same
// result on rank r: x_r + x_{r-1} + ... + x_{r-P+1} (the AllreduceRing left fold,
// cuda_allreduce_ring.cc:85-112), where x_r is the rank's locally reduced value.
//
//   HipHostWorkspace<T>   (CudaHostWorkspace, cuda_allreduce_ring.cc:122-142): the ring runs
//       on pinned host boxes; the local pre-reduce is a left fold ptrs[0] op= ptrs[i] in
//       pointer order (cuda_collectives_host.h:108-119), done on the device; each round's
//       scratch += inbox is hydra_reduce_host (the gfx950 kernel behind a staged copy), where
//       the reference runs its CPU sum<T>.
//   HipDeviceWorkspace<T> (CudaDeviceWorkspace, :144-170): scratch is ptrs[0] itself; the local
//       pre-reduce is the pairwise tree of CudaLocalNativeReduce (cuda_collectives_native.h:
//       93-122) in pointer order (the reference shuffles the order at random, :53, so for
//       floats with > 2 pointers it is itself nondeterministic; pointer order is one of its
//       outcomes); each round's fold runs on the device on a copy of the received box.  TCP
//       cannot read HBM, so the boxes the ring sends are pinned host memory: round 0 sends a
//       D2H copy of scratch and round k forwards the box received in round k-1 (which holds
//       exactly the bytes the reference's device outbox would).
//
// Pointers may live on several GPUs of the process, as CudaAllreduceRing accepts them
// (cuda_allreduce_ring.cc:34-42: one stream per pointer, on the pointer's device):
//   * every pointer's device is looked up once (hydra_pointer_device); owned streams and the
//     ordering events are created on it;
//   * the ring accumulates into one chosen pointer's device (findCudaDevicePointerClosestToDevice,
//     cuda_allreduce_ring.cc:153-157): the smallest PCI distance to the transport's device.  The
//     host runtime's TCP transport has no PCI device, so every distance is equal and the first
//     pointer is chosen (the reference picks one of the equals at random: ours is one outcome);
//   * each local-reduce step ptrs[a] op= ptrs[b] runs on a's device and stream, after a waits for
//     b's stream (cuda_collectives_native.h:100-115); across devices the kernel reads b over
//     peer access where hipDeviceCanAccessPeer allows it (enabled once, :63-84), otherwise b is
//     first copied to a buffer on a's device (the reference refuses that case);
//   * the broadcast copies the result to every pointer on that pointer's stream.
// One GPU cannot exercise the cross-device branches; the bookkeeping (detail::local_steps) is
// unit-tested on the CPU and the same code runs every single-device case.
// Only ReductionFunction SUM exists on this class, as in the reference (fn_ =
// CudaReductionFunction<T>::sum, cuda_allreduce_ring.cc:26).
#pragma once

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>
#include <vector>

#include "allreduce.h"
#include "gloo_reduce.h"
#include "../hydra_hip.h"

namespace hydra {

template <typename T>
struct HipHostWorkspace {};
template <typename T>
struct HipDeviceWorkspace {};

namespace detail {
using gloo_compat::enforce;

struct Pinned {  // CudaHostPointer<T>::alloc (cuda.cu:231-240)
  void* p = nullptr;
  Pinned() = default;
  explicit Pinned(size_t bytes) { enforce(hydra_malloc_host(bytes, &p)); }
  Pinned(const Pinned&) = delete;
  Pinned& operator=(const Pinned&) = delete;
  Pinned& operator=(Pinned&& o) noexcept {
    std::swap(p, o.p);
    return *this;
  }
  ~Pinned() {
    if (p) hydra_free_host(p);
  }
};

struct DeviceMem {
  void* p = nullptr;
  DeviceMem() = default;
  DeviceMem(int device, size_t bytes) { enforce(hydra_malloc(device, bytes ? bytes : 1, &p)); }
  DeviceMem(const DeviceMem&) = delete;
  DeviceMem& operator=(const DeviceMem&) = delete;
  DeviceMem(DeviceMem&& o) noexcept : p(o.p) { o.p = nullptr; }
  DeviceMem& operator=(DeviceMem&& o) noexcept {
    std::swap(p, o.p);
    return *this;
  }
  ~DeviceMem() {
    if (p) hydra_free(p);
  }
};
// ---- several devices per process: the local reduce's bookkeeping ---------------------------
// One step of a local reduction: buffer a op= buffer b, run on a's device and stream.  `staged`:
// a's device cannot read b's (no peer access), so b is first copied to a buffer on a's device.
struct LocalStep {
  size_t a, b;
  bool staged;
};

// CudaLocalNativeReduce's pairwise tree (cuda_collectives_native.h:93-122) in pointer order:
// level sz pairs (j, j + sz) for j a multiple of 2 sz; the result lands in pointer 0.  (The
// reference shuffles the order at random, :53, and drops pointers beyond the largest power of
// two, :36; every pointer is folded here.)
template <typename CanPeer>
std::vector<LocalStep> local_tree(const std::vector<int>& dev, CanPeer can_peer) {
  std::vector<LocalStep> v;
  for (size_t sz = 1; sz < dev.size(); sz *= 2)
    for (size_t j = 0; j + sz < dev.size(); j += 2 * sz)
      v.push_back({j, j + sz, dev[j] != dev[j + sz] && !can_peer(dev[j], dev[j + sz])});
  return v;
}

// CudaLocalHostReduce's order (cuda_collectives_host.h:108-119): target = ptrs[0], then
// target op= ptrs[i] for i = 1, 2, ... (a left fold in pointer order).
template <typename CanPeer>
std::vector<LocalStep> local_chain(const std::vector<int>& dev, CanPeer can_peer) {
  std::vector<LocalStep> v;
  for (size_t i = 1; i < dev.size(); i++)
    v.push_back({0, i, dev[0] != dev[i] && !can_peer(dev[0], dev[i])});
  return v;
}

// findCudaDevicePointerClosestToDevice (cuda_private.h:58-90): the pointer with the smallest
// PCI distance to the transport's device; the first of equals.
inline size_t closest_index(const std::vector<int>& distance) {
  size_t best = 0;
  int bd = INT_MAX;
  for (size_t i = 0; i < distance.size(); i++)
    if (distance[i] < bd) {
      bd = distance[i];
      best = i;
    }
  return best;
}

// Runs a step list on device buffers: per pointer i its device, stream and an ordering event;
// one staging buffer per destination that needs one.
class LocalReduce {
 public:
  LocalReduce() = default;
  LocalReduce(const LocalReduce&) = delete;
  LocalReduce& operator=(const LocalReduce&) = delete;
  ~LocalReduce() {
    for (auto e : ev_) hydra_event_destroy(e);
  }
  void init(std::vector<LocalStep> steps, const std::vector<int>& dev, size_t bytes) {
    steps_ = std::move(steps);
    // test switch HYDRA_TEST_LOCAL_STAGE (hydra_test_set): every step staged as if its two
    // pointers were on devices without peer access, so the one-GPU box runs the cross-device
    // staging branch (copy to a buffer on the destination's device, event waits) with real
    // kernels
    int64_t stage_all = 0;
    if (hydra_test_get(HYDRA_TEST_LOCAL_STAGE, &stage_all) == HYDRA_OK && stage_all == 1)
      for (LocalStep& s : steps_) s.staged = true;
    ev_.assign(dev.size(), nullptr);
    for (size_t i = 0; i < dev.size(); i++) enforce(hydra_event_create_on(dev[i], &ev_[i]));
    stage_.clear();
    stage_.resize(dev.size());
    for (const LocalStep& s : steps_)
      if (s.staged && !stage_[s.a].p) stage_[s.a] = DeviceMem(dev[s.a], bytes);
  }
  // buf[i]: the buffer standing for pointer i (pointer 0 may be a copy); streams[i] on dev[i]
  void run(const std::vector<void*>& buf, const std::vector<hydra_stream_t>& streams, int dt,
           int count, size_t bytes) {
    for (const LocalStep& s : steps_) {
      enforce(hydra_event_record(ev_[s.b], streams[s.b]));  // b's pending work first
      enforce(hydra_stream_wait_event(streams[s.a], ev_[s.b]));
      const void* src = buf[s.b];
      if (s.staged) {
        enforce(hydra_memcpy_async(stage_[s.a].p, buf[s.b], bytes, streams[s.a]));
        src = stage_[s.a].p;
      }
      enforce(hydra_reduce(HYDRA_SUM, dt, buf[s.a], buf[s.a], src, count, streams[s.a]));
    }
  }
  const std::vector<LocalStep>& steps() const { return steps_; }

 private:
  std::vector<LocalStep> steps_;
  std::vector<hydra_event_t> ev_;
  std::vector<DeviceMem> stage_;
};

// Per-pointer devices (CudaDevicePointer::create, cuda.cu:175-188); every pointer must be
// device memory.
template <typename T>
std::vector<int> pointer_devices(const std::vector<T*>& ptrs, const char* who) {
  std::vector<int> dev(ptrs.size(), -1);
  for (size_t i = 0; i < ptrs.size(); i++) {
    enforce(hydra_pointer_device(ptrs[i], &dev[i]));
    if (dev[i] < 0) throw EnforceNotMet(std::string(who) + ": ptrs must be device memory");
  }
  return dev;
}

// hydra_device_peer_access as the steps' predicate (enables access where it can).
inline bool peer_access(int a, int b) {
  int can = 0;
  enforce(hydra_device_peer_access(a, b, &can));
  return can != 0;
}

// Completion of run()'s last output copies, recorded on each caller stream as an event this
// object owns.  The destructor waits on these events before the pinned / device scratch the
// copies read is freed -- never on the caller's streams, which it does not own and which the
// caller may already have destroyed.
class OutputFence {
 public:
  OutputFence() = default;
  OutputFence(const OutputFence&) = delete;
  OutputFence& operator=(const OutputFence&) = delete;
  ~OutputFence() {
    wait_nothrow();
    for (auto e : ev_) hydra_event_destroy(e);
  }
  // every stream on `device`
  void record(int device, const std::vector<hydra_stream_t>& streams) {
    record(std::vector<int>(streams.size(), device), streams);
  }
  // streams[i] on devices[i] (events must be created on their stream's device, whatever device
  // is current on the calling thread)
  void record(const std::vector<int>& devices, const std::vector<hydra_stream_t>& streams) {
    while (ev_.size() < streams.size()) {
      hydra_event_t e = nullptr;
      enforce(hydra_event_create_on(devices[ev_.size()], &e));
      ev_.push_back(e);
    }
    for (size_t i = 0; i < streams.size(); i++) enforce(hydra_event_record(ev_[i], streams[i]));
    recorded_ = streams.size();
  }
  void wait_nothrow() {
    for (size_t i = 0; i < recorded_; i++) hydra_event_synchronize(ev_[i]);
  }

 private:
  std::vector<hydra_event_t> ev_;
  size_t recorded_ = 0;
};
}  // namespace detail

template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRing {
  static constexpr bool kDeviceWorkspace = std::is_same<W, HipDeviceWorkspace<T>>::value;
  static_assert(kDeviceWorkspace || std::is_same<W, HipHostWorkspace<T>>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  HipAllreduceRing(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, int count,
                   const std::vector<hydra_stream_t>& streams = std::vector<hydra_stream_t>())
      : ctx_(context), ptrs_(ptrs), count_(count), bytes_((size_t)count * sizeof(T)),
        synchronize_outputs_(streams.empty()) {
    using detail::enforce;
    if (ptrs_.empty()) throw EnforceNotMet("HipAllreduceRing: no pointers");
    if (count_ < 0) throw EnforceNotMet("HipAllreduceRing: negative count");
    if (!streams.empty() && streams.size() != ptrs_.size())
      throw EnforceNotMet("HipAllreduceRing: streams.size() != ptrs.size()");  // :30-33
    if (count_ == 0) return;  // nothing to move (pointers may be null)
    dev_ = detail::pointer_devices(ptrs_, "HipAllreduceRing");
    if (streams.empty()) {
      owned_.resize(ptrs_.size());
      for (size_t i = 0; i < owned_.size(); i++) enforce(hydra_stream_create(dev_[i], &owned_[i]));
      streams_ = owned_;
    } else {
      streams_ = streams;
    }
    // the pointer the ring accumulates into: closest to the transport (no PCI device: the first)
    root_ = kDeviceWorkspace ? detail::closest_index(std::vector<int>(ptrs_.size(), 0)) : 0;
    device_ = dev_[root_];
    boxes_[0] = detail::Pinned(bytes_ ? bytes_ : 1);
    boxes_[1] = detail::Pinned(bytes_ ? bytes_ : 1);
    if (kDeviceWorkspace) {
      inbox_dev_ = detail::DeviceMem(device_, bytes_);
      if (ptrs_.size() > 1) local_.init(detail::local_tree(dev_, detail::peer_access), dev_, bytes_);
    } else {
      scratch_host_ = detail::Pinned(bytes_ ? bytes_ : 1);
      if (ptrs_.size() > 1) {
        local_dev_ = detail::DeviceMem(device_, bytes_);
        local_.init(detail::local_chain(dev_, detail::peer_access), dev_, bytes_);
      }
    }
  }

  ~HipAllreduceRing() {
    // outputs may still be copying from pinned scratch on the caller's streams: wait for the
    // fence events run() recorded (not the streams) before the pinned / device buffers are freed
    fence_.wait_nothrow();
    for (auto s : owned_) hydra_stream_destroy(s);
  }
  HipAllreduceRing(const HipAllreduceRing&) = delete;
  HipAllreduceRing& operator=(const HipAllreduceRing&) = delete;

  void run() {
    using detail::enforce;
    if (count_ == 0) return;
    const int dt = gloo_compat::dtype_of<T>();
    hydra_stream_t s0 = streams_[root_];
    // ---- local reduce: scratch holds this rank's value x_r
    void* scratch;
    std::vector<void*> buf(ptrs_.begin(), ptrs_.end());
    if (kDeviceWorkspace) {
      // CudaLocalNativeReduce tree into ptrs[0] (each step on its destination's device), then
      // into the ring's pointer when that is another one (cudaDeviceReduce's target copy)
      local_.run(buf, streams_, dt, count_, bytes_);
      if (root_ != 0) {
        enforce(hydra_stream_synchronize(streams_[0]));
        enforce(hydra_memcpy_async(ptrs_[root_], ptrs_[0], bytes_, s0));
      }
      scratch = ptrs_[root_];
    } else {
      if (ptrs_.size() > 1) {  // ptrs[0] op= ptrs[i] in order, in place on a copy of ptrs[0]
        for (size_t i = 1; i < streams_.size(); i++) enforce(hydra_stream_synchronize(streams_[i]));
        enforce(hydra_memcpy_async(local_dev_.p, ptrs_[0], bytes_, s0));
        buf[0] = local_dev_.p;
        local_.run(buf, streams_, dt, count_, bytes_);
        enforce(hydra_memcpy_async(scratch_host_.p, local_dev_.p, bytes_, s0));
      } else {
        enforce(hydra_memcpy_async(scratch_host_.p, ptrs_[0], bytes_, s0));
      }
      scratch = scratch_host_.p;
    }
    // ---- the ring (cuda_allreduce_ring.cc:79-112)
    const int P = ctx_->size;
    if (P > 1 && count_ > 0) {
      const int right = (ctx_->rank + 1) % P, left = (ctx_->rank + P - 1) % P;
      const auto tmo = ctx_->getTimeout();
      enforce(hydra_memcpy_async(boxes_[0].p, scratch, bytes_, s0));  // outbox = scratch
      enforce(hydra_stream_synchronize(s0));
      int out = 0;
      for (int round = 0; round < P - 1; round++) {
        void* ob = boxes_[out].p;
        void* ib = boxes_[out ^ 1].p;
        auto send = ctx_->createUnboundBuffer(ob, bytes_);
        auto recv = ctx_->createUnboundBuffer(ib, bytes_);
        recv->recv(left, kSlot, 0, bytes_);
        send->send(right, kSlot, 0, bytes_);
        recv->waitRecv(tmo);
        if (kDeviceWorkspace) {
          enforce(hydra_memcpy_async(inbox_dev_.p, ib, bytes_, s0));
          enforce(hydra_reduce(HYDRA_SUM, dt, scratch, scratch, inbox_dev_.p, count_, s0));
          enforce(hydra_stream_synchronize(s0));  // ib is the next round's outbox
        } else {
          if (!lease_) lease_.reset(new gloo_compat::ContextPool::Lease(
                           gloo_compat::ContextPool::instance(device_).acquire()));
          enforce(hydra_reduce_host(lease_->get(), HYDRA_SUM, dt, scratch, scratch, ib, count_));
        }
        send->waitSend(tmo);
        out ^= 1;  // forward what was just received (outbox <- inbox, :100-103)
      }
      lease_.reset();
    }
    // ---- broadcast the result to every device pointer (:114-120), each on its own stream
    // (a copy to another device is a peer copy; hipMemcpyDefault routes it)
    enforce(hydra_stream_synchronize(s0));
    for (size_t i = 0; i < ptrs_.size(); i++)
      if (!kDeviceWorkspace || i != root_)
        enforce(hydra_memcpy_async(ptrs_[i], scratch, bytes_, streams_[i]));
    fence_.record(dev_, streams_);
    if (synchronize_outputs_)
      for (auto s : streams_) enforce(hydra_stream_synchronize(s));
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x12) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  size_t bytes_;
  bool synchronize_outputs_;
  int device_ = -1;     // the ring's device (dev_[root_])
  size_t root_ = 0;     // the pointer the ring accumulates into (device workspace)
  std::vector<int> dev_;  // per pointer
  std::vector<hydra_stream_t> streams_, owned_;
  detail::Pinned boxes_[2], scratch_host_;
  detail::DeviceMem inbox_dev_, local_dev_;
  detail::LocalReduce local_;
  std::unique_ptr<gloo_compat::ContextPool::Lease> lease_;
  detail::OutputFence fence_;  // declared last: destroyed first, before any scratch
};

// hydra::HipAllreduceRingChunked<T, W> -- the HIP analog of gloo::CudaAllreduceRingChunked<T, W>
// (gloo/gloo/cuda_allreduce_ring_chunked.{h,cc}): same constructor and run(), same result on
// every rank -- AllreduceRingChunked's (allreduce_ring_chunked.h) over each rank's locally
// reduced value.  The local reduce is CudaLocalNativeReduce's pairwise tree in pointer order
// for both workspaces (cudaDeviceReduce, cuda_collectives_device.h:29-56; memcpy for one
// pointer), the ring is the shared chunked schedule (allreduce.h detail::chunked_ring, 2P
// chunks of max(256, ceil(n / 2P))), and the broadcast copies the result to every pointer.
//   HipHostWorkspace<T>:   scratch and inboxes are pinned host memory; each fold is
//       hydra_reduce_host, i.e. the gfx950 kernel streaming the pinned chunks (zero-copy).
//   HipDeviceWorkspace<T>: scratch is ptrs[0] on the device; each fold copies the received
//       chunk to a device inbox, runs the kernel on the device chunk and refreshes the pinned
//       mirror the transport sends from (TCP cannot read HBM).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRingChunked {
  static constexpr bool kDeviceWorkspace = std::is_same<W, HipDeviceWorkspace<T>>::value;
  static_assert(kDeviceWorkspace || std::is_same<W, HipHostWorkspace<T>>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  HipAllreduceRingChunked(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                          int count,
                          const std::vector<hydra_stream_t>& streams = std::vector<hydra_stream_t>())
      : ctx_(context), ptrs_(ptrs), count_(count), bytes_((size_t)count * sizeof(T)),
        synchronize_outputs_(streams.empty()) {
    using detail::enforce;
    if (ptrs_.empty()) throw EnforceNotMet("HipAllreduceRingChunked: no pointers");
    if (count_ < 0) throw EnforceNotMet("HipAllreduceRingChunked: negative count");
    if (!streams.empty() && streams.size() != ptrs_.size())
      throw EnforceNotMet("HipAllreduceRingChunked: streams.size() != ptrs.size()");
    const size_t chunks = 2 * (size_t)ctx_->size;  // cuda_allreduce_ring_chunked.cc:57-60
    chunk_ = std::max<size_t>(256, ((size_t)count_ + chunks - 1) / chunks);
    if (count_ == 0) return;
    dev_ = detail::pointer_devices(ptrs_, "HipAllreduceRingChunked");
    device_ = dev_[0];  // the tree's root: the ring runs on ptrs[0]'s device
    if (streams.empty()) {
      owned_.resize(ptrs_.size());
      for (size_t i = 0; i < owned_.size(); i++) enforce(hydra_stream_create(dev_[i], &owned_[i]));
      streams_ = owned_;
    } else {
      streams_ = streams;
    }
    if (ptrs_.size() > 1) local_.init(detail::local_tree(dev_, detail::peer_access), dev_, bytes_);
    scratch_host_ = detail::Pinned(bytes_);
    inbox_[0] = detail::Pinned(chunk_ * sizeof(T));
    inbox_[1] = detail::Pinned(chunk_ * sizeof(T));
    if (kDeviceWorkspace) inbox_dev_ = detail::DeviceMem(device_, chunk_ * sizeof(T));
  }

  ~HipAllreduceRingChunked() {
    // outputs may still be copying from pinned scratch on the caller's streams: wait for the
    // fence events run() recorded (not the streams) before the pinned / device buffers are freed
    fence_.wait_nothrow();
    for (auto s : owned_) hydra_stream_destroy(s);
  }
  HipAllreduceRingChunked(const HipAllreduceRingChunked&) = delete;
  HipAllreduceRingChunked& operator=(const HipAllreduceRingChunked&) = delete;

  void run() {
    using detail::enforce;
    if (count_ == 0) return;
    const int dt = gloo_compat::dtype_of<T>();
    hydra_stream_t s0 = streams_[0];
    // CudaLocalNativeReduce tree, in place, each step on its destination's device and stream
    local_.run(std::vector<void*>(ptrs_.begin(), ptrs_.end()), streams_, dt, count_, bytes_);
    char* const dscratch = reinterpret_cast<char*>(ptrs_[0]);
    char* const hscratch = static_cast<char*>(scratch_host_.p);
    enforce(hydra_memcpy_async(hscratch, dscratch, bytes_, s0));
    enforce(hydra_stream_synchronize(s0));
    if (ctx_->size > 1) {
      if (!kDeviceWorkspace)
        lease_.reset(new gloo_compat::ContextPool::Lease(
            gloo_compat::ContextPool::instance(device_).acquire()));
      auto fold = [&](char* dst, const char* box, size_t n) {
        if (!kDeviceWorkspace) {
          enforce(hydra_reduce_host(lease_->get(), HYDRA_SUM, dt, dst, dst, box, n));
          return;
        }
        char* dev = dscratch + (dst - hscratch);
        enforce(hydra_memcpy_async(inbox_dev_.p, box, n * sizeof(T), s0));
        enforce(hydra_reduce(HYDRA_SUM, dt, dev, dev, inbox_dev_.p, n, s0));
        enforce(hydra_memcpy_async(dst, dev, n * sizeof(T), s0));  // what the next send reads
        enforce(hydra_stream_synchronize(s0));
      };
      auto copy = [&](char* dst, const char* box, size_t n) {
        std::memcpy(dst, box, n * sizeof(T));
        if (kDeviceWorkspace) {
          enforce(hydra_memcpy_async(dscratch + (dst - hscratch), box, n * sizeof(T), s0));
          enforce(hydra_stream_synchronize(s0));  // the inbox is reused two steps later
        }
      };
      detail::chunked_ring(*ctx_, hscratch, (size_t)count_, sizeof(T), chunk_,
                           static_cast<char*>(inbox_[0].p), static_cast<char*>(inbox_[1].p),
                           kSlot, fold, copy);
      lease_.reset();
    }
    // broadcast (cudaDeviceBroadcast): every pointer gets the result on its own stream
    if (kDeviceWorkspace) {
      enforce(hydra_stream_synchronize(s0));
      for (size_t i = 1; i < ptrs_.size(); i++)
        enforce(hydra_memcpy_async(ptrs_[i], dscratch, bytes_, streams_[i]));
    } else {
      for (size_t i = 0; i < ptrs_.size(); i++)
        enforce(hydra_memcpy_async(ptrs_[i], hscratch, bytes_, streams_[i]));
    }
    fence_.record(dev_, streams_);
    if (synchronize_outputs_)
      for (auto s : streams_) enforce(hydra_stream_synchronize(s));
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x14) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  size_t bytes_, chunk_ = 0;
  bool synchronize_outputs_;
  int device_ = -1;
  std::vector<int> dev_;  // per pointer
  std::vector<hydra_stream_t> streams_, owned_;
  detail::Pinned scratch_host_, inbox_[2];
  detail::DeviceMem inbox_dev_;
  detail::LocalReduce local_;
  std::unique_ptr<gloo_compat::ContextPool::Lease> lease_;
  detail::OutputFence fence_;  // declared last: destroyed first, before any scratch
};

}  // namespace hydra
