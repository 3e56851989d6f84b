// include/hydra/hip_allreduce_extra.h -- OUT OF SCOPE, opt-in: the HIP-workspace twins of the
// Algorithm-API classes in allreduce_extra.h (SURVEY.md §2 "Other Gloo collectives").  Kept with
// their tests (pytest marker `extra`, HYDRA_EXTRA_TESTS=1); not part of the default build, test
// run or bench:
//   HipAllreduceBcube<T, W>           gloo/gloo/cuda_allreduce_bcube.cc:111-200, 358-410
//   HipAllreduceLocal<T>              gloo/gloo/cuda_allreduce_local.cc:17-66
//   HipAllreduceHalvingDoubling<T, W> gloo/gloo/cuda_allreduce_halving_doubling.cc:246-408
#pragma once

#include "allreduce_extra.h"
#include "hip_allreduce_ring.h"

namespace hydra {

// hydra::HipAllreduceBcube<T, W> -- gloo::CudaAllreduceBcube<T, W> (cuda_allreduce_bcube.cc:
// 111-200, 358-410): the local reduce into a pinned scratch (host workspace: cudaHostReduce's
// left fold in pointer order below kOnDeviceThreshold = 256 KiB, algorithm.cc:16, else
// cudaDeviceReduce's pairwise tree; device workspace: the tree), then the old-style
// AllreduceBcube schedule (the BCUBE schedule for P a power of two, row a17) on the scratch with
// every fold (scratch op= received, :151) on the gfx950 kernel, then every pointer gets the
// result.  Other P are refused as by hydra::AllreduceBcube<T>.
template <typename T, typename W>
class HipAllreduceBcube {
  static constexpr bool kDeviceWorkspace = std::is_same<W, HipDeviceWorkspace<T>>::value;
  static_assert(kDeviceWorkspace || std::is_same<W, HipHostWorkspace<T>>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");
  static constexpr size_t kOnDeviceThreshold = 256 * 1024;  // algorithm.cc:16

 public:
  HipAllreduceBcube(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                    int count,
                    const std::vector<hydra_stream_t>& streams = std::vector<hydra_stream_t>())
      : ctx_(context), ptrs_(ptrs), count_(count), bytes_((size_t)count * sizeof(T)),
        synchronize_outputs_(streams.empty()) {
    using detail::enforce;
    if (ptrs_.empty()) throw EnforceNotMet("HipAllreduceBcube: no pointers");
    if (count_ < 0) throw EnforceNotMet("HipAllreduceBcube: negative count");
    if (ctx_->size & (ctx_->size - 1))
      throw EnforceNotMet("HipAllreduceBcube: the number of ranks must be a power of the base (2)");
    if (!streams.empty() && streams.size() != ptrs_.size())
      throw EnforceNotMet("HipAllreduceBcube: streams.size() != ptrs.size()");
    if (count_ == 0) return;
    enforce(hydra_pointer_device(ptrs_[0], &device_));
    if (device_ < 0) throw EnforceNotMet("HipAllreduceBcube: ptrs must be device memory");
    for (T* p : ptrs_) {
      int d = -1;
      enforce(hydra_pointer_device(p, &d));
      if (d != device_)
        throw EnforceNotMet("HipAllreduceBcube: all pointers must be on one device");
    }
    if (streams.empty()) {
      owned_.resize(ptrs_.size());
      for (auto& s : owned_) enforce(hydra_stream_create(device_, &s));
      streams_ = owned_;
    } else {
      streams_ = streams;
    }
    scratch_host_ = detail::Pinned(bytes_);
    local_dev_ = detail::DeviceMem(device_, bytes_);
    if (kDeviceWorkspace) inbox_dev_ = detail::DeviceMem(device_, bytes_);
  }

  ~HipAllreduceBcube() {
    // outputs may still be copying from pinned scratch on the caller's streams: wait for the
    // fence events run() recorded (not the streams) before the pinned / device buffers are freed
    fence_.wait_nothrow();
    for (auto s : owned_) hydra_stream_destroy(s);
  }
  HipAllreduceBcube(const HipAllreduceBcube&) = delete;
  HipAllreduceBcube& operator=(const HipAllreduceBcube&) = delete;

  void run() {
    using detail::enforce;
    if (count_ == 0) return;
    const int dt = gloo_compat::dtype_of<T>();
    hydra_stream_t s0 = streams_[0];
    for (size_t i = 1; i < streams_.size(); i++) enforce(hydra_stream_synchronize(streams_[i]));
    // ---- local reduce into a device copy (the inputs stay untouched until the broadcast)
    char* const dscratch = static_cast<char*>(local_dev_.p);
    enforce(hydra_memcpy_async(dscratch, ptrs_[0], bytes_, s0));
    if (!kDeviceWorkspace && bytes_ < kOnDeviceThreshold) {  // cudaHostReduce: left fold
      for (size_t i = 1; i < ptrs_.size(); i++)
        enforce(hydra_reduce(HYDRA_SUM, dt, dscratch, dscratch, ptrs_[i], count_, s0));
    } else {  // cudaDeviceReduce: pairwise tree; operand j is ptrs[j] (dscratch for j = 0)
      std::vector<const void*> v(ptrs_.begin(), ptrs_.end());
      std::vector<void*> out(ptrs_.size(), nullptr);
      out[0] = dscratch;
      v[0] = dscratch;
      for (size_t sz = 1; sz < ptrs_.size(); sz *= 2)
        for (size_t j = 0; j + sz < ptrs_.size(); j += 2 * sz) {
          if (!out[j]) {  // never write the caller's inputs: fold into a device temporary
            temps_.emplace_back(new detail::DeviceMem(device_, bytes_));
            out[j] = temps_.back()->p;
          }
          enforce(hydra_reduce(HYDRA_SUM, dt, out[j], v[j], v[j + sz], count_, s0));
          v[j] = out[j];
        }
    }
    char* const hscratch = static_cast<char*>(scratch_host_.p);
    enforce(hydra_memcpy_async(hscratch, dscratch, bytes_, s0));
    enforce(hydra_stream_synchronize(s0));
    temps_.clear();
    if (ctx_->size > 1) {
      if (!kDeviceWorkspace)
        lease_.reset(new gloo_compat::ContextPool::Lease(
            gloo_compat::ContextPool::instance(device_).acquire()));
      AllreduceOptions opts(ctx_);
      opts.setAlgorithm(AllreduceOptions::BCUBE);
      opts.setOutput(reinterpret_cast<T*>(hscratch), (size_t)count_);
      opts.setReduceFunction([&](void* c, const void* a, const void* b, size_t n) {
        if (!kDeviceWorkspace) {
          enforce(hydra_reduce_host(lease_->get(), HYDRA_SUM, dt, c, a, b, n));
          return;
        }
        // folds only touch regions no all-gather copy has written: the device copy is current
        char* dev = dscratch + (static_cast<const char*>(a) - hscratch);
        enforce(hydra_memcpy_async(inbox_dev_.p, b, n * sizeof(T), s0));
        enforce(hydra_reduce(HYDRA_SUM, dt, dev, dev, inbox_dev_.p, n, s0));
        enforce(hydra_memcpy_async(c, dev, n * sizeof(T), s0));
        enforce(hydra_stream_synchronize(s0));
      });
      allreduce(opts);
      lease_.reset();
    }
    for (size_t i = 0; i < ptrs_.size(); i++)
      enforce(hydra_memcpy_async(ptrs_[i], hscratch, bytes_, streams_[i]));
    fence_.record(device_, streams_);
    if (synchronize_outputs_)
      for (auto s : streams_) enforce(hydra_stream_synchronize(s));
  }

 private:
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  size_t bytes_;
  bool synchronize_outputs_;
  int device_ = -1;
  std::vector<hydra_stream_t> streams_, owned_;
  detail::Pinned scratch_host_;
  detail::DeviceMem local_dev_, inbox_dev_;
  std::vector<std::unique_ptr<detail::DeviceMem>> temps_;
  std::unique_ptr<gloo_compat::ContextPool::Lease> lease_;
  detail::OutputFence fence_;  // declared last: destroyed first, before any scratch
};

// hydra::HipAllreduceLocal<T> -- gloo::CudaAllreduceLocal<T> (cuda_allreduce_local.cc:17-66):
// the device pointers of one process reduced into ptrs[0] by the pairwise tree of
// cudaDeviceReduce (cuda_collectives_device.h:29-56) on the gfx950 kernel, then copied to every
// pointer on its stream (cudaDeviceBroadcast).  No communication; outputs are synchronized
// unless the caller passes streams.
template <typename T>
class HipAllreduceLocal {
 public:
  HipAllreduceLocal(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                    int count,
                    const std::vector<hydra_stream_t>& streams = std::vector<hydra_stream_t>())
      : ctx_(context), ptrs_(ptrs), count_(count), synchronize_outputs_(streams.empty()) {
    using detail::enforce;
    if (count_ < 0) throw EnforceNotMet("HipAllreduceLocal: negative count");
    if (!streams.empty() && streams.size() != ptrs_.size())
      throw EnforceNotMet("HipAllreduceLocal: streams.size() != ptrs.size()");
    if (count_ == 0 || ptrs_.size() < 2) return;
    for (T* p : ptrs_) {
      int d = -1;
      enforce(hydra_pointer_device(p, &d));
      if (d < 0) throw EnforceNotMet("HipAllreduceLocal: ptrs must be device memory");
      if (device_ >= 0 && d != device_)
        throw EnforceNotMet("HipAllreduceLocal: all pointers must be on one device");
      device_ = d;
    }
    if (streams.empty()) {
      owned_.resize(ptrs_.size());
      for (auto& s : owned_) enforce(hydra_stream_create(device_, &s));
      streams_ = owned_;
    } else {
      streams_ = streams;
    }
  }
  ~HipAllreduceLocal() {
    // outputs may still be copying from pinned scratch on the caller's streams: wait for the
    // fence events run() recorded (not the streams) before the pinned / device buffers are freed
    fence_.wait_nothrow();
    for (auto s : owned_) hydra_stream_destroy(s);
  }
  HipAllreduceLocal(const HipAllreduceLocal&) = delete;
  HipAllreduceLocal& operator=(const HipAllreduceLocal&) = delete;

  void run() {
    using detail::enforce;
    if (count_ == 0 || ptrs_.size() < 2) return;
    const int dt = gloo_compat::dtype_of<T>();
    hydra_stream_t s0 = streams_[0];
    for (size_t i = 1; i < streams_.size(); i++) enforce(hydra_stream_synchronize(streams_[i]));
    for (size_t sz = 1; sz < ptrs_.size(); sz *= 2)
      for (size_t j = 0; j + sz < ptrs_.size(); j += 2 * sz)
        enforce(hydra_reduce(HYDRA_SUM, dt, ptrs_[j], ptrs_[j], ptrs_[j + sz], count_, s0));
    enforce(hydra_stream_synchronize(s0));
    for (size_t i = 1; i < ptrs_.size(); i++)
      enforce(hydra_memcpy_async(ptrs_[i], ptrs_[0], (size_t)count_ * sizeof(T), streams_[i]));
    fence_.record(device_, streams_);
    if (synchronize_outputs_)
      for (auto s : streams_) enforce(hydra_stream_synchronize(s));
  }

 private:
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  bool synchronize_outputs_;
  int device_ = -1;
  std::vector<hydra_stream_t> streams_, owned_;
  detail::OutputFence fence_;  // declared last: destroyed first, before any scratch
};

// hydra::HipAllreduceHalvingDoubling<T, W> -- the analog of gloo::CudaAllreduceHalvingDoubling
// <T, W> (gloo/gloo/cuda_allreduce_halving_doubling.cc:246-408, non-pipelined): the local reduce
// on the device as the reference picks it (host workspace below kOnDeviceThreshold = 256 KiB:
// cudaHostReduce's left fold, :478-481; otherwise cudaDeviceReduce's pairwise tree), then
// AllreduceHalvingDoubling's schedule
// (detail::halving_doubling, shared with the host class) on a pinned host copy of the bucket,
// every fold (scratch op= received, :282-285, :299-302) on the gfx950 kernel -- zero-copy on
// the pinned box (host workspace) or on the device copy after an H2D of the box (device
// workspace).  Received finished pieces are copies (:340-341, :370-373).  Every pointer ends
// with the pinned copy's bits, identical on every rank.
template <typename T, typename W>
class HipAllreduceHalvingDoubling {
  static constexpr bool kDeviceWorkspace = std::is_same<W, HipDeviceWorkspace<T>>::value;
  static_assert(kDeviceWorkspace || std::is_same<W, HipHostWorkspace<T>>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");
  static constexpr size_t kOnDeviceThreshold = 256 * 1024;  // algorithm.cc:16

 public:
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context,
                              const std::vector<T*>& ptrs, int count,
                              const std::vector<hydra_stream_t>& streams =
                                  std::vector<hydra_stream_t>())
      : ctx_(context), ptrs_(ptrs), count_(count), bytes_((size_t)count * sizeof(T)),
        synchronize_outputs_(streams.empty()),
        geo_(context->size, context->rank, count < 0 ? 0 : (size_t)count) {
    using detail::enforce;
    if (ptrs_.empty()) throw EnforceNotMet("HipAllreduceHalvingDoubling: no pointers");
    if (count_ < 0) throw EnforceNotMet("HipAllreduceHalvingDoubling: negative count");
    if (!streams.empty() && streams.size() != ptrs_.size())
      throw EnforceNotMet("HipAllreduceHalvingDoubling: streams.size() != ptrs.size()");
    if (count_ == 0) return;
    enforce(hydra_pointer_device(ptrs_[0], &device_));
    if (device_ < 0)
      throw EnforceNotMet("HipAllreduceHalvingDoubling: ptrs must be device memory");
    for (T* p : ptrs_) {
      int d = -1;
      enforce(hydra_pointer_device(p, &d));
      if (d != device_)
        throw EnforceNotMet("HipAllreduceHalvingDoubling: all pointers must be on one device");
    }
    if (streams.empty()) {
      owned_.resize(ptrs_.size());
      for (auto& s : owned_) enforce(hydra_stream_create(device_, &s));
      streams_ = owned_;
    } else {
      streams_ = streams;
    }
    scratch_host_ = detail::Pinned(bytes_);
    const size_t box = std::max<size_t>(geo_.inbox_elems(), 1) * sizeof(T);
    inbox_ = detail::Pinned(box);
    if (kDeviceWorkspace) inbox_dev_ = detail::DeviceMem(device_, box);
  }

  ~HipAllreduceHalvingDoubling() {
    // outputs may still be copying from pinned scratch on the caller's streams: wait for the
    // fence events run() recorded (not the streams) before the pinned / device buffers are freed
    fence_.wait_nothrow();
    for (auto s : owned_) hydra_stream_destroy(s);
  }
  HipAllreduceHalvingDoubling(const HipAllreduceHalvingDoubling&) = delete;
  HipAllreduceHalvingDoubling& operator=(const HipAllreduceHalvingDoubling&) = delete;

  void run() {
    using detail::enforce;
    if (count_ == 0) return;
    const int dt = gloo_compat::dtype_of<T>();
    hydra_stream_t s0 = streams_[0];
    for (size_t i = 1; i < streams_.size(); i++) enforce(hydra_stream_synchronize(streams_[i]));
    if (!kDeviceWorkspace && bytes_ < kOnDeviceThreshold) {  // cudaHostReduce: left fold (:478-481)
      for (size_t i = 1; i < ptrs_.size(); i++)
        enforce(hydra_reduce(HYDRA_SUM, dt, ptrs_[0], ptrs_[0], ptrs_[i], count_, s0));
    } else {  // cudaDeviceReduce's pairwise tree, in place (the outputs are overwritten anyway)
      for (size_t sz = 1; sz < ptrs_.size(); sz *= 2)
        for (size_t j = 0; j + sz < ptrs_.size(); j += 2 * sz)
          enforce(hydra_reduce(HYDRA_SUM, dt, ptrs_[j], ptrs_[j], ptrs_[j + sz], count_, s0));
    }
    char* const dscratch = reinterpret_cast<char*>(ptrs_[0]);
    char* const hscratch = static_cast<char*>(scratch_host_.p);
    enforce(hydra_memcpy_async(hscratch, dscratch, bytes_, s0));
    enforce(hydra_stream_synchronize(s0));
    if (ctx_->size > 1) {
      if (!kDeviceWorkspace)
        lease_.reset(new gloo_compat::ContextPool::Lease(
            gloo_compat::ContextPool::instance(device_).acquire()));
      // Folds only ever touch regions no copy has written yet, so the device copy is current
      // wherever the device workspace folds.
      auto fold = [&](char* dst, const char* box, size_t n) {
        if (!kDeviceWorkspace) {
          enforce(hydra_reduce_host(lease_->get(), HYDRA_SUM, dt, dst, dst, box, n));
          return;
        }
        char* dev = dscratch + (dst - hscratch);
        enforce(hydra_memcpy_async(inbox_dev_.p, box, n * sizeof(T), s0));
        enforce(hydra_reduce(HYDRA_SUM, dt, dev, dev, inbox_dev_.p, n, s0));
        enforce(hydra_memcpy_async(dst, dev, n * sizeof(T), s0));  // what later sends read
        enforce(hydra_stream_synchronize(s0));
      };
      detail::halving_doubling(*ctx_, geo_, hscratch, (size_t)count_, sizeof(T),
                               static_cast<char*>(inbox_.p), kSlot, fold);
      lease_.reset();
    }
    // broadcast (localBroadcastOp_): every pointer gets the pinned copy's result
    for (size_t i = 0; i < ptrs_.size(); i++)
      enforce(hydra_memcpy_async(ptrs_[i], hscratch, bytes_, streams_[i]));
    fence_.record(device_, streams_);
    if (synchronize_outputs_)
      for (auto s : streams_) enforce(hydra_stream_synchronize(s));
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x15) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  size_t bytes_;
  bool synchronize_outputs_;
  detail::HalvingDoublingGeometry geo_;
  int device_ = -1;
  std::vector<hydra_stream_t> streams_, owned_;
  detail::Pinned scratch_host_, inbox_;
  detail::DeviceMem inbox_dev_;
  std::unique_ptr<gloo_compat::ContextPool::Lease> lease_;
  detail::OutputFence fence_;  // declared last: destroyed first, before any scratch
};

}  // namespace hydra
