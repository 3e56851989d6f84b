// include/hydra/allreduce.h -- C++ host runtime mirroring hydra/Gloo's new-style allreduce API
// for the bucket-reduction path (libhydra_host.so, built with g++; talks to the GPU only through
// the C-ABI in include/hydra_hip.h).
//
// Mirrors (same names, argument meaning and error behaviour):
//   gloo::Context(rank, size) + rendezvous::Context::connectFullMesh   gloo/gloo/context.h:26-58,
//                                                                       rendezvous/context.cc:32-69
//   gloo::AllreduceOptions {setInput(s), setOutput(s), setReduceFunction, setAlgorithm, setTag,
//                           setMaxSegmentSize, setTimeout}          gloo/gloo/allreduce.h:89-199
//   gloo::allreduce(opts)  (RING; P==1 short circuit)                 gloo/gloo/allreduce.cc:99-422
//   gloo::APipeAllreduceOptions / apipe_allreduce (bew_allreduce_a)   gloo/gloo/pipeallreduce-a.h:32-397,
//                                                                       pipeallreduce-a.cc:27-61
//   gloo::EnforceNotMet / gloo::IoException ("Timed out ...")        common/logging.h:21, common/error.h:45
// Transport: loopback/LAN TCP, one reader and one writer thread per pair, FIFO per pair,
// receives land directly in the posted buffer (gloo/gloo/transport/tcp/pair.cc:486-533 idea).
#pragma once

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>


namespace hydra {

class EnforceNotMet : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

class IoException : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// ---- rendezvous stores (HashStore: threads of one process; FileStore: processes) ----------
class Store {
 public:
  virtual ~Store() = default;
  virtual void set(const std::string& key, const std::string& value) = 0;
  virtual std::string get(const std::string& key, std::chrono::milliseconds timeout) = 0;
};

class HashStore : public Store {
 public:
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key, std::chrono::milliseconds timeout) override;

 private:
  std::mutex mu_;
  std::map<std::string, std::string> kv_;
};

class FileStore : public Store {
 public:
  explicit FileStore(std::string dir) : dir_(std::move(dir)) {}
  void set(const std::string& key, const std::string& value) override;
  std::string get(const std::string& key, std::chrono::milliseconds timeout) override;

 private:
  std::string dir_;
};

namespace transport {
class Pair;
class Device;
}  // namespace transport

// A buffer registered with the context: non-owning (ptr, size) view that can be the source of
// sends and the target of receives (gloo::transport::UnboundBuffer, unbound_buffer.h:32-120).
class UnboundBuffer {
 public:
  UnboundBuffer(class Context* ctx, void* ptr, size_t size) : ctx_(ctx), ptr(ptr), size(size) {}
  ~UnboundBuffer();
  void send(int dst, uint64_t slot, size_t offset, size_t nbytes);
  void recv(int src, uint64_t slot, size_t offset, size_t nbytes);
  void waitSend(std::chrono::milliseconds timeout);  // oldest outstanding send completes
  void waitRecv(std::chrono::milliseconds timeout);  // oldest outstanding recv completes

  Context* const ctx_;
  void* const ptr;
  const size_t size;

  struct Op;
  std::mutex mu_;
  std::vector<std::shared_ptr<Op>> sends_, recvs_;
};

class Context {
 public:
  Context(int rank, int size);
  ~Context();
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;

  // Full mesh over TCP on `host` (ephemeral ports published through the store under `prefix`).
  void connectFullMesh(Store& store, const std::string& host = "127.0.0.1",
                       const std::string& prefix = "hydra");
  std::unique_ptr<UnboundBuffer> createUnboundBuffer(void* ptr, size_t size) {
    return std::unique_ptr<UnboundBuffer>(new UnboundBuffer(this, ptr, size));
  }
  // Where the ring's receive slots live (the reference news them per call, allreduce.cc:
  // 225-229).  Default: the heap.  With a pinned allocator (gloo_compat::pinnedAlloc/Free) the
  // TCP receives land in page-locked memory that the GPU reducer reads in place over PCIe
  // (hydra_reduce_host's zero-copy path) instead of staging it -- SURVEY §8f row 1.  The buffer
  // is cached per context and reused by later collectives on it.
  struct ScratchAllocator {
    void* (*alloc)(size_t) = nullptr;
    void (*release)(void*) = nullptr;
  };
  void setScratchAllocator(ScratchAllocator a);
  char* scratch(size_t bytes);
  void setTimeout(std::chrono::milliseconds t) { timeout_ = t; }
  std::chrono::milliseconds getTimeout() const { return timeout_; }
  transport::Pair* getPair(int peer);
  void closeConnections();
  // A timed-out or failed operation poisons the whole context, as the reference's
  // context_->signalException does (gloo/gloo/transport/tcp/unbound_buffer.cc:66-76): every pair
  // fails its pending operations with `msg`, closes its socket and joins its threads, so no
  // late peer message can land in a buffer the caller is about to free; later operations on the
  // context fail at once.
  void signalException(const std::string& msg);

  const int rank;
  const int size;

 private:
  std::chrono::milliseconds timeout_{30000};  // gloo/gloo/context.cc:18
  std::vector<std::unique_ptr<transport::Pair>> pairs_;
  ScratchAllocator scratch_alloc_;
  void* scratch_ = nullptr;
  size_t scratch_bytes_ = 0;
  bool scratch_heap_ = true;
  void releaseScratch();
};

class AllreduceOptions {
 public:
  using Func = std::function<void(void*, const void*, const void*, size_t)>;
  enum Algorithm { UNSPECIFIED = 0, RING = 1, BCUBE = 2 };
  static constexpr size_t kMaxSegmentSize = 1024 * 1024;  // allreduce.h:78

  explicit AllreduceOptions(const std::shared_ptr<Context>& context)
      : context(context), timeout(context->getTimeout()) {}

  void setAlgorithm(Algorithm a) { algorithm = a; }
  template <typename T>
  void setInput(T* ptr, size_t n) { setInputs(&ptr, 1, n); }
  template <typename T>
  void setInputs(std::vector<T*> ptrs, size_t n) { setInputs(ptrs.data(), ptrs.size(), n); }
  template <typename T>
  void setInputs(T** ptrs, size_t len, size_t n) {
    setBufs(in, reinterpret_cast<void**>(ptrs), len, n, sizeof(T));
  }
  template <typename T>
  void setOutput(T* ptr, size_t n) { setOutputs(&ptr, 1, n); }
  template <typename T>
  void setOutputs(std::vector<T*> ptrs, size_t n) { setOutputs(ptrs.data(), ptrs.size(), n); }
  template <typename T>
  void setOutputs(T** ptrs, size_t len, size_t n) {
    setBufs(out, reinterpret_cast<void**>(ptrs), len, n, sizeof(T));
  }
  // untyped forms (element size explicit), for C callers
  void setInputsRaw(void** ptrs, size_t len, size_t n, size_t esize) {
    setBufs(in, ptrs, len, n, esize);
  }
  void setOutputsRaw(void** ptrs, size_t len, size_t n, size_t esize) {
    setBufs(out, ptrs, len, n, esize);
  }
  void setReduceFunction(Func fn) { reduce = std::move(fn); }
  void setTag(uint32_t t) { tag = t; }
  void setMaxSegmentSize(size_t s) { maxSegmentSize = s; }
  void setTimeout(std::chrono::milliseconds t) { timeout = t; }

  std::shared_ptr<Context> context;
  std::chrono::milliseconds timeout;
  Algorithm algorithm = UNSPECIFIED;
  std::vector<std::unique_ptr<UnboundBuffer>> in, out;
  size_t elements = 0, elementSize = 0;
  Func reduce;
  uint32_t tag = 0;
  size_t maxSegmentSize = kMaxSegmentSize;

 private:
  void setBufs(std::vector<std::unique_ptr<UnboundBuffer>>& v, void** ptrs, size_t len, size_t n,
               size_t esize) {
    elements = n;
    elementSize = esize;
    v.clear();
    for (size_t i = 0; i < len; i++) v.push_back(context->createUnboundBuffer(ptrs[i], n * esize));
  }
};

void allreduce(const AllreduceOptions& opts);

// ---- new-style reduce to a root (gloo/gloo/reduce.h:20-110, reduce.cc:21-262) -------------
// The other new-style caller of the reduce function (reduce.cc:195): a ring reduce-scatter
// with reduce(out + off, in + off, tmp, n), then every rank sends its chunk to the root.  Only
// the root's output is defined; the other ranks' outputs hold what the reference's schedule
// leaves there (reproduced too).
class ReduceOptions {
 public:
  using Func = AllreduceOptions::Func;
  static constexpr size_t kMaxSegmentSize = 1024 * 1024;  // reduce.h:92

  explicit ReduceOptions(const std::shared_ptr<Context>& context)
      : context(context), timeout(context->getTimeout()) {}

  template <typename T>
  void setInput(T* ptr, size_t n) { setInputRaw(ptr, n, sizeof(T)); }
  template <typename T>
  void setOutput(T* ptr, size_t n) { setOutputRaw(ptr, n, sizeof(T)); }
  void setInputRaw(void* ptr, size_t n, size_t esize) {
    elements = n;
    elementSize = esize;
    in = context->createUnboundBuffer(ptr, n * esize);
  }
  void setOutputRaw(void* ptr, size_t n, size_t esize) {
    elements = n;
    elementSize = esize;
    out = context->createUnboundBuffer(ptr, n * esize);
  }
  void setRoot(int r) { root = r; }
  void setReduceFunction(Func fn) { reduce = std::move(fn); }
  void setTag(uint32_t t) { tag = t; }
  void setMaxSegmentSize(size_t s) { maxSegmentSize = s; }
  void setTimeout(std::chrono::milliseconds t) { timeout = t; }

  std::shared_ptr<Context> context;
  std::chrono::milliseconds timeout;
  std::unique_ptr<UnboundBuffer> in, out;
  size_t elements = 0, elementSize = 0;
  int root = -1;
  Func reduce;
  uint32_t tag = 0;
  size_t maxSegmentSize = kMaxSegmentSize;
};

void reduce(ReduceOptions& opts);

// ---- bew_allreduce_a: the buffer split over two rails, two concurrent rings ----------------
enum class SplitTable { AA, AG };  // calculateElements_AA (default) / _AG (env ALLREDUCE_GLEX)
void calculateElements(SplitTable t, int P, size_t n, size_t* e1, size_t* e2);

class APipeAllreduceOptions {
 public:
  APipeAllreduceOptions(const std::shared_ptr<Context>& context,
                        const std::shared_ptr<Context>& context2)
      : opts3(context), opts2(context2), size_(context->size) {}
  template <typename T>
  void setInput(T* ptr, size_t n) { setSplit(reinterpret_cast<char*>(ptr), n, sizeof(T), true); }
  template <typename T>
  void setOutput(T* ptr, size_t n) { setSplit(reinterpret_cast<char*>(ptr), n, sizeof(T), false); }
  void setInputRaw(void* p, size_t n, size_t es) { setSplit(static_cast<char*>(p), n, es, true); }
  void setOutputRaw(void* p, size_t n, size_t es) { setSplit(static_cast<char*>(p), n, es, false); }
  void setReduceFunction(AllreduceOptions::Func fn) {
    opts2.setReduceFunction(fn);
    opts3.setReduceFunction(fn);
  }
  void setAlgorithm(AllreduceOptions::Algorithm a) {
    opts2.setAlgorithm(a);
    opts3.setAlgorithm(a);
  }
  void setSplitTable(SplitTable t) { table_ = t; }

  AllreduceOptions opts3;  // rail 1: elements [0, e1) on `context`   (pipeallreduce-a.h:51-53)
  AllreduceOptions opts2;  // rail 2: elements [e1, n) on `context2`

 private:
  void setSplit(char* p, size_t n, size_t es, bool input);
  int size_;
  SplitTable table_ = SplitTable::AA;
};

void apipe_allreduce(APipeAllreduceOptions& opts);

// ---- old-style Algorithm API (gloo/gloo/algorithm.h:20-96, allreduce_ring.h:20-125) --------
enum ReductionType { SUM = 1, PRODUCT = 2, MAX = 3, MIN = 4, CUSTOM = 1000 };

// gloo::ReductionFunction<T>: a (type, fn) pair, fn(x, y, n) computes x = op(x, y).  hydra's
// GPU instances come from include/hydra/gloo_reduce.h (gpuReductionFunction<T>()).
template <typename T>
class ReductionFunction {
 public:
  using Function = void(T*, const T*, size_t);
  ReductionFunction(ReductionType type, Function* fn) : type_(type), fn_(fn) {}
  ReductionType type() const { return type_; }
  void call(T* x, const T* y, size_t n) const { fn_(x, y, n); }

 private:
  ReductionType type_;
  Function* fn_;
};

// gloo::AllreduceRing<T>: P-1 rounds, each sends the full outbox to rank+1 and folds the inbox
// from rank-1 into ptrs[0] (x = x op inbox), so rank r ends with x_r op x_{r-1} op ... (its own
// left fold -- ranks differ in the last bits for floats, exactly like the reference).  The
// reference's notification handshake (allreduce_ring.h:97-103) is implicit here: a receive is
// only posted once this rank's inbox is free, and the FIFO transport holds the sender's bytes.
template <typename T>
class AllreduceRing {
 public:
  AllreduceRing(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, int count,
                const ReductionFunction<T>* fn)
      : ctx_(context), ptrs_(ptrs), count_(count), bytes_((size_t)count * sizeof(T)), fn_(fn) {
    if (!fn_) throw EnforceNotMet("AllreduceRing: null reduction function");
    if (ptrs_.empty()) throw EnforceNotMet("AllreduceRing: no pointers");
    boxes_[0].resize(bytes_);
    boxes_[1].resize(bytes_);
  }

  void run() {
    for (size_t i = 1; i < ptrs_.size(); i++) fn_->call(ptrs_[0], ptrs_[i], count_);
    const int P = ctx_->size;
    if (P > 1 && count_ > 0) {
      const int right = (ctx_->rank + 1) % P, left = (ctx_->rank + P - 1) % P;
      std::memcpy(boxes_[0].data(), ptrs_[0], bytes_);  // outbox = local value
      int out = 0;
      for (int round = 0; round < P - 1; round++) {
        auto ob = ctx_->createUnboundBuffer(boxes_[out].data(), bytes_);
        auto ib = ctx_->createUnboundBuffer(boxes_[out ^ 1].data(), bytes_);
        ib->recv(left, kSlot, 0, bytes_);
        ob->send(right, kSlot, 0, bytes_);
        ib->waitRecv(ctx_->getTimeout());
        fn_->call(ptrs_[0], reinterpret_cast<const T*>(boxes_[out ^ 1].data()), count_);
        ob->waitSend(ctx_->getTimeout());
        out ^= 1;  // next round forwards what was just received (allreduce_ring.h:92-94)
      }
    }
    for (size_t i = 1; i < ptrs_.size(); i++) std::memcpy(ptrs_[i], ptrs_[0], bytes_);
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x10) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  size_t bytes_;
  const ReductionFunction<T>* fn_;
  std::vector<char> boxes_[2];
};

// gloo::AllreduceRingChunked<T> (allreduce_ring_chunked.h:20-248): 2P chunks of
// max(256, ceil(count/2P)) elements.  Rank r seeds chunks 2r and 2r+1; each later step i
// (reduce pass rounds 2..2P-1, then broadcast pass rounds 0..2P-3) receives chunk co(i) from
// rank-1 into inbox[i&1], folds it into ptrs[0] (x = x op inbox) or, in the broadcast pass,
// copies it, and forwards that chunk to rank+1.  Every rank ends with the same bits: chunk c,
// seeded by s = c/2, is x_{s-1} op (x_{s-2} op (... op x_s)).  The reference's notification
// handshake is implicit (a receive is posted only once its inbox is free; the transport holds
// early bytes), and empty chunks move nothing instead of the reference's 1-element
// placeholder (:218-225), which its receiver ignores.
namespace detail {
// AllreduceRingChunked's schedule (allreduce_ring_chunked.h:77-200) over `count` elements of
// `es` bytes at `base` (host memory the transport sends from): 2P chunks of `chunk` elements,
// two inboxes of `chunk` elements, a reduce pass whose steps call fold(dst, box, n) (dst op=
// box) and a broadcast pass whose steps call copy(dst, box, n).  Shared by the host class
// and HipAllreduceRingChunked<T, W> (cuda_allreduce_ring_chunked.cc), which differ only in
// where the fold runs.
template <typename Fold, typename Copy>
void chunked_ring(Context& ctx, char* base, size_t count, size_t es, size_t chunk, char* inbox0,
                  char* inbox1, uint64_t slot, Fold fold, Copy copy) {
  const int P = ctx.size, r = ctx.rank;
  if (P <= 1 || count == 0) return;
  const int right = (r + 1) % P, left = (r + P - 1) % P;
  const int C = 2 * P, steps = 2 * C - 4;
  const auto tmo = ctx.getTimeout();
  auto out = ctx.createUnboundBuffer(base, count * es);
  char* inbox[2] = {inbox0, inbox1};
  std::unique_ptr<UnboundBuffer> in[2] = {ctx.createUnboundBuffer(inbox0, chunk * es),
                                          ctx.createUnboundBuffer(inbox1, chunk * es)};
  std::vector<char> sent(steps, 0);
  auto chunk_of = [&](int i) {  // chunk received at step i
    const int round = i < C - 2 ? i + 2 : i - (C - 2);
    return ((2 * r) - (round & ~1) + (round & 1) + C) % C;
  };
  auto len_of = [&](int co) {
    const size_t off = (size_t)co * chunk;
    return off >= count ? (size_t)0 : std::min(chunk, count - off);
  };
  auto post_recv = [&](int i) {
    const size_t l = len_of(chunk_of(i));
    if (l) in[i & 1]->recv(left, slot, 0, l * es);
  };
  auto post_send = [&](int i, int co) {
    const size_t l = len_of(co);
    if (l) out->send(right, slot, (size_t)co * chunk * es, l * es);
    sent[i] = l != 0;
  };
  int waited = 0;  // sends completed in order (waitSend pops the oldest)
  auto wait_sends_through = [&](int i) {
    for (; waited <= i && waited < steps; waited++)
      if (sent[waited]) out->waitSend(tmo);
  };
  post_recv(0);
  post_recv(1);
  post_send(0, 2 * r);
  post_send(1, 2 * r + 1);
  for (int i = 0; i < steps; i++) {
    const int co = chunk_of(i);
    const size_t l = len_of(co);
    char* dst = base + (size_t)co * chunk * es;
    if (l) {
      in[i & 1]->waitRecv(tmo);
      wait_sends_through(i);  // a still-queued send of this chunk must not see the update
      if (i < C - 2) fold(dst, inbox[i & 1], l);
      else copy(dst, inbox[i & 1], l);
    }
    if (i + 2 < steps) {
      post_recv(i + 2);  // inbox[i&1] is free again
      post_send(i + 2, co);
    }
  }
  wait_sends_through(steps - 1);
}
}  // namespace detail

template <typename T>
class AllreduceRingChunked {
 public:
  AllreduceRingChunked(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                       int count, const ReductionFunction<T>* fn)
      : ctx_(context), ptrs_(ptrs), count_(count), fn_(fn) {
    if (!fn_) throw EnforceNotMet("AllreduceRingChunked: null reduction function");
    if (ptrs_.empty()) throw EnforceNotMet("AllreduceRingChunked: no pointers");
    if (count_ < 0) throw EnforceNotMet("AllreduceRingChunked: negative count");
    chunks_ = 2 * (size_t)ctx_->size;
    chunk_ = std::max<size_t>(256, ((size_t)count_ + chunks_ - 1) / chunks_);
    for (auto& b : inbox_) b.resize(chunk_ * sizeof(T));
  }

  void run() {
    const size_t bytes = (size_t)count_ * sizeof(T);
    for (size_t i = 1; i < ptrs_.size(); i++) fn_->call(ptrs_[0], ptrs_[i], count_);
    detail::chunked_ring(
        *ctx_, reinterpret_cast<char*>(ptrs_[0]), (size_t)count_, sizeof(T), chunk_,
        inbox_[0].data(), inbox_[1].data(), kSlot,
        [this](char* dst, const char* box, size_t l) {
          fn_->call(reinterpret_cast<T*>(dst), reinterpret_cast<const T*>(box), l);
        },
        [](char* dst, const char* box, size_t l) { std::memcpy(dst, box, l * sizeof(T)); });
    for (size_t i = 1; i < ptrs_.size(); i++) std::memcpy(ptrs_[i], ptrs_[0], bytes);
  }

 private:
  static constexpr uint64_t kSlot = uint64_t(0x11) << 56;
  std::shared_ptr<Context> ctx_;
  std::vector<T*> ptrs_;
  int count_;
  const ReductionFunction<T>* fn_;
  size_t chunks_ = 0, chunk_ = 0;
  std::vector<char> inbox_[2];
};

}  // namespace hydra
