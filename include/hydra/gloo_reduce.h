// include/hydra/gloo_reduce.h -- header-only C++ shim: libhydra_hip.so behind Gloo's
// reduction plug-points.  Drop-in for a Gloo/hydra build (no Gloo headers needed here: the
// shim produces the exact callable shapes Gloo consumes).
//
//   gloo::AllreduceOptions::Func = std::function<void(void*, const void*, const void*, size_t)>
//       (gloo/gloo/allreduce.h:36, set with setReduceFunction :179-181, called at
//        allreduce.cc:301-305 with c == a == out[0]+recvOffset, b == tmp scratch)
//     -> hydra::gloo_compat::hostSum<T>()      host buffers (what gloo's ring hands over):
//                                               staged H2D -> gfx950 kernel -> D2H, synchronous
//     -> hydra::gloo_compat::deviceSum<T>(s)   device buffers, enqueued on stream s
//   gloo::ReductionFunction<T>::Function = void(T*, const T*, size_t)  (algorithm.h:59-96)
//     -> hydra::gloo_compat::hostSumInPlace<T>  (for ReductionFunction<T>{SUM, &fn})
//   gloo::CudaReductionFunction<T> device fn  void(T*, const T*, size_t, stream) (cuda.h:286-350)
//     -> hydra::gloo_compat::deviceSumInPlace<T>
//
// Errors: a non-zero hydra status is handed to an error policy, a template parameter of every
// shim (`Errors`, default HYDRA_GLOO_ERRORS):
//   HYDRA_ERR_TIMEOUT           -> Errors::io_failed      (gloo: IoException, common/error.h:45,
//                                                           as tcp/unbound_buffer.cc:80-84 throws)
//   any other non-zero status   -> Errors::enforce_failed (gloo: EnforceNotMet, as GLOO_ENFORCE,
//                                                           common/logging.h:21,42)
// DefaultErrors throws this header's own EnforceNotMet / IoException (no Gloo headers needed).
// A caller built against Gloo includes include/hydra/gloo_errors.h INSTEAD: it makes
// GlooErrors -- gloo::EnforceNotMet and gloo::IoException themselves -- the default, so a
// reference caller's existing `catch (const gloo::EnforceNotMet&)` sees the shim's failures.
// Threading: staging contexts come from a process-wide pool (one per concurrent caller), so the
// two rails of bew_allreduce_a (pipeallreduce-a.cc:32-50) reduce concurrently without sharing.
#pragma once
#define HYDRA_GLOO_REDUCE_H_INCLUDED 1

#include <cstddef>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../hydra_hip.h"

namespace hydra {
namespace gloo_compat {

class EnforceNotMet : public std::runtime_error {
 public:
  EnforceNotMet(int code, const std::string& what)
      : std::runtime_error("[hydra_hip] " + what + " (status " + std::to_string(code) + ")"),
        code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

class IoException : public std::runtime_error {
 public:
  IoException(int code, const std::string& what)
      : std::runtime_error("[hydra_hip] " + what), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

// The error policy's shape: [[noreturn]] static hooks taking the status, hydra_last_error() and
// the failing call's text.
struct DefaultErrors {
  [[noreturn]] static void enforce_failed(int code, const std::string& msg, const char* call) {
    (void)call;
    throw EnforceNotMet(code, msg);
  }
  [[noreturn]] static void io_failed(int code, const std::string& msg, const char* call) {
    (void)call;
    throw IoException(code, msg);
  }
};

#ifndef HYDRA_GLOO_ERRORS
#define HYDRA_GLOO_ERRORS ::hydra::gloo_compat::DefaultErrors
#endif

template <typename Errors = HYDRA_GLOO_ERRORS>
inline void enforce(int rc, const char* call = "hydra_hip call") {
  if (rc == HYDRA_OK) return;
  const std::string msg = hydra_last_error();
  if (rc == HYDRA_ERR_TIMEOUT) Errors::io_failed(rc, msg, call);
  Errors::enforce_failed(rc, msg, call);
}

// dtype tag of a C++ element type (gloo::float16 is a 2-byte struct: pass HYDRA_FLOAT16 via
// the explicit overloads below; bf16 likewise).
template <typename T>
constexpr int dtype_of() {
  static_assert(std::is_arithmetic<T>::value, "use the explicit-dtype overloads for f16/bf16");
  return std::is_same<T, float>::value      ? HYDRA_FLOAT32
         : std::is_same<T, double>::value   ? HYDRA_FLOAT64
         : std::is_same<T, int8_t>::value   ? HYDRA_INT8
         : std::is_same<T, uint8_t>::value  ? HYDRA_UINT8
         : std::is_same<T, int32_t>::value  ? HYDRA_INT32
         : std::is_same<T, uint32_t>::value ? HYDRA_UINT32
         : std::is_same<T, int64_t>::value  ? HYDRA_INT64
         : std::is_same<T, uint64_t>::value ? HYDRA_UINT64
         : (sizeof(T) == 8 && std::is_unsigned<T>::value) ? HYDRA_UINT64
         : (sizeof(T) == 8) ? HYDRA_INT64
                            : -1;
}

// Staging contexts for host-resident buffers: a process-wide pool.  A reduce call takes a free
// context for its duration, so concurrent callers (the two rails of bew_allreduce_a) never share
// one, and callers on short-lived threads (apipe_allreduce spawns its rail threads per call,
// pipeallreduce-a.cc:32-50) reuse contexts instead of creating device buffers every time.
class ContextPool {
 public:
  class Lease {
   public:
    Lease(ContextPool* p, hydra_ctx_t c) : p_(p), c_(c) {}
    Lease(Lease&& o) noexcept : p_(o.p_), c_(o.c_) { o.c_ = nullptr; }
    Lease(const Lease&) = delete;
    Lease& operator=(const Lease&) = delete;
    ~Lease() {
      if (c_) p_->release(c_);
    }
    hydra_ctx_t get() const { return c_; }

   private:
    ContextPool* p_;
    hydra_ctx_t c_;
  };

  static ContextPool& instance(int device = 0) {
    // one pool per device and process; deliberately never destroyed: at process exit the HIP
    // runtime may already be torn down, so no HIP call may run then
    static std::mutex* m = new std::mutex;
    static std::map<int, ContextPool*>* pools = new std::map<int, ContextPool*>;
    std::lock_guard<std::mutex> g(*m);
    ContextPool*& p = (*pools)[device];
    if (!p) p = new ContextPool(device);
    return *p;
  }
  template <typename Errors = HYDRA_GLOO_ERRORS>
  Lease acquire() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        hydra_ctx_t c = free_.back();
        free_.pop_back();
        return Lease(this, c);
      }
    }
    hydra_ctx_t c = nullptr;
    enforce<Errors>(hydra_ctx_create(device_, &c), "hydra_ctx_create");
    return Lease(this, c);
  }
 private:
  explicit ContextPool(int device) : device_(device) {}
  void release(hydra_ctx_t c) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(c);
  }
  int device_;
  std::mutex mu_;
  std::vector<hydra_ctx_t> free_;
};

// Pinned host allocations (hipHostMalloc) for receive slots the GPU reducer reads in place;
// pinnedAlloc returns null when no GPU is present (the caller then falls back to the heap).
inline void* pinnedAlloc(size_t bytes) {
  void* p = nullptr;
  return hydra_malloc_host(bytes, &p) == HYDRA_OK ? p : nullptr;
}
inline void pinnedFree(void* p) { hydra_free_host(p); }

using Func = std::function<void(void*, const void*, const void*, size_t)>;

// --- AllreduceOptions::Func ------------------------------------------------------------------
template <typename Errors = HYDRA_GLOO_ERRORS>
Func hostReduce(int op, int dtype, int device = 0) {
  return [op, dtype, device](void* c, const void* a, const void* b, size_t n) {
    auto lease = ContextPool::instance(device).acquire<Errors>();
    enforce<Errors>(hydra_reduce_host(lease.get(), op, dtype, c, a, b, n), "hydra_reduce_host");
  };
}

template <typename T, typename Errors = HYDRA_GLOO_ERRORS>
Func hostSum(int device = 0) {
  return hostReduce<Errors>(HYDRA_SUM, dtype_of<T>(), device);
}

template <typename Errors = HYDRA_GLOO_ERRORS>
Func deviceReduce(int op, int dtype, hydra_stream_t stream = nullptr) {
  return [op, dtype, stream](void* c, const void* a, const void* b, size_t n) {
    enforce<Errors>(hydra_reduce(op, dtype, c, a, b, n, stream), "hydra_reduce");
  };
}

template <typename T, typename Errors = HYDRA_GLOO_ERRORS>
Func deviceSum(hydra_stream_t stream = nullptr) {
  return deviceReduce<Errors>(HYDRA_SUM, dtype_of<T>(), stream);
}

// --- ReductionFunction<T>::Function (x = op(x, y)) ---------------------------------------------
template <typename T, typename Errors = HYDRA_GLOO_ERRORS>
void hostSumInPlace(T* x, const T* y, size_t n) {
  auto lease = ContextPool::instance().acquire<Errors>();
  enforce<Errors>(hydra_reduce_host(lease.get(), HYDRA_SUM, dtype_of<T>(), x, x, y, n),
                  "hydra_reduce_host");
}

// Explicit-dtype form for element types that are not C++ arithmetic types: gloo::float16 (a
// 2-byte struct, HYDRA_FLOAT16, with its store quirk) or a bf16 struct (HYDRA_BFLOAT16).
template <typename T, int DTYPE, typename Errors = HYDRA_GLOO_ERRORS>
void hostSumInPlaceAs(T* x, const T* y, size_t n) {
  static_assert(DTYPE == HYDRA_FLOAT16 || DTYPE == HYDRA_BFLOAT16 || sizeof(T) != 2,
                "2-byte element types need HYDRA_FLOAT16 or HYDRA_BFLOAT16");
  auto lease = ContextPool::instance().acquire<Errors>();
  enforce<Errors>(hydra_reduce_host(lease.get(), HYDRA_SUM, DTYPE, x, x, y, n),
                  "hydra_reduce_host");
}

// --- an old-style ReductionFunction<T> whose fn is the GPU sum ------------------------------
// Works for gloo::ReductionFunction<T> (algorithm.h:59-96) and hydra::ReductionFunction<T>
// (include/hydra/allreduce.h):  gpuReductionFunction<gloo::ReductionFunction<float>, float>(
// gloo::SUM)  ->  a pointer usable wherever ReductionFunction<float>::sum is.
template <typename RF, typename T, typename Errors = HYDRA_GLOO_ERRORS, typename Enum>
const RF* gpuReductionFunction(Enum sum) {
  static const RF fn(sum, &hostSumInPlace<T, Errors>);
  return &fn;
}

// the same for explicit-dtype element types, e.g.
//   gpuReductionFunctionAs<gloo::ReductionFunction<gloo::float16>, gloo::float16, HYDRA_FLOAT16>(
//       gloo::SUM)
template <typename RF, typename T, int DTYPE, typename Errors = HYDRA_GLOO_ERRORS, typename Enum>
const RF* gpuReductionFunctionAs(Enum sum) {
  static const RF fn(sum, &hostSumInPlaceAs<T, DTYPE, Errors>);
  return &fn;
}

// --- CudaReductionFunction<T> device function shape (x = op(x, y) on a stream) ---------------
template <typename T, typename Errors = HYDRA_GLOO_ERRORS>
void deviceSumInPlace(T* x, const T* y, size_t n, hydra_stream_t stream) {
  enforce<Errors>(hydra_reduce(HYDRA_SUM, dtype_of<T>(), x, x, y, n, stream), "hydra_reduce");
}

}  // namespace gloo_compat
}  // namespace hydra
