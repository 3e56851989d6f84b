// oracle/ref_harness.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
//
// A thin extern "C" driver around the *reference's own* hot-path code, compiled straight from
// the sources under /root/reference/gloo by oracle/Makefile into oracle/_ref/libgloo_ref.so.
// Nothing here re-implements the reference: every result comes from the reference's functions
//   gloo::sum/product/max/min<T>   gloo/gloo/math.h:15-73
//   gloo::allreduce (ring, bcube)  gloo/gloo/allreduce.cc:99-422
//   gloo::reduce (ring + gather)   gloo/gloo/reduce.cc:21-262
//   rendezvous + TCP loopback      gloo/gloo/rendezvous/context.cc:32-69, transport/tcp/*
// driven the way the reference's own tests drive them (thread per rank, in-process HashStore,
// one shared TCP device on the loopback interface: gloo/gloo/test/base_test.h:73-156).
//
// Used only by oracle/gen_golden.py (golden fixtures, this container), tests/ (cross-checks) and
// bench.py's cpu_baseline leg (kind "reference").

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gloo/allreduce.h"
#include "gloo/common/error.h"
#include "gloo/math.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo/types.h"

namespace {

// dtype codes: identical numbering to include/hydra_hip.h (hydra_dtype_t).
enum {
  D_INT8 = 0, D_UINT8 = 1, D_INT32 = 2, D_UINT32 = 3, D_INT64 = 4, D_UINT64 = 5,
  D_FLOAT32 = 6, D_FLOAT64 = 7, D_FLOAT16 = 8,
};
// op codes: identical numbering to hydra_op_t.
enum { OP_SUM = 0, OP_PRODUCT = 1, OP_MAX = 2, OP_MIN = 3 };

using Fn = void (*)(void*, const void*, const void*, size_t);

template <typename T>
Fn pick(int op) {
  switch (op) {
    case OP_SUM: return &gloo::sum<T>;
    case OP_PRODUCT: return &gloo::product<T>;
    case OP_MAX: return &gloo::max<T>;
    case OP_MIN: return &gloo::min<T>;
  }
  return nullptr;
}

Fn lookup(int op, int dtype, size_t* esize) {
  switch (dtype) {
    case D_INT8: *esize = 1; return pick<int8_t>(op);
    case D_UINT8: *esize = 1; return pick<uint8_t>(op);
    case D_INT32: *esize = 4; return pick<int32_t>(op);
    case D_UINT32: *esize = 4; return pick<uint32_t>(op);
    case D_INT64: *esize = 8; return pick<int64_t>(op);
    case D_UINT64: *esize = 8; return pick<uint64_t>(op);
    case D_FLOAT32: *esize = 4; return pick<float>(op);
    case D_FLOAT64: *esize = 8; return pick<double>(op);
    case D_FLOAT16: *esize = 2; return pick<gloo::float16>(op);
  }
  return nullptr;
}

void set_err(char* err, size_t len, const std::string& s) {
  if (err && len) {
    std::strncpy(err, s.c_str(), len - 1);
    err[len - 1] = 0;
  }
}

std::shared_ptr<gloo::transport::Device> loopback_device() {
  gloo::transport::tcp::attr attr;
  attr.hostname = "127.0.0.1";
  return gloo::transport::tcp::CreateDevice(attr);
}

// Typed setInputs/setOutputs: AllreduceOptions only takes typed pointers (allreduce.h:116-177).
template <typename T>
void set_bufs(gloo::AllreduceOptions& o, void** in, void** out, int nptr, size_t n) {
  std::vector<T*> o_ptrs, i_ptrs;
  for (int i = 0; i < nptr; i++) o_ptrs.push_back(static_cast<T*>(out[i]));
  o.setOutputs(o_ptrs, n);
  if (in) {
    for (int i = 0; i < nptr; i++) i_ptrs.push_back(static_cast<T*>(in[i]));
    o.setInputs(i_ptrs, n);
  }
}

void set_bufs_dt(int dtype, gloo::AllreduceOptions& o, void** in, void** out, int nptr, size_t n) {
  switch (dtype) {
    case D_INT8: set_bufs<int8_t>(o, in, out, nptr, n); break;
    case D_UINT8: set_bufs<uint8_t>(o, in, out, nptr, n); break;
    case D_INT32: set_bufs<int32_t>(o, in, out, nptr, n); break;
    case D_UINT32: set_bufs<uint32_t>(o, in, out, nptr, n); break;
    case D_INT64: set_bufs<int64_t>(o, in, out, nptr, n); break;
    case D_UINT64: set_bufs<uint64_t>(o, in, out, nptr, n); break;
    case D_FLOAT32: set_bufs<float>(o, in, out, nptr, n); break;
    case D_FLOAT64: set_bufs<double>(o, in, out, nptr, n); break;
    case D_FLOAT16: set_bufs<gloo::float16>(o, in, out, nptr, n); break;
  }
}

// Run fn(rank, context) on P threads sharing one HashStore + loopback device (base_test.h:116-156).
int spawn(int P, const std::function<void(int, std::shared_ptr<gloo::Context>)>& fn,
          char* err, size_t errlen) {
  gloo::rendezvous::HashStore store;
  auto dev = loopback_device();
  std::vector<std::thread> threads;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  std::string first_err;
  for (int r = 0; r < P; r++) {
    threads.emplace_back([&, r]() {
      std::shared_ptr<gloo::rendezvous::Context> ctx;
      try {
        ctx = std::make_shared<gloo::rendezvous::Context>(r, P);
        ctx->connectFullMesh(store, dev);
        fn(r, ctx);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        if (first_err.empty()) first_err = e.what();
      }
      // every rank finishes before any connection closes (base_test.h:142-155)
      std::unique_lock<std::mutex> l(mu);
      arrived++;
      cv.notify_all();
      cv.wait(l, [&] { return arrived == P; });
    });
  }
  for (auto& t : threads) t.join();
  if (!first_err.empty()) {
    set_err(err, errlen, first_err);
    return 1;
  }
  return 0;
}

}  // namespace

extern "C" {

// c[i] = op(a[i], b[i]) through the reference's own gloo::{sum,product,max,min}<T>.
int ref_op(int op, int dtype, void* c, const void* a, const void* b, size_t n) {
  size_t es = 0;
  Fn f = lookup(op, dtype, &es);
  if (!f) return 1;
  f(c, a, b, n);
  return 0;
}

int ref_sum(int dtype, void* c, const void* a, const void* b, size_t n) {
  return ref_op(OP_SUM, dtype, c, a, b, n);
}

// Reference fp32<->fp16 conversions (gloo/gloo/types.h:207-290).
unsigned short ref_float2half(float f) { return gloo::cpu_float2half_rn(f).x; }
float ref_half2float(unsigned short h) {
  gloo::float16 v;
  v.x = h;
  return gloo::cpu_half2float(v);
}

// One gloo::allreduce over P thread-ranks.  in/out are P*nptr pointers laid out [rank][ptr];
// in == NULL means in-place on out (allreduce_test.cc:302-350).  algorithm: 1 RING, 2 BCUBE.
int ref_allreduce(int P, int nptr, int op, int dtype, size_t n, void** in, void** out,
                  size_t max_segment, int algorithm, long timeout_ms, char* err, size_t errlen) {
  size_t es = 0;
  Fn f = lookup(op, dtype, &es);
  if (!f) return 2;
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    gloo::AllreduceOptions o(ctx);
    o.setAlgorithm(static_cast<gloo::AllreduceOptions::Algorithm>(algorithm));
    set_bufs_dt(dtype, o, in ? in + r * nptr : nullptr, out + r * nptr, nptr, n);
    o.setReduceFunction(f);
    if (max_segment) o.setMaxSegmentSize(max_segment);
    if (timeout_ms > 0) o.setTimeout(std::chrono::milliseconds(timeout_ms));
    gloo::allreduce(o);
  }, err, errlen);
}

// Timeout semantics probe (allreduce_test.cc:381-397): rank 0 runs an allreduce with a short
// timeout while rank 1 never joins.  Returns 0 and copies the exception text if IoException.
int ref_allreduce_timeout(long timeout_ms, char* what, size_t len) {
  int rc = 3;
  spawn(2, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    if (r != 0) return;
    uint64_t buf = 0;
    gloo::AllreduceOptions o(ctx);
    o.setOutput(&buf, 1);
    o.setReduceFunction(Fn(&gloo::sum<uint64_t>));
    o.setTimeout(std::chrono::milliseconds(timeout_ms));
    try {
      gloo::allreduce(o);
    } catch (const gloo::IoException& e) {
      set_err(what, len, e.what());
      rc = 0;
    }
  }, nullptr, 0);
  return rc;
}

// Single-thread timing of the reference reduction on caller buffers: best-of `reps` seconds per
// call, `iters` calls per rep.  c may alias a (in place, as the ring calls it: allreduce.cc:301).
double ref_time_op(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                   int iters, int reps) {
  size_t es = 0;
  Fn f = lookup(op, dtype, &es);
  if (!f) return -1.0;
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) f(c, a, b, n);
    auto t1 = std::chrono::steady_clock::now();
    double s = std::chrono::duration<double>(t1 - t0).count() / iters;
    if (s < best) best = s;
  }
  return best;
}

// The reference's own new_allreduce_ring benchmark body (benchmark/main.cc:321-358, one input
// per rank, out-of-place, RING, gloo::sum<float>) on P loopback thread-ranks; per-iteration wall
// time of rank 0 in ns goes to samples_ns[iters] (runner.cc:683-702).
int ref_bench_ring(int P, size_t n, int warmup, int iters, double* samples_ns, char* err,
                   size_t errlen) {
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    std::vector<float> in(n), out(n);
    for (size_t j = 0; j < n; j++) in[j] = float(j * P + r);
    gloo::AllreduceOptions o(ctx);
    o.setInput(in.data(), n);
    o.setOutput(out.data(), n);
    o.setAlgorithm(gloo::AllreduceOptions::Algorithm::RING);
    o.setReduceFunction(Fn(&gloo::sum<float>));
    for (int i = 0; i < warmup; i++) gloo::allreduce(o);
    for (int i = 0; i < iters; i++) {
      auto t0 = std::chrono::steady_clock::now();
      gloo::allreduce(o);
      auto t1 = std::chrono::steady_clock::now();
      if (r == 0) samples_ns[i] = std::chrono::duration<double, std::nano>(t1 - t0).count();
    }
  }, err, errlen);
}

}  // extern "C"

// AllreduceOptions::Func-shaped handle on the reference's own gloo::sum<float> (math.h:15-23),
// so the host runtime's bench can use the reference reduction as its CPU baseline reducer.
extern "C" void ref_sum_f32(void* c, const void* a, const void* b, size_t n) {
  gloo::sum<float>(c, a, b, n);
}

// ---- old-style AllreduceRing<T> (gloo/gloo/allreduce_ring.h:20-125), §8f row 3 ------------
#include "gloo/allreduce_ring.h"

namespace {
template <typename T>
int run_old_ring(int P, int nptr, size_t n, void** bufs, char* err, size_t errlen) {
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    gloo::AllreduceRing<T> algo(ctx, ptrs, (int)n, gloo::ReductionFunction<T>::sum);
    algo.run();
  }, err, errlen);
}
}  // namespace

// ---- AllreduceRingChunked<T> (gloo/gloo/allreduce_ring_chunked.h:20-248) -----------------
#include "gloo/allreduce_ring_chunked.h"

namespace {
template <typename T>
int run_chunked_ring(int P, int nptr, size_t n, void** bufs, char* err, size_t errlen) {
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    gloo::AllreduceRingChunked<T> algo(ctx, ptrs, (int)n, gloo::ReductionFunction<T>::sum);
    algo.run();
  }, err, errlen);
}
}  // namespace

extern "C" int ref_allreduce_ring_chunked(int P, int nptr, int dtype, size_t n, void** bufs,
                                          char* err, size_t errlen) {
  switch (dtype) {
    case D_FLOAT32: return run_chunked_ring<float>(P, nptr, n, bufs, err, errlen);
    case D_INT32: return run_chunked_ring<int32_t>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT16: return run_chunked_ring<gloo::float16>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT64: return run_chunked_ring<double>(P, nptr, n, bufs, err, errlen);
  }
  return 2;
}

// ---- AllreduceHalvingDoubling<T> (gloo/gloo/allreduce_halving_doubling.h:37-411) ----------
#include "gloo/allreduce_halving_doubling.h"

namespace {
template <typename T>
int run_halving_doubling(int P, int nptr, size_t n, void** bufs, char* err, size_t errlen) {
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    gloo::AllreduceHalvingDoubling<T> algo(ctx, ptrs, (int)n, gloo::ReductionFunction<T>::sum);
    algo.run();
  }, err, errlen);
}
}  // namespace

extern "C" int ref_allreduce_halving_doubling(int P, int nptr, int dtype, size_t n, void** bufs,
                                              char* err, size_t errlen) {
  switch (dtype) {
    case D_FLOAT32: return run_halving_doubling<float>(P, nptr, n, bufs, err, errlen);
    case D_INT32: return run_halving_doubling<int32_t>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT16: return run_halving_doubling<gloo::float16>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT64: return run_halving_doubling<double>(P, nptr, n, bufs, err, errlen);
  }
  return 2;
}

// ---- old-style AllreduceBcube<T> (gloo/gloo/allreduce_bcube.h) ---------------------------
#include "gloo/allreduce_bcube.h"

namespace {
template <typename T>
int run_bcube_old(int P, int nptr, size_t n, void** bufs, char* err, size_t errlen) {
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    gloo::AllreduceBcube<T> algo(ctx, ptrs, (int)n, gloo::ReductionFunction<T>::sum);
    algo.run();
  }, err, errlen);
}
}  // namespace

extern "C" int ref_allreduce_bcube_old(int P, int nptr, int dtype, size_t n, void** bufs,
                                       char* err, size_t errlen) {
  switch (dtype) {
    case D_FLOAT32: return run_bcube_old<float>(P, nptr, n, bufs, err, errlen);
    case D_INT32: return run_bcube_old<int32_t>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT16: return run_bcube_old<gloo::float16>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT64: return run_bcube_old<double>(P, nptr, n, bufs, err, errlen);
  }
  return 2;
}

// In place on bufs ([rank][ptr]), ReductionFunction<T>::sum; dtype: float32, int32, float16.
extern "C" int ref_allreduce_ring_old(int P, int nptr, int dtype, size_t n, void** bufs,
                                      char* err, size_t errlen) {
  switch (dtype) {
    case D_FLOAT32: return run_old_ring<float>(P, nptr, n, bufs, err, errlen);
    case D_INT32: return run_old_ring<int32_t>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT16: return run_old_ring<gloo::float16>(P, nptr, n, bufs, err, errlen);
    case D_FLOAT64: return run_old_ring<double>(P, nptr, n, bufs, err, errlen);
  }
  return 2;
}

// ---- new-style gloo::reduce (gloo/gloo/reduce.cc:21-262): the other caller of the Func ---
#include "gloo/reduce.h"

namespace {
template <typename T>
void set_reduce_bufs(gloo::ReduceOptions& o, void* in, void* out, size_t n) {
  if (in) o.setInput(static_cast<T*>(in), n);
  o.setOutput(static_cast<T*>(out), n);
}
}  // namespace

// One gloo::reduce to `root` over P thread-ranks.  in/out are P pointers (in == NULL: in
// place on out, reduce_test.cc:27-33).  Every rank's out is left as the reference leaves it.
extern "C" int ref_reduce(int P, int op, int dtype, size_t n, void** in, void** out, int root,
                          size_t max_segment, long timeout_ms, char* err, size_t errlen) {
  size_t es = 0;
  Fn f = lookup(op, dtype, &es);
  if (!f) return 2;
  return spawn(P, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    gloo::ReduceOptions o(ctx);
    void* ip = in ? in[r] : nullptr;
    switch (dtype) {
      case D_INT8: set_reduce_bufs<int8_t>(o, ip, out[r], n); break;
      case D_UINT8: set_reduce_bufs<uint8_t>(o, ip, out[r], n); break;
      case D_INT32: set_reduce_bufs<int32_t>(o, ip, out[r], n); break;
      case D_UINT32: set_reduce_bufs<uint32_t>(o, ip, out[r], n); break;
      case D_INT64: set_reduce_bufs<int64_t>(o, ip, out[r], n); break;
      case D_UINT64: set_reduce_bufs<uint64_t>(o, ip, out[r], n); break;
      case D_FLOAT32: set_reduce_bufs<float>(o, ip, out[r], n); break;
      case D_FLOAT64: set_reduce_bufs<double>(o, ip, out[r], n); break;
      case D_FLOAT16: set_reduce_bufs<gloo::float16>(o, ip, out[r], n); break;
    }
    o.setRoot(root);
    o.setReduceFunction(f);
    if (max_segment) o.setMaxSegmentSize(max_segment);
    if (timeout_ms > 0) o.setTimeout(std::chrono::milliseconds(timeout_ms));
    gloo::reduce(o);
  }, err, errlen);
}

// ReduceTest.TestTimeout (reduce_test.cc:91-108): root 0 alone with a 10 ms timeout.
extern "C" int ref_reduce_timeout(long timeout_ms, char* what, size_t len) {
  int rc = 3;
  spawn(2, [&](int r, std::shared_ptr<gloo::Context> ctx) {
    if (r != 0) return;
    uint64_t buf = 0;
    gloo::ReduceOptions o(ctx);
    o.setOutput(&buf, 1);
    o.setRoot(0);
    o.setReduceFunction(Fn(&gloo::sum<uint64_t>));
    o.setTimeout(std::chrono::milliseconds(timeout_ms));
    try {
      gloo::reduce(o);
    } catch (const gloo::IoException& e) {
      set_err(what, len, e.what());
      rc = 0;
    }
  }, nullptr, 0);
  return rc;
}
