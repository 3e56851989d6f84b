// host_capi.cpp -- extern "C" drivers of the host runtime (include/hydra_host.h).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/hydra/allreduce.h"
#include "../../../include/hydra/gloo_reduce.h"
#include "../../../include/hydra/hip_allreduce_ring.h"
#include "../../../include/hydra_host.h"
#include "capi_util.h"

using hydra::capi::esize_of;
using hydra::capi::make_reducer;
using hydra::capi::set_err;
using hydra::capi::spawn;

namespace {
template <typename T>
const hydra::ReductionFunction<T>* reduction_function(int reducer, hydra_inplace_fn fn,
                                                      std::unique_ptr<hydra::ReductionFunction<T>>* custom) {
  using RF = hydra::ReductionFunction<T>;
  if (reducer == HYDRA_REDUCER_FN) {
    if (!fn) return nullptr;
    custom->reset(new RF(hydra::CUSTOM, reinterpret_cast<typename RF::Function*>(fn)));
    return custom->get();
  }
  return hydra::gloo_compat::gpuReductionFunction<RF, T>(hydra::SUM);
}

template <typename T>
int old_ring(int kind, int P, int nptr, size_t n, void** bufs, int reducer, hydra_inplace_fn fn,
             char* err, size_t errlen) {  // kind: 0 AllreduceRing, 1 AllreduceRingChunked
  std::unique_ptr<hydra::ReductionFunction<T>> custom;
  const hydra::ReductionFunction<T>* rf = reduction_function<T>(reducer, fn, &custom);
  if (!rf) {
    set_err(err, errlen, "null reduce function");
    return 2;
  }
  return spawn(P, 1, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    if (kind == 1) {
      hydra::AllreduceRingChunked<T> algo(c[0], ptrs, (int)n, rf);
      algo.run();
    } else {
      hydra::AllreduceRing<T> algo(c[0], ptrs, (int)n, rf);
      algo.run();
    }
  });
}
template <typename T>
int hip_ring(int P, int nptr, size_t n, void** bufs, int workspace, int user_streams, char* err,
             size_t errlen, int kind = 0) {  // kind: 0 ring, 1 chunked
  const bool chunked = kind == 1;
  return spawn(P, 1, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    std::vector<hydra_stream_t> streams;
    if (user_streams) {
      int dev = 0;  // an empty bucket may come with null pointers
      if (n) hydra::gloo_compat::enforce(hydra_pointer_device(ptrs[0], &dev));
      streams.resize(nptr);
      for (auto& s : streams) hydra::gloo_compat::enforce(hydra_stream_create(dev, &s));
    }
    if (chunked && workspace == HYDRA_WORKSPACE_DEVICE) {
      hydra::HipAllreduceRingChunked<T, hydra::HipDeviceWorkspace<T>> algo(c[0], ptrs, (int)n,
                                                                           streams);
      algo.run();
    } else if (chunked) {
      hydra::HipAllreduceRingChunked<T, hydra::HipHostWorkspace<T>> algo(c[0], ptrs, (int)n,
                                                                         streams);
      algo.run();
    } else if (workspace == HYDRA_WORKSPACE_DEVICE) {
      hydra::HipAllreduceRing<T, hydra::HipDeviceWorkspace<T>> algo(c[0], ptrs, (int)n, streams);
      algo.run();
    } else {
      hydra::HipAllreduceRing<T, hydra::HipHostWorkspace<T>> algo(c[0], ptrs, (int)n, streams);
      algo.run();
    }
    for (auto s : streams) {  // caller-provided streams: outputs are async until synchronized
      hydra::gloo_compat::enforce(hydra_stream_synchronize(s));
      hydra_stream_destroy(s);
    }
    // the algorithm has been destroyed (its streams, events, pinned and device scratch freed):
    // a device fault first reported here belongs to that teardown
    int dev = 0;
    if (n) hydra::gloo_compat::enforce(hydra_pointer_device(ptrs[0], &dev));
    if (hydra_device_check(dev) != 0)
      throw hydra::EnforceNotMet(std::string("after the algorithm's teardown: ") +
                                 hydra_last_error());
  });
}
}  // namespace

extern "C" {

int hydra_host_allreduce_threads(int P, int nptr, int op, int dtype, size_t n, void** in,
                                 void** out, size_t max_segment, int algorithm, int reducer,
                                 hydra_reduce_fn fn, long timeout_ms, char* err, size_t errlen) {
  const size_t es = esize_of(dtype);
  if (!es || P < 1 || nptr < 1 || !out) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  return spawn(P, 1, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    hydra::AllreduceOptions o(c[0]);
    o.setAlgorithm(static_cast<hydra::AllreduceOptions::Algorithm>(algorithm));
    o.setOutputsRaw(out + r * nptr, nptr, n, es);
    if (in) o.setInputsRaw(in + r * nptr, nptr, n, es);
    int red = reducer;
    if (red == HYDRA_REDUCER_GPU_PINNED) {  // pinned receive slots (zero-copy GPU reduces)
      c[0]->setScratchAllocator({&hydra::gloo_compat::pinnedAlloc, &hydra::gloo_compat::pinnedFree});
      red = HYDRA_REDUCER_GPU;
    }
    o.setReduceFunction(make_reducer(red, op, dtype, fn));
    if (max_segment) o.setMaxSegmentSize(max_segment);
    if (timeout_ms > 0) o.setTimeout(std::chrono::milliseconds(timeout_ms));
    hydra::allreduce(o);
  });
}

int hydra_host_apipe_threads(int P, int dtype, size_t n, void** in, void** out, int table,
                             int reducer, hydra_reduce_fn fn, char* err, size_t errlen) {
  const size_t es = esize_of(dtype);
  if (!es || P < 1 || !out || !in) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  return spawn(P, 2, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    hydra::APipeAllreduceOptions o(c[0], c[1]);
    o.setSplitTable(table == HYDRA_SPLIT_AG ? hydra::SplitTable::AG : hydra::SplitTable::AA);
    o.setInputRaw(in[r], n, es);
    o.setOutputRaw(out[r], n, es);
    o.setAlgorithm(hydra::AllreduceOptions::RING);
    o.setReduceFunction(make_reducer(reducer, HYDRA_SUM, dtype, fn));
    hydra::apipe_allreduce(o);
  });
}

int hydra_host_bench(int config, int P, size_t n, int warmup, int iters, int reducer_mode,
                     hydra_reduce_fn fn, double* samples_ns, char* err, size_t errlen) {
  if ((config != 1 && config != 3) || P < 1 || !samples_ns ||
      (reducer_mode == HYDRA_REDUCER_GPU_PINNED_RANK0 && !fn)) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  return spawn(P, config == 3 ? 2 : 1, err, errlen,
               [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    int reducer = reducer_mode;
    if (reducer == HYDRA_REDUCER_GPU_PINNED_RANK0)
      reducer = r == 0 ? HYDRA_REDUCER_GPU_PINNED : HYDRA_REDUCER_FN;
    // GPU_PINNED: the receive slots and the output are pinned blocks (hydra_malloc_host), so
    // every segment reduce is the zero-copy kernel over PCIe.  (Round 2
    // registered a heap vector instead; hydra registers no transient heap memory any more:
    // DESIGN.md §10.)
    const bool pinned = reducer == HYDRA_REDUCER_GPU_PINNED;
    std::vector<float> in(n), out_heap(pinned ? 0 : n);
    struct PinnedOut {
      float* p = nullptr;
      ~PinnedOut() {
        if (p) hydra_free_host(p);
      }
    } pout;
    if (pinned) {
      for (auto& ctx : c)
        ctx->setScratchAllocator({&hydra::gloo_compat::pinnedAlloc, &hydra::gloo_compat::pinnedFree});
      void* q = nullptr;
      hydra::gloo_compat::enforce(hydra_malloc_host((n ? n : 1) * sizeof(float), &q));
      pout.p = static_cast<float*>(q);
      std::fill(pout.p, pout.p + n, 0.0f);
      reducer = HYDRA_REDUCER_GPU;
    }
    float* out = pinned ? pout.p : out_heap.data();
    auto time_it = [&](const std::function<void()>& run) {
      for (int i = 0; i < warmup; i++) run();
      for (int i = 0; i < iters; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        run();
        const auto t1 = std::chrono::steady_clock::now();
        if (r == 0) samples_ns[i] = std::chrono::duration<double, std::nano>(t1 - t0).count();
      }
    };
    if (config == 1) {  // NewAllreduceBenchmark: in[j] = j*P + r, out of place (main.cc:329-358)
      for (size_t j = 0; j < n; j++) in[j] = float(j * (size_t)P + (size_t)r);
      hydra::AllreduceOptions o(c[0]);
      o.setInput(in.data(), n);
      o.setOutput(out, n);
      o.setAlgorithm(hydra::AllreduceOptions::RING);
      o.setReduceFunction(make_reducer(reducer, HYDRA_SUM, HYDRA_FLOAT32, fn));
      time_it([&] { hydra::allreduce(o); });
    } else {  // aAllreduceBenchmark: in[i] = i*(rank+1.0), out = 0 (main.cc:629-664)
      for (size_t j = 0; j < n; j++) in[j] = float((double)j * (r + 1.0));
      hydra::APipeAllreduceOptions o(c[0], c[1]);
      o.setInput(in.data(), n);
      o.setOutput(out, n);
      o.setAlgorithm(hydra::AllreduceOptions::RING);
      o.setReduceFunction(make_reducer(reducer, HYDRA_SUM, HYDRA_FLOAT32, fn));
      time_it([&] { hydra::apipe_allreduce(o); });
    }
  });
}

static int algorithm_ring(int kind, int P, int nptr, int dtype, size_t n, void** bufs,
                          int reducer, hydra_inplace_fn fn, char* err, size_t errlen) {
  if (P < 1 || nptr < 1 || !bufs || n > (size_t)INT32_MAX) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  switch (dtype) {
    case HYDRA_FLOAT32: return old_ring<float>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_INT32: return old_ring<int32_t>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_FLOAT64: return old_ring<double>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_FLOAT16:
      if (reducer != HYDRA_REDUCER_FN) break;
      return old_ring<uint16_t>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
  }
  set_err(err, errlen, "unsupported dtype for AllreduceRing");
  return 3;
}

int hydra_host_allreduce_ring_old_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                          int reducer, hydra_inplace_fn fn, char* err,
                                          size_t errlen) {
  return algorithm_ring(0, P, nptr, dtype, n, bufs, reducer, fn, err, errlen);
}

int hydra_host_allreduce_ring_chunked_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                              int reducer, hydra_inplace_fn fn, char* err,
                                              size_t errlen) {
  return algorithm_ring(1, P, nptr, dtype, n, bufs, reducer, fn, err, errlen);
}

int hydra_host_hip_ring_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                int workspace, int user_streams, char* err, size_t errlen) {
  if (P < 1 || nptr < 1 || !dev_bufs || n > (size_t)INT32_MAX) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  switch (dtype) {
    case HYDRA_FLOAT32: return hip_ring<float>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
    case HYDRA_INT32: return hip_ring<int32_t>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
    case HYDRA_FLOAT64: return hip_ring<double>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
    case HYDRA_INT64: return hip_ring<int64_t>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
  }
  set_err(err, errlen, "unsupported dtype for HipAllreduceRing");
  return 3;
}

int hydra_host_hip_ring_chunked_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                        int workspace, int user_streams, char* err,
                                        size_t errlen) {
  if (P < 1 || nptr < 1 || !dev_bufs || n > (size_t)INT32_MAX) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  switch (dtype) {
    case HYDRA_FLOAT32:
      return hip_ring<float>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen, 1);
    case HYDRA_INT32:
      return hip_ring<int32_t>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen, 1);
    case HYDRA_FLOAT64:
      return hip_ring<double>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen, 1);
    case HYDRA_INT64:
      return hip_ring<int64_t>(P, nptr, n, dev_bufs, workspace, user_streams, err, errlen, 1);
  }
  set_err(err, errlen, "unsupported dtype for HipAllreduceRingChunked");
  return 3;
}

void hydra_host_calculate_elements(int table, int P, size_t n, size_t* e1, size_t* e2) {
  hydra::calculateElements(table == HYDRA_SPLIT_AG ? hydra::SplitTable::AG : hydra::SplitTable::AA,
                           P, n, e1, e2);
}

int hydra_host_reduce_threads(int P, int op, int dtype, size_t n, void** in, void** out,
                              int root, size_t max_segment, int reducer, hydra_reduce_fn fn,
                              long timeout_ms, char* err, size_t errlen) {
  const size_t es = esize_of(dtype);
  if (!es || P < 1 || !out) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  return spawn(P, 1, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    hydra::ReduceOptions o(c[0]);
    if (in) o.setInputRaw(in[r], n, es);
    o.setOutputRaw(out[r], n, es);
    o.setRoot(root);
    int red = reducer;
    if (red == HYDRA_REDUCER_GPU_PINNED) {
      c[0]->setScratchAllocator({&hydra::gloo_compat::pinnedAlloc, &hydra::gloo_compat::pinnedFree});
      red = HYDRA_REDUCER_GPU;
    }
    o.setReduceFunction(make_reducer(red, op, dtype, fn));
    if (max_segment) o.setMaxSegmentSize(max_segment);
    if (timeout_ms > 0) o.setTimeout(std::chrono::milliseconds(timeout_ms));
    hydra::reduce(o);
  });
}

int hydra_host_reduce_timeout_probe(long timeout_ms, char* what, size_t len) {
  int rc = 3;
  spawn(2, 1, nullptr, 0, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    if (r != 0) return;  // ReduceTest.TestTimeout (reduce_test.cc:91-108): rank 1 never joins
    uint64_t buf = 0;
    hydra::ReduceOptions o(c[0]);
    o.setOutput(&buf, 1);
    o.setRoot(0);
    o.setReduceFunction([](void* x, const void* a, const void* b, size_t n) {
      for (size_t i = 0; i < n; i++)
        static_cast<uint64_t*>(x)[i] =
            static_cast<const uint64_t*>(a)[i] + static_cast<const uint64_t*>(b)[i];
    });
    o.setTimeout(std::chrono::milliseconds(timeout_ms));
    try {
      hydra::reduce(o);
    } catch (const hydra::IoException& e) {
      set_err(what, len, e.what());
      rc = 0;
    }
  });
  return rc;
}

// A SLOW peer (not a dead one): rank 0 times out, rank 1 joins `delay_ms` later and sends its
// data.  Rank 0's context must be poisoned by the timeout (every pair closed, as the reference's
// signalException), so the late bytes land nowhere: rank 0 refills its bucket with a sentinel
// right after the exception and checks it once rank 1 is done.  *intact = 1 when untouched.
int hydra_host_slow_peer_probe(long timeout_ms, long delay_ms, size_t n, char* what, size_t len,
                               int* intact) {
  int rc = 3;
  std::atomic<int> late_done{0};
  *intact = 0;
  spawn(2, 1, nullptr, 0, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    std::vector<uint64_t> buf(n, (uint64_t)r + 1);
    auto ub = c[0]->createUnboundBuffer(buf.data(), n * sizeof(uint64_t));
    const uint64_t slot = 77;
    if (r == 1) {  // the slow peer: its send arrives after rank 0 gave up
      std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
      try {
        ub->send(0, slot, 0, n * sizeof(uint64_t));
        ub->waitSend(std::chrono::milliseconds(2000));
      } catch (const std::exception&) {  // rank 0 closed the connection: fails, never hangs
      }
      late_done = 1;
      return;
    }
    // the receive lands straight in the caller's bucket, as the ring's all-gather does
    ub->recv(1, slot, 0, n * sizeof(uint64_t));
    try {
      ub->waitRecv(std::chrono::milliseconds(timeout_ms));
    } catch (const hydra::IoException& e) {
      set_err(what, len, e.what());
      rc = 0;
    }
    std::fill(buf.begin(), buf.end(), 0x5a5a5a5a5a5a5a5aull);  // the caller reuses its memory
    while (!late_done) std::this_thread::sleep_for(std::chrono::milliseconds(5));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    *intact = std::all_of(buf.begin(), buf.end(),
                          [](uint64_t v) { return v == 0x5a5a5a5a5a5a5a5aull; }) ? 1 : 0;
    // later operations on the poisoned context fail at once instead of waiting
    const auto t0 = std::chrono::steady_clock::now();
    try {
      ub->recv(1, slot + 1, 0, sizeof(uint64_t));
      ub->waitRecv(std::chrono::milliseconds(5000));
      rc = 4;
    } catch (const hydra::IoException&) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(1000)) rc = 5;
    }
  });
  return rc;
}

int hydra_host_timeout_probe(long timeout_ms, char* what, size_t len) {
  int rc = 3;
  spawn(2, 1, nullptr, 0, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    if (r != 0) return;
    uint64_t buf = 0;
    hydra::AllreduceOptions o(c[0]);
    o.setOutput(&buf, 1);
    o.setReduceFunction([](void* x, const void* a, const void* b, size_t n) {
      for (size_t i = 0; i < n; i++)
        static_cast<uint64_t*>(x)[i] =
            static_cast<const uint64_t*>(a)[i] + static_cast<const uint64_t*>(b)[i];
    });
    o.setTimeout(std::chrono::milliseconds(timeout_ms));
    try {
      hydra::allreduce(o);
    } catch (const hydra::IoException& e) {
      set_err(what, len, e.what());
      rc = 0;
    }
  });
  return rc;
}

}  // extern "C"
