// extra_capi.cpp -- OUT OF SCOPE, opt-in: C drivers of the other old-style Algorithm-API classes
// (include/hydra_host_extra.h) -> libhydra_host_extra.so.  Only the `extra` tests load it.
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../../include/hydra/allreduce_extra.h"
#include "../../../include/hydra/hip_allreduce_extra.h"
#include "../../../include/hydra_host_extra.h"
#include "capi_util.h"

using hydra::capi::set_err;
using hydra::capi::spawn;

namespace {

// kind: 2 AllreduceHalvingDoubling, 3 old-style AllreduceBcube, 4 AllreduceLocal
template <typename T>
int algorithm(int kind, int P, int nptr, size_t n, void** bufs, int reducer, hydra_inplace_fn fn,
              char* err, size_t errlen) {
  using RF = hydra::ReductionFunction<T>;
  const RF* rf = nullptr;
  std::unique_ptr<RF> custom;
  if (reducer == HYDRA_REDUCER_FN) {
    if (!fn) {
      set_err(err, errlen, "null reduce function");
      return 2;
    }
    custom.reset(new RF(hydra::CUSTOM, reinterpret_cast<typename RF::Function*>(fn)));
    rf = custom.get();
  } else {
    rf = hydra::gloo_compat::gpuReductionFunction<RF, T>(hydra::SUM);
  }
  return spawn(P, 1, err, errlen, [&](int r, std::vector<std::shared_ptr<hydra::Context>>& c) {
    std::vector<T*> ptrs;
    for (int i = 0; i < nptr; i++) ptrs.push_back(static_cast<T*>(bufs[r * nptr + i]));
    if (kind == 4) {
      hydra::AllreduceLocal<T> algo(c[0], ptrs, (int)n, rf);
      algo.run();
    } else if (kind == 3) {
      hydra::AllreduceBcube<T> algo(c[0], ptrs, (int)n, rf);
      algo.run();
    } else {
      hydra::AllreduceHalvingDoubling<T> algo(c[0], ptrs, (int)n, rf);
      algo.run();
    }
  });
}

int algorithm_dt(int kind, int P, int nptr, int dtype, size_t n, void** bufs, int reducer,
                 hydra_inplace_fn fn, char* err, size_t errlen) {
  if (P < 1 || nptr < 1 || !bufs || n > (size_t)INT32_MAX) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  switch (dtype) {
    case HYDRA_FLOAT32: return algorithm<float>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_INT32: return algorithm<int32_t>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_FLOAT64: return algorithm<double>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
    case HYDRA_FLOAT16:
      if (reducer != HYDRA_REDUCER_FN) break;
      return algorithm<uint16_t>(kind, P, nptr, n, bufs, reducer, fn, err, errlen);
  }
  set_err(err, errlen, "unsupported dtype for this Algorithm class");
  return 3;
}

// kind: 2 HipAllreduceHalvingDoubling, 3 HipAllreduceLocal, 4 HipAllreduceBcube
template <typename T>
int hip_algorithm(int kind, int P, int nptr, size_t n, void** bufs, int workspace,
                  int user_streams, char* err, size_t errlen) {
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
    const bool devws = workspace == HYDRA_WORKSPACE_DEVICE;
    if (kind == 4 && devws) {
      hydra::HipAllreduceBcube<T, hydra::HipDeviceWorkspace<T>> algo(c[0], ptrs, (int)n, streams);
      algo.run();
    } else if (kind == 4) {
      hydra::HipAllreduceBcube<T, hydra::HipHostWorkspace<T>> algo(c[0], ptrs, (int)n, streams);
      algo.run();
    } else if (kind == 3) {
      hydra::HipAllreduceLocal<T> algo(c[0], ptrs, (int)n, streams);
      algo.run();
    } else if (devws) {
      hydra::HipAllreduceHalvingDoubling<T, hydra::HipDeviceWorkspace<T>> algo(c[0], ptrs, (int)n,
                                                                               streams);
      algo.run();
    } else {
      hydra::HipAllreduceHalvingDoubling<T, hydra::HipHostWorkspace<T>> algo(c[0], ptrs, (int)n,
                                                                             streams);
      algo.run();
    }
    for (auto s : streams) {  // caller-provided streams: outputs are async until synchronized
      hydra::gloo_compat::enforce(hydra_stream_synchronize(s));
      hydra_stream_destroy(s);
    }
    int dev = 0;
    if (n) hydra::gloo_compat::enforce(hydra_pointer_device(ptrs[0], &dev));
    if (hydra_device_check(dev) != 0)
      throw hydra::EnforceNotMet(std::string("after the algorithm's teardown: ") +
                                 hydra_last_error());
  });
}

int hip_algorithm_dt(int kind, int P, int nptr, int dtype, size_t n, void** dev_bufs,
                     int workspace, int user_streams, char* err, size_t errlen) {
  if (P < 1 || nptr < 1 || !dev_bufs || n > (size_t)INT32_MAX) {
    set_err(err, errlen, "invalid arguments");
    return 2;
  }
  switch (dtype) {
    case HYDRA_FLOAT32:
      return hip_algorithm<float>(kind, P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
    case HYDRA_INT32:
      return hip_algorithm<int32_t>(kind, P, nptr, n, dev_bufs, workspace, user_streams, err,
                                    errlen);
    case HYDRA_FLOAT64:
      return hip_algorithm<double>(kind, P, nptr, n, dev_bufs, workspace, user_streams, err, errlen);
    case HYDRA_INT64:
      return hip_algorithm<int64_t>(kind, P, nptr, n, dev_bufs, workspace, user_streams, err,
                                    errlen);
  }
  set_err(err, errlen, "unsupported dtype for this Hip Algorithm class");
  return 3;
}

}  // namespace

extern "C" {

int hydra_host_allreduce_halving_doubling_threads(int P, int nptr, int dtype, size_t n,
                                                  void** bufs, int reducer, hydra_inplace_fn fn,
                                                  char* err, size_t errlen) {
  return algorithm_dt(2, P, nptr, dtype, n, bufs, reducer, fn, err, errlen);
}

int hydra_host_allreduce_bcube_old_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                           int reducer, hydra_inplace_fn fn, char* err,
                                           size_t errlen) {
  return algorithm_dt(3, P, nptr, dtype, n, bufs, reducer, fn, err, errlen);
}

int hydra_host_allreduce_local_threads(int P, int nptr, int dtype, size_t n, void** bufs,
                                       int reducer, hydra_inplace_fn fn, char* err,
                                       size_t errlen) {
  return algorithm_dt(4, P, nptr, dtype, n, bufs, reducer, fn, err, errlen);
}

int hydra_host_hip_halving_doubling_threads(int P, int nptr, int dtype, size_t n,
                                            void** dev_bufs, int workspace, int user_streams,
                                            char* err, size_t errlen) {
  return hip_algorithm_dt(2, P, nptr, dtype, n, dev_bufs, workspace, user_streams, err, errlen);
}

int hydra_host_hip_local_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                 int workspace, int user_streams, char* err, size_t errlen) {
  return hip_algorithm_dt(3, P, nptr, dtype, n, dev_bufs, workspace, user_streams, err, errlen);
}

int hydra_host_hip_bcube_threads(int P, int nptr, int dtype, size_t n, void** dev_bufs,
                                 int workspace, int user_streams, char* err, size_t errlen) {
  return hip_algorithm_dt(4, P, nptr, dtype, n, dev_bufs, workspace, user_streams, err, errlen);
}

}  // extern "C"
