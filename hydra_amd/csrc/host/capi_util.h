// capi_util.h -- helpers shared by the host runtime's C drivers (host_capi.cpp and the opt-in
// extra_capi.cpp): error text and the thread-per-rank harness.
#pragma once

#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/hydra/allreduce.h"
#include "../../../include/hydra/gloo_reduce.h"
#include "../../../include/hydra_host.h"

namespace hydra {
namespace capi {

inline void set_err(char* err, size_t len, const std::string& s) {
  if (err && len) {
    std::strncpy(err, s.c_str(), len - 1);
    err[len - 1] = 0;
  }
}

inline hydra::AllreduceOptions::Func make_reducer(int reducer, int op, int dtype, hydra_reduce_fn fn) {
  if (reducer == HYDRA_REDUCER_FN) {
    if (!fn) throw hydra::EnforceNotMet("null reduce function");
    return [fn](void* c, const void* a, const void* b, size_t n) { fn(c, a, b, n); };
  }
  return hydra::gloo_compat::hostReduce(op, dtype, 0);
}

inline size_t esize_of(int dtype) {
  static const size_t sz[] = {1, 1, 4, 4, 8, 8, 4, 8, 2, 2};
  return (dtype >= 0 && dtype <= 9) ? sz[dtype] : 0;
}

// Spawn P threads; each gets a connected context (two when rails == 2).
inline int spawn(int P, int rails, char* err, size_t errlen,
          const std::function<void(int, std::vector<std::shared_ptr<hydra::Context>>&)>& body) {
  hydra::HashStore store;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  std::string first;
  std::vector<std::thread> th;
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      std::vector<std::shared_ptr<hydra::Context>> ctx;
      try {
        for (int k = 0; k < rails; k++) {
          ctx.push_back(std::make_shared<hydra::Context>(r, P));
          ctx.back()->connectFullMesh(store, "127.0.0.1", "rail" + std::to_string(k));
        }
        body(r, ctx);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        if (first.empty()) first = e.what();
      }
      // every rank finishes before any connection closes (base_test.h:142-155)
      std::unique_lock<std::mutex> l(mu);
      arrived++;
      cv.notify_all();
      cv.wait(l, [&] { return arrived == P; });
    });
  }
  for (auto& t : th) t.join();
  if (!first.empty()) {
    set_err(err, errlen, first);
    return 1;
  }
  return 0;
}


}  // namespace capi
}  // namespace hydra
