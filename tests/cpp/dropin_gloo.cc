// tests/cpp/dropin_gloo.cc -- TEST HARNESS: the drop-in proven inside the reference itself.
//
// Runs the REFERENCE's own collectives -- gloo::allreduce's ring (gloo/gloo/allreduce.cc:147-422,
// its multi-input local reduce :46-83 with two pointers per rank), gloo::reduce
// (gloo/gloo/reduce.cc:21-262, the Func's other new-style caller, :195), and the old-style
// gloo::AllreduceRing<T> / AllreduceRingChunked<T> (allreduce_ring.h:20-125,
// allreduce_ring_chunked.h:20-248) -- compiled from
// /root/reference by oracle/Makefile into oracle/_ref/libgloo_ref.so, on thread-ranks with an
// in-process HashStore and a loopback TCP device (the reference's own test setup,
// gloo/gloo/test/base_test.h:73-156).  Each case runs twice on identical inputs:
//   reducer "gloo"   the reference's gloo::sum<T> / ReductionFunction<T>::sum (math.h:15-23)
//   reducer "hydra"  libhydra_hip.so through include/hydra/gloo_reduce.h, plugged in exactly
//                    where a user would: AllreduceOptions::setReduceFunction(Func)
//                    (allreduce.h:36,179-181; called at allreduce.cc:301-305) and the
//                    ReductionFunction<T>* argument of AllreduceRing<T> (algorithm.h:59-96)
// and reports whether every rank's bytes are identical, plus per-iteration timings of both
// (rank 0 wall time around each collective, ranks released together, as runner.cc:683-702).
//
// Built by oracle/Makefile (it needs the reference headers, present only in the build
// container); the binary travels to the GPU box, where tests/test_gpu_dropin.py runs it.
//
// usage: dropin_gloo <mode> <P> <n> <f32|i32|f16> [timed_iters] [max_segment]
//   mode: new_ring | new_ring2 (2 pointers per rank) | new_reduce (root P-1) | old_ring |
//         old_ring_chunked | errors (the shim's failures as the reference's exception types)
// prints one JSON object on stdout; exit 0 iff both runs finished (equality is in the JSON).

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "gloo/algorithm.h"
#include "gloo/allreduce.h"
#include "gloo/allreduce_ring.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/reduce.h"
#include "gloo/math.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo/types.h"

// the shim with Gloo's own exception types (gloo::EnforceNotMet / gloo::IoException)
#include "hydra/gloo_errors.h"

namespace {

struct Barrier {  // reusable: all P threads leave wait() together
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> l(mu_);
    const long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(l, [&] { return gen_ != gen; });
    }
  }
  int n_, count_ = 0;
  long gen_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
};

template <typename T>
std::vector<T> make_input(int P, int r, size_t n);

// fold-order-sensitive fp32: uniform [-1, 1) scaled by 2^(3r mod 17), so a different
// association changes the low bits (the oracle's stress pattern)
template <>
std::vector<float> make_input<float>(int P, int r, size_t n) {
  std::mt19937 g(1234u + 97u * (unsigned)P + (unsigned)r);
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  const float scale = std::ldexp(1.0f, (3 * r) % 17);
  std::vector<float> x(n);
  for (auto& v : x) v = u(g) * scale;
  return x;
}

template <>
std::vector<int32_t> make_input<int32_t>(int P, int r, size_t n) {
  std::vector<int32_t> x(n);
  for (size_t i = 0; i < n; i++) x[i] = (int32_t)((i * 2654435761u + (unsigned)r * 40503u) & 0xfffff) - 0x80000;
  (void)P;
  return x;
}

// gloo::float16 (types.h): uniform [-4, 4) through the reference's own conversion; the in-place
// ring exercises float16's store quirk (types.h:112-130) on both sides
template <>
std::vector<gloo::float16> make_input<gloo::float16>(int P, int r, size_t n) {
  std::mt19937 g(4321u + 97u * (unsigned)P + (unsigned)r);
  std::uniform_real_distribution<float> u(-4.0f, 4.0f);
  std::vector<gloo::float16> x(n);
  for (auto& v : x) v = gloo::cpu_float2half_rn(u(g));
  return x;
}

// the hydra plug-ins per element type: the Func and the old-style ReductionFunction<T>
template <typename T>
gloo::AllreduceOptions::Func hydra_func() {
  return gloo::AllreduceOptions::Func(hydra::gloo_compat::hostSum<T>());
}
template <>
gloo::AllreduceOptions::Func hydra_func<gloo::float16>() {
  return gloo::AllreduceOptions::Func(hydra::gloo_compat::hostReduce(HYDRA_SUM, HYDRA_FLOAT16));
}
template <typename T>
const gloo::ReductionFunction<T>* hydra_rf() {
  return hydra::gloo_compat::gpuReductionFunction<gloo::ReductionFunction<T>, T>(gloo::SUM);
}
template <>
const gloo::ReductionFunction<gloo::float16>* hydra_rf<gloo::float16>() {
  return hydra::gloo_compat::gpuReductionFunctionAs<gloo::ReductionFunction<gloo::float16>,
                                                    gloo::float16, HYDRA_FLOAT16>(gloo::SUM);
}

struct RunOut {
  std::vector<std::vector<uint8_t>> bytes;  // [rank] output after the first collective
  std::vector<double> iter_ms;              // rank 0, timed iterations
  std::string error;
};

template <typename T>
RunOut run_case(const std::string& mode, int P, size_t n, bool hydra, int iters, size_t ms) {
  RunOut out;
  out.bytes.resize(P);
  gloo::rendezvous::HashStore store;
  gloo::transport::tcp::attr attr;
  attr.hostname = "127.0.0.1";
  auto dev = gloo::transport::tcp::CreateDevice(attr);
  Barrier bar(P);
  std::mutex mu;
  std::vector<std::thread> th;
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r]() {
      try {
        auto ctx = std::make_shared<gloo::rendezvous::Context>(r, P);
        ctx->connectFullMesh(store, dev);
        std::vector<T> x = make_input<T>(P, r, n);
        std::vector<T> x2 = make_input<T>(P, r + P, n);  // new_ring2's second pointer
        std::vector<T> rin = x;                          // new_reduce's input (out of place)
        std::function<void()> once;
        std::unique_ptr<gloo::Algorithm> old;
        // the drop-in: the gfx950 chunk-sum behind the Func / ReductionFunction plug-points
        const gloo::AllreduceOptions::Func func =
            hydra ? hydra_func<T>()
                  : gloo::AllreduceOptions::Func(
                        static_cast<void (*)(void*, const void*, const void*, size_t)>(&gloo::sum<T>));
        const gloo::ReductionFunction<T>* fn = hydra ? hydra_rf<T>() : gloo::ReductionFunction<T>::sum;
        if (mode == "new_ring" || mode == "new_ring2") {
          once = [&]() {
            gloo::AllreduceOptions o(ctx);
            o.setAlgorithm(gloo::AllreduceOptions::Algorithm::RING);
            if (mode == "new_ring2")  // two local inputs: the Func also pre-reduces (:61-80)
              o.setOutputs(std::vector<T*>{x.data(), x2.data()}, n);
            else
              o.setOutput(x.data(), n);
            if (ms) o.setMaxSegmentSize(ms);
            o.setReduceFunction(func);
            gloo::allreduce(o);
          };
        } else if (mode == "new_reduce") {
          once = [&]() {  // out of place to the last rank: reduce(out+off, in+off, tmp, n)
            gloo::ReduceOptions o(ctx);
            o.setInput(rin.data(), n);
            o.setOutput(x.data(), n);
            o.setRoot(P - 1);
            if (ms) o.setMaxSegmentSize(ms);
            o.setReduceFunction(func);
            gloo::reduce(o);
          };
        } else {
          std::vector<T*> ptrs{x.data()};
          if (mode == "old_ring_chunked")
            old.reset(new gloo::AllreduceRingChunked<T>(ctx, ptrs, (int)n, fn));
          else
            old.reset(new gloo::AllreduceRing<T>(ctx, ptrs, (int)n, fn));
          once = [&]() { old->run(); };
        }
        // HYDRA_DROPIN_REGISTER=1: a maintainer who also registers the bucket once
        // (hydra_host_register): the kernel then reads and writes it in place
        // over PCIe and only the reference's pageable scratch is staged
        const char* rg = std::getenv("HYDRA_DROPIN_REGISTER");
        const bool reg = hydra && rg && rg[0] == '1';
        if (reg) {
          hydra::gloo_compat::enforce(hydra_host_register(x.data(), n * sizeof(T)));
          if (mode == "new_ring2")
            hydra::gloo_compat::enforce(hydra_host_register(x2.data(), n * sizeof(T)));
        }
        bar.wait();
        once();
        {
          std::lock_guard<std::mutex> g(mu);
          out.bytes[r].assign(reinterpret_cast<uint8_t*>(x.data()),
                              reinterpret_cast<uint8_t*>(x.data()) + n * sizeof(T));
          if (mode == "new_ring2")  // both outputs of the rank
            out.bytes[r].insert(out.bytes[r].end(), reinterpret_cast<uint8_t*>(x2.data()),
                                reinterpret_cast<uint8_t*>(x2.data()) + n * sizeof(T));
        }
        for (int it = 0; it < iters + 1; it++) {  // one untimed warm-up, then `iters`
          bar.wait();
          const auto t0 = std::chrono::steady_clock::now();
          once();
          const double msec =
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
          if (r == 0 && it > 0) out.iter_ms.push_back(msec);
        }
        bar.wait();  // nobody closes its pairs while a peer still runs (base_test.h:142-155)
        old.reset();
        if (reg) {
          hydra_host_unregister(x.data());
          if (mode == "new_ring2") hydra_host_unregister(x2.data());
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        if (out.error.empty()) out.error = e.what();
        // a failed rank cannot rejoin the barrier protocol: abort the process, loudly
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        std::fflush(stderr);
        std::_Exit(2);
      }
    });
  }
  for (auto& t : th) t.join();
  return out;
}

uint64_t fnv1a(const std::vector<std::vector<uint8_t>>& v) {
  uint64_t h = 1469598103934665603ull;
  for (const auto& b : v)
    for (uint8_t c : b) h = (h ^ c) * 1099511628211ull;
  return h;
}

double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p / 100.0 * (v.size() - 1) + 0.5))];
}

template <typename T>
int run_all(const std::string& mode, int P, size_t n, int iters, size_t ms, const char* dt) {
  // HYDRA_DROPIN_REF_ONLY=1 (CPU self-test of the harness): the second run is the reference too
  const char* ro = std::getenv("HYDRA_DROPIN_REF_ONLY");
  const bool ref_only = ro && ro[0] == '1';
  RunOut ref = run_case<T>(mode, P, n, false, iters, ms);
  // HYDRA_DROPIN_TRACE=1: every hydra Func call of the hydra run recorded (hydra_host_trace):
  // which operands went zero-copy or staged, rounds, resident or launched, and the time split
  const char* tr = std::getenv("HYDRA_DROPIN_TRACE");
  const bool trace = !ref_only && tr && tr[0] == '1';
  if (trace) hydra_host_trace(1);
  RunOut hyd = run_case<T>(mode, P, n, !ref_only, iters, ms);
  std::string trace_json = "null";
  if (trace) {
    hydra_host_trace(0);
    size_t cnt = 0;
    hydra_host_trace_read(nullptr, 0, &cnt);
    std::vector<hydra_host_call_t> v(cnt);
    hydra_host_trace_read(v.data(), cnt, &cnt);
    double tot = 0, cin = 0, wt = 0, cout = 0, iv = 0, rd = 0, res = 0, elems = 0;
    double zc[3] = {0, 0, 0}, st[3] = {0, 0, 0};
    std::vector<double> totals;
    for (const auto& c : v) {
      tot += c.total_us, cin += c.copy_in_us, wt += c.wait_us, cout += c.copy_out_us;
      iv += c.intervals, rd += c.rounds, res += c.resident, elems += (double)c.n;
      for (int k = 0; k < 3; k++) zc[k] += (double)c.zero_copy_bytes[k], st[k] += (double)c.staged_bytes[k];
      totals.push_back(c.total_us);
    }
    const double k = cnt ? (double)cnt : 1.0;
    char b[1024];
    std::snprintf(b, sizeof b,
                  "{\"calls\": %zu, \"elements_avg\": %.1f, \"intervals_avg\": %.3f, "
                  "\"rounds_avg\": %.3f, \"resident_frac\": %.3f, \"total_us_avg\": %.2f, "
                  "\"total_us_p50\": %.2f, \"copy_in_us_avg\": %.2f, \"wait_us_avg\": %.2f, "
                  "\"copy_out_us_avg\": %.2f, \"zero_copy_MB\": [%.3f, %.3f, %.3f], "
                  "\"staged_MB\": [%.3f, %.3f, %.3f]}",
                  cnt, elems / k, iv / k, rd / k, res / k, tot / k, pct(totals, 50), cin / k,
                  wt / k, cout / k, zc[0] / k / 1e6, zc[1] / k / 1e6, zc[2] / k / 1e6,
                  st[0] / k / 1e6, st[1] / k / 1e6, st[2] / k / 1e6);
    trace_json = b;
  }
  size_t mism = 0, first = (size_t)-1;
  int first_rank = -1;
  for (int r = 0; r < P; r++)
    for (size_t i = 0; i < ref.bytes[r].size(); i++)
      if (ref.bytes[r][i] != hyd.bytes[r][i]) {
        if (!mism) first = i, first_rank = r;
        mism++;
      }
  bool ranks_equal = true;
  for (int r = 1; r < P; r++) ranks_equal = ranks_equal && ref.bytes[r] == ref.bytes[0];
  auto avg = [](const std::vector<double>& v) {
    double s = 0;
    for (double x : v) s += x;
    return v.empty() ? 0.0 : s / v.size();
  };
  const double bytes = (double)n * sizeof(T);
  auto gib = [&](double msec) { return msec > 0 ? bytes / (msec * 1e-3) / (1024.0 * 1024 * 1024) : 0; };
  std::printf(
      "{\"mode\": \"%s\", \"P\": %d, \"n\": %zu, \"dtype\": \"%s\", \"max_segment\": %zu, "
      "\"mismatched_bytes\": %zu, \"first_mismatch\": [%d, %lld], \"ref_ranks_equal\": %s, "
      "\"fnv_ref\": \"%016llx\", \"fnv_hydra\": \"%016llx\", \"iters\": %d, "
      "\"ref_ms\": {\"p50\": %.4f, \"p99\": %.4f, \"avg\": %.4f, \"GiBps_avg\": %.4f}, "
      "\"hydra_ms\": {\"p50\": %.4f, \"p99\": %.4f, \"avg\": %.4f, \"GiBps_avg\": %.4f}, "
      "\"hydra_trace\": %s}\n",
      mode.c_str(), P, n, dt, ms, mism, first_rank, mism ? (long long)first : -1LL,
      ranks_equal ? "true" : "false", (unsigned long long)fnv1a(ref.bytes),
      (unsigned long long)fnv1a(hyd.bytes), iters, pct(ref.iter_ms, 50), pct(ref.iter_ms, 99),
      avg(ref.iter_ms), gib(avg(ref.iter_ms)), pct(hyd.iter_ms, 50), pct(hyd.iter_ms, 99),
      avg(hyd.iter_ms), gib(avg(hyd.iter_ms)), trace_json.c_str());
  return 0;
}

// mode "errors": the shim's failures reach a reference caller as the reference's own types.
//  (1) an invalid call inside the reference's gloo::allreduce: one process (the P = 1
//      short-circuit, allreduce.cc:129-133) with two outputs, so allreduce runs the local reduce
//      (genLocalReduceFunction, :46-83) through the hydra Func -- with an element type code the
//      library rejects.  The failure must leave gloo::allreduce as gloo::EnforceNotMet
//      (common/logging.h:21,42), caught where a reference caller catches GLOO_ENFORCE failures.
//      (With P > 1 the ring would unwind with its scratch receive still posted, allreduce.cc:
//      225-300 -- the reference's own timeout tests leave the process after that, too.)
//  (2) the timeout status (HYDRA_ERR_TIMEOUT, e.g. hydra_comm_wait) through the same policy:
//      gloo::IoException (common/error.h:45), what tcp/unbound_buffer.cc:80-84 throws.
int run_errors(size_t n) {
  auto caught = [](const std::function<void()>& f, std::string* msg) -> std::string {
    try {
      f();
    } catch (const gloo::EnforceNotMet& e) {
      *msg = e.what();
      return "gloo::EnforceNotMet";
    } catch (const gloo::IoException& e) {
      *msg = e.what();
      return "gloo::IoException";
    } catch (const std::exception& e) {
      *msg = e.what();
      return "other";
    }
    return "none";
  };
  gloo::rendezvous::HashStore store;
  gloo::transport::tcp::attr attr;
  attr.hostname = "127.0.0.1";
  auto dev = gloo::transport::tcp::CreateDevice(attr);
  auto ctx = std::make_shared<gloo::rendezvous::Context>(0, 1);
  ctx->connectFullMesh(store, dev);
  std::vector<float> x(n, 1.0f), x2(n, 2.0f);
  std::string m1, m2, m3;
  const std::string t1 = caught(
      [&]() {
        gloo::AllreduceOptions o(ctx);
        o.setOutputs(std::vector<float*>{x.data(), x2.data()}, n);
        o.setReduceFunction(hydra::gloo_compat::hostReduce(HYDRA_SUM, 42 /* no such dtype */));
        gloo::allreduce(o);
      },
      &m1);
  // the same allreduce with a valid Func still runs afterwards (nothing left half-done)
  const std::string t2 = caught(
      [&]() {
        gloo::AllreduceOptions o(ctx);
        o.setOutputs(std::vector<float*>{x.data(), x2.data()}, n);
        o.setReduceFunction(hydra_func<float>());
        gloo::allreduce(o);
      },
      &m2);
  const bool sum_ok = x[0] == 3.0f && x[n - 1] == 3.0f && x2[n - 1] == 3.0f;
  const std::string t3 = caught(
      [&]() { hydra::gloo_compat::enforce(HYDRA_ERR_TIMEOUT, "hydra_comm_wait"); }, &m3);
  auto esc = [](std::string v) {
    std::string o;
    for (char ch : v) {
      if (ch == '"' || ch == '\\') o += '\\';
      if (ch == '\n') ch = ' ';
      o += ch;
    }
    return o;
  };
  std::printf(
      "{\"mode\": \"errors\", \"invalid_call\": \"%s\", \"invalid_msg\": \"%s\", "
      "\"valid_after\": \"%s\", \"valid_msg\": \"%s\", \"valid_sum_ok\": %s, "
      "\"timeout_status\": \"%s\", \"timeout_msg\": \"%s\"}\n",
      t1.c_str(), esc(m1).c_str(), t2.c_str(), esc(m2).c_str(), sum_ok ? "true" : "false",
      t3.c_str(), esc(m3).c_str());
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  // HYDRA_DROPIN_OPT="key=value,...": hydra_set_option calls before anything runs (the test's
  // way to pick a library option for this process; the library itself reads no environment)
  if (const char* o = std::getenv("HYDRA_DROPIN_OPT")) {
    std::string spec(o);
    size_t at = 0;
    while (at < spec.size()) {
      size_t end = spec.find(',', at);
      if (end == std::string::npos) end = spec.size();
      const std::string kv = spec.substr(at, end - at);
      const size_t eq = kv.find('=');
      if (eq != std::string::npos &&
          hydra_set_option(std::atoi(kv.substr(0, eq).c_str()),
                           std::strtoll(kv.substr(eq + 1).c_str(), nullptr, 10)) != 0) {
        std::fprintf(stderr, "hydra_set_option(%s): %s\n", kv.c_str(), hydra_last_error());
        return 2;
      }
      at = end + 1;
    }
  }
  if (argc >= 2 && std::string(argv[1]) == "errors")
    return run_errors(argc > 3 ? std::strtoull(argv[3], nullptr, 10) : 1000);
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s <new_ring|old_ring> <P> <n> <f32|i32> [iters] [max_segment]\n",
                 argv[0]);
    return 64;
  }
  const std::string mode = argv[1], dt = argv[4];
  const int P = std::atoi(argv[2]);
  const size_t n = std::strtoull(argv[3], nullptr, 10);
  const int iters = argc > 5 ? std::atoi(argv[5]) : 0;
  const size_t ms = argc > 6 ? std::strtoull(argv[6], nullptr, 10) : 0;
  const bool known = mode == "new_ring" || mode == "new_ring2" || mode == "new_reduce" ||
                     mode == "old_ring" || mode == "old_ring_chunked";
  if (!known || P < 1 || P > 16 || n < 1 || (dt != "f32" && dt != "i32" && dt != "f16")) {
    std::fprintf(stderr, "bad arguments\n");
    return 64;
  }
  if (mode.rfind("old_", 0) == 0 && ms) {
    std::fprintf(stderr, "max_segment applies to the new-style collectives only\n");
    return 64;
  }
  if (dt == "f16") return run_all<gloo::float16>(mode, P, n, iters, ms, "f16");
  return dt == "f32" ? run_all<float>(mode, P, n, iters, ms, "f32")
                     : run_all<int32_t>(mode, P, n, iters, ms, "i32");
}
