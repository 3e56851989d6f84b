// Sanitizer driver for the host runtime (transport + ring + rail split + reduce), built by
// tests/test_sanitizers.py with -fsanitize=thread and with -fsanitize=address,undefined.
// Mirrors AllreduceNewTest.Default (gloo/gloo/test/allreduce_test.cc:302-362) and the
// bew_allreduce_a split on thread-ranks over loopback TCP, with a plain CPU sum as the reducer
// (the product's GPU reducer is exercised by the GPU tests).  Exit 0 = all results correct.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "hydra/allreduce.h"
#include "hydra/allreduce_extra.h"  // the opt-in classes are race-checked too

static void sum_u64(void* c, const void* a, const void* b, size_t n) {
  for (size_t i = 0; i < n; i++)
    static_cast<uint64_t*>(c)[i] = static_cast<const uint64_t*>(a)[i] +
                                   static_cast<const uint64_t*>(b)[i];
}

// Context::setScratchAllocator: counted allocations (the GPU users install pinned memory here)
static std::atomic<int> g_allocs{0}, g_frees{0};
static void* count_alloc(size_t b) {
  g_allocs++;
  return std::malloc(b);
}
static void count_free(void* p) {
  g_frees++;
  std::free(p);
}
static void* decline_alloc(size_t) { return nullptr; }  // e.g. pinned memory without a GPU

static int run(int P, int nptr, size_t n, bool inplace, bool apipe, int alloc_mode = 0) {
  hydra::HashStore store;
  std::vector<std::thread> th;
  std::vector<int> bad(P, 0);
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      try {
        auto c1 = std::make_shared<hydra::Context>(r, P);
        c1->connectFullMesh(store, "127.0.0.1", "a");
        if (alloc_mode == 1) c1->setScratchAllocator({&count_alloc, &count_free});
        if (alloc_mode == 2) c1->setScratchAllocator({&decline_alloc, &count_free});
        std::shared_ptr<hydra::Context> c2;
        if (apipe) {
          c2 = std::make_shared<hydra::Context>(r, P);
          c2->connectFullMesh(store, "127.0.0.1", "b");
        }
        const size_t stride = (size_t)P * nptr;
        std::vector<std::vector<uint64_t>> in(nptr, std::vector<uint64_t>(n)),
            out(nptr, std::vector<uint64_t>(n, 0));
        for (int i = 0; i < nptr; i++)
          for (size_t k = 0; k < n; k++) in[i][k] = k * stride + (size_t)r * nptr + i;
        if (apipe) {
          hydra::APipeAllreduceOptions o(c1, c2);
          o.setInput(in[0].data(), n);
          o.setOutput(out[0].data(), n);
          o.setReduceFunction(&sum_u64);
          hydra::apipe_allreduce(o);
        } else {
          hydra::AllreduceOptions o(c1);
          std::vector<uint64_t*> optr, iptr;
          for (int i = 0; i < nptr; i++) {
            if (inplace) out[i] = in[i];
            optr.push_back(out[i].data());
            iptr.push_back(in[i].data());
          }
          o.setOutputs(optr, n);
          if (!inplace) o.setInputs(iptr, n);
          o.setReduceFunction(&sum_u64);
          o.setMaxSegmentSize(128);
          hydra::allreduce(o);
        }
        const size_t base = stride * (stride - 1) / 2;
        const int nout = apipe ? 1 : nptr;
        const size_t s2 = apipe ? (size_t)P * P : stride * stride;
        const size_t b2 = apipe ? (size_t)P * (P - 1) / 2 : base;
        for (int i = 0; i < nout; i++)
          for (size_t k = 0; k < n; k++)
            if (out[i][k] != k * s2 + b2) bad[r] = 1;
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        bad[r] = 1;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int b : bad)
    if (b) return 1;
  return 0;
}

static void isum_u64(uint64_t* x, const uint64_t* y, size_t n) {
  for (size_t i = 0; i < n; i++) x[i] += y[i];
}

// Old-style Algorithm API: AllreduceRing<T> / AllreduceRingChunked<T> /
// AllreduceHalvingDoubling<T> (allreduce_ring.h, allreduce_ring_chunked.h,
// allreduce_halving_doubling.h, allreduce_bcube.h) with several pointers per rank.  kind: 0 ring,
// 1 chunked, 2 halving-doubling, 3 old-style bcube.
static int run_algorithm(int P, int nptr, int n, int kind) {
  hydra::HashStore store;
  std::vector<std::thread> th;
  std::vector<int> bad(P, 0);
  static const hydra::ReductionFunction<uint64_t> fn(hydra::SUM, &isum_u64);
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      try {
        auto c = std::make_shared<hydra::Context>(r, P);
        c->connectFullMesh(store, "127.0.0.1", "alg");
        const size_t stride = (size_t)P * nptr;
        std::vector<std::vector<uint64_t>> buf(nptr, std::vector<uint64_t>(n));
        std::vector<uint64_t*> ptrs;
        for (int i = 0; i < nptr; i++) {
          for (int k = 0; k < n; k++) buf[i][k] = k * stride + (size_t)r * nptr + i;
          ptrs.push_back(buf[i].data());
        }
        for (int it = 0; it < 2; it++) {  // the algorithm object is reusable across runs
          if (kind == 3) {
            hydra::AllreduceBcube<uint64_t> a(c, ptrs, n, &fn);
            a.run();
          } else if (kind == 2) {
            hydra::AllreduceHalvingDoubling<uint64_t> a(c, ptrs, n, &fn);
            a.run();
          } else if (kind == 1) {
            hydra::AllreduceRingChunked<uint64_t> a(c, ptrs, n, &fn);
            a.run();
          } else {
            hydra::AllreduceRing<uint64_t> a(c, ptrs, n, &fn);
            a.run();
          }
          const uint64_t mul = it == 0 ? 1 : stride;  // 2nd run sums the 1st run's outputs
          for (int i = 0; i < nptr; i++)
            for (int k = 0; k < n; k++) {
              const uint64_t first = k * stride * stride + stride * (stride - 1) / 2;
              if (buf[i][k] != first * mul) bad[r] = 1;
            }
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        bad[r] = 1;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int b : bad)
    if (b) return 1;
  return 0;
}

// ReduceTest.Default (gloo/gloo/test/reduce_test.cc:22-86): every rank takes a turn as root.
static int run_reduce(int P, size_t n, bool inplace) {
  hydra::HashStore store;
  std::vector<std::thread> th;
  std::vector<int> bad(P, 0);
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      try {
        auto c = std::make_shared<hydra::Context>(r, P);
        c->connectFullMesh(store, "127.0.0.1", "r");
        std::vector<uint64_t> in(n), out(n);
        for (int root = 0; root < P; root++) {
          for (size_t k = 0; k < n; k++) in[k] = k * P + r;
          hydra::ReduceOptions o(c);
          if (inplace) {
            out = in;
          } else {
            std::fill(out.begin(), out.end(), 0);
            o.setInput(in.data(), n);
          }
          o.setOutput(out.data(), n);
          o.setRoot(root);
          o.setReduceFunction(&sum_u64);
          o.setMaxSegmentSize(128);
          hydra::reduce(o);
          if (r == root)
            for (size_t k = 0; k < n; k++)
              if (out[k] != k * P * P + (size_t)P * (P - 1) / 2) bad[r]++;
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        bad[r]++;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int b : bad)
    if (b) return 1;
  return 0;
}

// Concurrent aborts of the same pairs (round 2 advisor: a second abort() must not return before
// the first has joined the pair's threads): three threads per rank call signalException /
// closeConnections at once after an allreduce; every call returns, nothing races.
static int run_concurrent_abort(int P) {
  hydra::HashStore store;
  std::vector<std::thread> th;
  std::vector<int> bad(P, 0);
  for (int r = 0; r < P; r++) {
    th.emplace_back([&, r] {
      try {
        auto c = std::make_shared<hydra::Context>(r, P);
        c->connectFullMesh(store, "127.0.0.1", "abort");
        std::vector<uint64_t> x(4096, (uint64_t)r);
        hydra::AllreduceOptions o(c);
        o.setOutput(x.data(), x.size());
        o.setReduceFunction(&sum_u64);
        hydra::allreduce(o);
        std::vector<std::thread> q;
        for (int k = 0; k < 3; k++)
          q.emplace_back([&, k] {
            if (k == 1)
              c->closeConnections();
            else
              c->signalException("concurrent abort " + std::to_string(k));
          });
        for (auto& t : q) t.join();
      } catch (const std::exception& e) {
        std::fprintf(stderr, "rank %d: %s\n", r, e.what());
        bad[r] = 1;
      }
    });
  }
  for (auto& t : th) t.join();
  for (int b : bad)
    if (b) return 1;
  return 0;
}

int main() {
  int fails = 0;
  for (int P : {2, 3})
    if (run_concurrent_abort(P)) {
      std::fprintf(stderr, "FAIL concurrent abort P=%d\n", P);
      fails++;
    }
  for (int P : {1, 2, 3, 4})
    for (bool inplace : {true, false})
      for (size_t n : {(size_t)1, (size_t)1000, (size_t)20011})
        if (run_reduce(P, n, inplace)) {
          std::fprintf(stderr, "FAIL reduce P=%d n=%zu inplace=%d\n", P, n, (int)inplace);
          fails++;
        }
  for (int P : {1, 2, 3, 4})
    for (int nptr : {1, 2})
      for (bool inplace : {true, false})
        for (size_t n : {(size_t)1, (size_t)100, (size_t)10000}) {
          if (run(P, nptr, n, inplace, false)) {
            std::fprintf(stderr, "FAIL allreduce P=%d nptr=%d n=%zu inplace=%d\n", P, nptr, n,
                         (int)inplace);
            fails++;
          }
        }
  for (int P : {2, 3})
    for (size_t n : {(size_t)1000, (size_t)70000})
      if (run(P, 1, n, false, true)) {
        std::fprintf(stderr, "FAIL apipe P=%d n=%zu\n", P, n);
        fails++;
      }
  // scratch allocator: used once per context (cached across the ring's segments), released
  // with the context; a declining allocator falls back to the heap (never handed to release)
  if (run(3, 1, 10000, true, false, 1) || g_allocs.load() != 3 || g_frees.load() != 3) {
    std::fprintf(stderr, "FAIL scratch allocator allocs=%d frees=%d\n", g_allocs.load(),
                 g_frees.load());
    fails++;
  }
  if (run(2, 1, 10000, true, false, 2) || g_frees.load() != 3) {
    std::fprintf(stderr, "FAIL declining scratch allocator\n");
    fails++;
  }
  static const char* kNames[] = {"AllreduceRing", "AllreduceRingChunked",
                                 "AllreduceHalvingDoubling", "AllreduceBcube"};
  for (int kind : {0, 1, 2})
    for (int P : {1, 2, 3, 5, 7})
      for (int nptr : {1, 2})
        for (int n : {1, 1000, 20011})
          if (run_algorithm(P, nptr, n, kind)) {
            std::fprintf(stderr, "FAIL %s P=%d nptr=%d n=%d\n", kNames[kind], P, nptr, n);
            fails++;
          }
  for (int P : {1, 2, 4})  // AllreduceBcube: powers of the base only
    for (int nptr : {1, 2})
      for (int n : {1, 1000, 20011})
        if (run_algorithm(P, nptr, n, 3)) {
          std::fprintf(stderr, "FAIL %s P=%d nptr=%d n=%d\n", kNames[3], P, nptr, n);
          fails++;
        }
  std::printf("%s\n", fails ? "FAILED" : "OK");
  return fails ? 1 : 0;
}
