// probe_host_floor.cc -- per-call cost of hydra_reduce_host from C++ (no Python in the loop):
// what the reference ring pays per segment when its Func is the hydra host sum
// (allreduce.cc:301-305: synchronous, c == a, b = the scratch slot).
// Modes: registered (hydra_host_register'ed mmap buffers), pinned (hydra_malloc_host blocks),
// pageable (malloc'ed, odd offsets: CPU-staged), mixed (a / c registered, b pageable: the drop-in
// inside the reference's ring with a registered bucket).  Sizes from argv (elements), default
// 64 1024 16384 262144.  Prints one JSON document: median / p10 / p90 microseconds per call.
// Build: hydra_amd/csrc/Makefile (-> scripts/probe_host_floor).  Run on the GPU box.
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hydra_hip.h"

#define CK(x)                                                              \
  do {                                                                     \
    int rc_ = (x);                                                         \
    if (rc_) {                                                             \
      std::fprintf(stderr, "%s: %d %s\n", #x, rc_, hydra_last_error());    \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(std::strtoull(argv[i], nullptr, 10));
  if (sizes.empty()) sizes = {64, 1024, 16384, 262144};
  size_t big = 1 << 22;  // elements per buffer (room for the largest size + the offsets)
  for (size_t n : sizes) big = std::max(big, (n + 4096 + 1023) / 1024 * 1024);
  hydra_ctx_t ctx;
  // HYDRA_RESIDENT=0 in this probe's environment: the same calls with the resident reducer
  // off (the library itself reads no environment; HYDRA_OPT_RESIDENT is its option)
  const char* env = std::getenv("HYDRA_RESIDENT");
  const bool resident = !(env && env[0] == '0');
  CK(hydra_set_option(HYDRA_OPT_RESIDENT, resident ? 1 : 0));
  CK(hydra_ctx_create(0, &ctx));
  // registered: mmap'ed, never returned to the allocator
  float* ra = static_cast<float*>(mmap(nullptr, big * 4, PROT_READ | PROT_WRITE,
                                       MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
  float* rb = static_cast<float*>(mmap(nullptr, big * 4, PROT_READ | PROT_WRITE,
                                       MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
  CK(hydra_host_register(ra, big * 4));
  CK(hydra_host_register(rb, big * 4));
  void *pa, *pb;
  CK(hydra_malloc_host(big * 4, &pa));
  CK(hydra_malloc_host(big * 4, &pb));
  std::vector<float> ga(big + 16), gb(big + 16);
  struct Mode {
    const char* name;
    float* a;
    float* b;
  } modes[] = {{"registered", ra + 1024, rb + 1024},
               {"pinned", static_cast<float*>(pa) + 1024, static_cast<float*>(pb) + 1024},
               {"pageable", ga.data() + 3, gb.data() + 5},
               // the reference ring's own call (allreduce.cc:301-305) after the maintainer
               // registered the bucket: c == a in the registered bucket, b in the ring's
               // pageable scratch (new uint8_t[], :225-229)
               {"mixed", ra + 1024, gb.data() + 5}};
  for (auto& m : modes)
    for (size_t i = 0; i < big - 2048; i++) m.a[i] = 1.0f, m.b[i] = 0.5f;
  uint64_t calls0 = 0, launches0 = 0;
  CK(hydra_ctx_stats(ctx, &calls0, &launches0));
  std::printf("{\"probe\": \"scripts/probe_host_floor\", \"rows\": [");
  bool first = true;
  for (size_t n : sizes)
    for (auto& m : modes) {
      const int k = (int)std::max<size_t>(100, std::min<size_t>(5000, 200000000 / (12 * n + 1)));
      std::vector<double> us(k);
      for (int w = 0; w < std::min(50, k); w++) CK(hydra_reduce_host(ctx, HYDRA_SUM, HYDRA_FLOAT32, m.a, m.a, m.b, n));
      for (int i = 0; i < k; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        CK(hydra_reduce_host(ctx, HYDRA_SUM, HYDRA_FLOAT32, m.a, m.a, m.b, n));
        us[i] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                    .count();
      }
      std::sort(us.begin(), us.end());
      std::printf("%s{\"elements\": %zu, \"mode\": \"%s\", \"calls\": %d, \"us_median\": %.2f, "
                  "\"us_p10\": %.2f, \"us_p90\": %.2f}",
                  first ? "" : ", ", n, m.name, k, us[k / 2], us[k / 10], us[k * 9 / 10]);
      first = false;
      std::fflush(stdout);
    }
  uint64_t calls = 0, launches = 0;
  CK(hydra_ctx_stats(ctx, &calls, &launches));
  std::printf("], \"resident\": %s, \"resident_calls\": %llu, \"resident_launches\": %llu}\n",
              resident ? "true" : "false", (unsigned long long)(calls - calls0),
              (unsigned long long)(launches - launches0));
  CK(hydra_host_unregister(ra));
  CK(hydra_host_unregister(rb));
  CK(hydra_free_host(pa));
  CK(hydra_free_host(pb));
  CK(hydra_ctx_destroy(ctx));
  return 0;
}
