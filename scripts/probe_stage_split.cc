// probe_stage_split.cc -- interleaved A/B of how many rounds a staged (pageable) host call is
// cut into (hydra_ctx_set_option HYDRA_OPT_STAGE_SPLIT; the default is 4).  For each
// size the splits take turns in short blocks, rotated every repetition, so drift on the box
// (page cache, helper-thread placement, other tenants) lands on every setting alike.  c == a,
// both pageable, as the ring calls an unregistered Func.  Prints one JSON document: median and
// p10 microseconds per split.  Build: hydra_amd/csrc/Makefile.  Run on the GPU box.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "hydra_hip.h"

#define CK(x)                                                           \
  do {                                                                  \
    int rc_ = (x);                                                      \
    if (rc_) {                                                          \
      std::fprintf(stderr, "%s: %d %s\n", #x, rc_, hydra_last_error()); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

int main(int argc, char** argv) {
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; i++) sizes.push_back(std::strtoull(argv[i], nullptr, 10));
  if (sizes.empty()) sizes = {262144, 1048576, 4194304};
  const int splits[] = {1, 2, 4, 8};
  constexpr int S = 4;
  hydra_ctx_t ctx;
  CK(hydra_ctx_create(0, &ctx));
  std::printf("{\"probe\": \"scripts/probe_stage_split\", \"rows\": [");
  bool first = true;
  for (size_t n : sizes) {
    std::vector<float> a(n + 16, 1.0f), b(n + 16, 0.5f);
    float* pa = a.data() + 3;  // odd offsets: ragged pages, as a heap buffer has
    float* pb = b.data() + 5;
    const int block = (int)std::max<size_t>(3, std::min<size_t>(40, 20000000 / (12 * n + 1)));
    const int reps = 12;
    std::vector<double> us[S];
    for (int w = 0; w < 10; w++) CK(hydra_reduce_host(ctx, HYDRA_SUM, HYDRA_FLOAT32, pa, pa, pb, n));
    for (int r = 0; r < reps; r++)
      for (int j = 0; j < S; j++) {
        const int k = (j + r) % S;
        CK(hydra_ctx_set_option(ctx, HYDRA_OPT_STAGE_SPLIT, splits[k]));
        CK(hydra_reduce_host(ctx, HYDRA_SUM, HYDRA_FLOAT32, pa, pa, pb, n));  // settle
        for (int i = 0; i < block; i++) {
          const auto t0 = std::chrono::steady_clock::now();
          CK(hydra_reduce_host(ctx, HYDRA_SUM, HYDRA_FLOAT32, pa, pa, pb, n));
          us[k].push_back(
              std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                  .count());
        }
      }
    CK(hydra_ctx_set_option(ctx, HYDRA_OPT_STAGE_SPLIT, 4));
    for (int k = 0; k < S; k++) {
      std::sort(us[k].begin(), us[k].end());
      const size_t m = us[k].size();
      std::printf("%s{\"elements\": %zu, \"split\": %d, \"calls\": %zu, \"us_median\": %.2f, "
                  "\"us_p10\": %.2f}",
                  first ? "" : ", ", n, splits[k], m, us[k][m / 2], us[k][m / 10]);
      first = false;
    }
    std::fflush(stdout);
  }
  std::printf("]}\n");
  CK(hydra_ctx_destroy(ctx));
  return 0;
}
