// CPU unit test of the per-pointer device bookkeeping of hydra::HipAllreduceRing /
// HipAllreduceRingChunked with pointers on several GPUs of one process:
// which local-reduce steps run, in which order, on which pointer's device, and which of them
// must stage the source because the two devices have no peer access.  Reference:
// CudaLocalNativeReduce (cuda_collectives_native.h:40-120), CudaLocalHostReduce
// (cuda_collectives_host.h:108-119), findCudaDevicePointerClosestToDevice (cuda_private.h:58-90).
// Built and run by tests/test_local_steps.py (no GPU, no HIP runtime).
#include <cstdio>
#include <cstdlib>
#include <set>
#include <utility>
#include <vector>

#include "hydra/hip_allreduce_ring.h"

using hydra::detail::LocalStep;

static int failures = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "%s:%d: CHECK(%s)\n", __FILE__, __LINE__, #c); \
      failures++;                                                 \
    }                                                             \
  } while (0)

static bool same(const std::vector<LocalStep>& v, const std::vector<LocalStep>& w) {
  if (v.size() != w.size()) return false;
  for (size_t i = 0; i < v.size(); i++)
    if (v[i].a != w[i].a || v[i].b != w[i].b || v[i].staged != w[i].staged) return false;
  return true;
}

int main() {
  // an 8-GPU node where every pair has peer access (xGMI full mesh)
  auto all = [](int, int) { return true; };
  // a node where devices {0,1,2,3} and {4,5,6,7} only see their own half
  auto halves = [](int a, int b) { return (a < 4) == (b < 4); };
  std::set<std::pair<int, int>> asked;
  auto logged = [&](int a, int b) {
    asked.insert({a, b});
    return true;
  };

  // one device, 1..9 pointers: the pairwise tree, every pointer folded, nothing staged
  for (int n = 1; n <= 9; n++) {
    std::vector<int> dev(n, 0);
    auto t = hydra::detail::local_tree(dev, halves);
    CHECK((int)t.size() == n - 1);  // every pointer except the root is folded exactly once
    std::vector<int> folded(n, 0);
    for (auto& s : t) {
      CHECK(!s.staged);
      CHECK(s.a < s.b);
      folded[s.b]++;
    }
    CHECK(folded[0] == 0);
    for (int i = 1; i < n; i++) CHECK(folded[i] == 1);
  }
  // 4 pointers on 4 devices: (0,1) (2,3) then (0,2) -- the reference's tree in pointer order
  {
    std::vector<int> dev{0, 1, 2, 3};
    CHECK(same(hydra::detail::local_tree(dev, all),
               {{0, 1, false}, {2, 3, false}, {0, 2, false}}));
    // a source is read from its destination's device: peer access is asked (a, b) that way
    asked.clear();
    (void)hydra::detail::local_tree(dev, logged);
    CHECK((asked == std::set<std::pair<int, int>>{{0, 1}, {2, 3}, {0, 2}}));
  }
  // 8 pointers split over two halves without cross access: only the last level stages
  {
    std::vector<int> dev{0, 1, 2, 3, 4, 5, 6, 7};
    auto t = hydra::detail::local_tree(dev, halves);
    CHECK(same(t, {{0, 1, false}, {2, 3, false}, {4, 5, false}, {6, 7, false},
                   {0, 2, false}, {4, 6, false}, {0, 4, true}}));
  }
  // two pointers on one device plus one elsewhere, no peer access: same-device pairs never stage
  {
    std::vector<int> dev{3, 3, 5};
    auto none = [](int, int) { return false; };
    CHECK(same(hydra::detail::local_tree(dev, none), {{0, 1, false}, {0, 2, true}}));
    // the host workspace's order: target = ptrs[0], then += ptrs[1], += ptrs[2]
    CHECK(same(hydra::detail::local_chain(dev, none), {{0, 1, false}, {0, 2, true}}));
  }
  // the host chain on 5 devices with full access: (0,i) in pointer order
  {
    std::vector<int> dev{4, 0, 1, 2, 3};
    CHECK(same(hydra::detail::local_chain(dev, all),
               {{0, 1, false}, {0, 2, false}, {0, 3, false}, {0, 4, false}}));
  }
  // the ring's pointer: smallest distance, first of equals
  CHECK(hydra::detail::closest_index({0, 0, 0}) == 0);
  CHECK(hydra::detail::closest_index({4, 2, 2, 6}) == 1);
  CHECK(hydra::detail::closest_index({7}) == 0);
  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("local steps ok\n");
  return 0;
}
