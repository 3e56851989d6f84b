// Compile check + usage sketch of include/hydra/gloo_reduce.h (no GPU needed to build).
//   g++ -std=c++14 -Iinclude examples/gloo_shim_example.cc -Lhydra_amd -lhydra_hip
// In a hydra/Gloo build the same line replaces `&gloo::sum<float>`:
//   opts.setReduceFunction(hydra::gloo_compat::hostSum<float>());
#include <cstdio>
#include <vector>

#include "hydra/gloo_reduce.h"

int main() {
  int ndev = 0;
  if (hydra_device_count(&ndev) != HYDRA_OK || ndev == 0) {
    std::printf("no GPU: %s\n", hydra_last_error());
    return 0;
  }
  std::vector<float> a(1000, 1.0f), b(1000, 2.0f);
  auto fn = hydra::gloo_compat::hostSum<float>();
  fn(a.data(), a.data(), b.data(), a.size());  // the ring's in-place call (allreduce.cc:301)
  hydra::gloo_compat::hostSumInPlace<float>(a.data(), b.data(), a.size());
  std::printf("a[0] = %g (expect 5)\n", a[0]);
  return a[0] == 5.0f ? 0 : 1;
}
