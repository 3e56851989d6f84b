// copy_pool_stress.cc -- hydra_amd/csrc/copy_pool.cpp under concurrent callers (CPU only; run
// under ThreadSanitizer and AddressSanitizer by tests/test_sanitizers.py): 4 threads -- the
// rails of bew_allreduce_a and more -- each copy_all()s job lists of ragged sizes around the
// fan-out threshold and checks every byte.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../hydra_amd/csrc/copy_pool.h"

int main() {
  std::vector<std::thread> th;
  std::vector<int> bad(4, 0);
  for (int t = 0; t < 4; t++)
    th.emplace_back([t, &bad] {
      unsigned seed = 1234u + t;
      for (int it = 0; it < 60; it++) {
        const int njobs = 1 + (int)(rand_r(&seed) % 4);
        std::vector<std::vector<unsigned char>> src(njobs), dst(njobs);
        std::vector<hydra::CopyJob> jobs;
        for (int j = 0; j < njobs; j++) {
          const size_t bytes = (rand_r(&seed) % 3 == 0) ? rand_r(&seed) % 4096
                                                          : (size_t)(rand_r(&seed) % (600u << 10));
          src[j].resize(bytes);
          dst[j].assign(bytes + 64, 0xEE);  // guard bytes past the copy
          for (size_t k = 0; k < bytes; k++) src[j][k] = (unsigned char)(k * 131 + j + it + t);
          jobs.push_back({dst[j].data(), src[j].data(), bytes});
        }
        hydra::copy_all(jobs.data(), jobs.size());
        for (int j = 0; j < njobs; j++) {
          const size_t bytes = src[j].size();
          if (std::memcmp(dst[j].data(), src[j].data(), bytes) != 0) bad[t]++;
          for (size_t k = bytes; k < bytes + 64; k++)
            if (dst[j][k] != 0xEE) bad[t]++;
        }
      }
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < 4; t++)
    if (bad[t]) {
      std::printf("FAIL thread %d: %d\n", t, bad[t]);
      return 1;
    }
  std::printf("OK\n");
  return 0;
}
