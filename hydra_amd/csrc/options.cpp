// options.cpp -- storage of the library options (options.h): plain C++, no HIP, so host-only
// units (copy_pool.cpp under the sanitizer tests) link it alone.
#include "options.h"

namespace hydra {
namespace {
std::atomic<int64_t> g_opt[kOptCount] = {};
std::atomic<bool> g_opt_set[kOptCount] = {};
}  // namespace

int64_t opt(int key) {
  if (key <= 0 || key >= kOptCount) return 0;
  return g_opt_set[key].load(std::memory_order_acquire) ? g_opt[key].load(std::memory_order_relaxed)
                                                        : opt_spec(key).dflt;
}

void opt_set(int key, int64_t value) {
  if (key <= 0 || key >= kOptCount) return;
  g_opt[key].store(value, std::memory_order_relaxed);
  g_opt_set[key].store(true, std::memory_order_release);
}

}  // namespace hydra
