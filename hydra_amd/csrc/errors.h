// errors.h -- status/message plumbing shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

namespace hydra {
int ok();                                     // clears the thread's message, returns HYDRA_OK
int fail(int code, const std::string& msg);   // sets the thread's message, returns code
int hip_fail(hipError_t e, const char* what);
// Measurement variants (A/B kernels, hydra_set_variant) exist only in the measurement build,
// libhydra_measure.so (-DHYDRA_MEASURE, include/hydra_measure.h); the product library always
// runs the tuned defaults.
#ifdef HYDRA_MEASURE
int current_variant();
#else
constexpr int current_variant() { return 0; }
#endif
// hydra_test_set / hydra_test_get's values (hydra_hip.h), readable from every translation unit
int64_t test_value(int key);
void test_count(int key);  // a read-only counter key += 1
}  // namespace hydra

#define HIP_TRY(expr)                                           \
  do {                                                          \
    hipError_t e__ = (expr);                                    \
    if (e__ != hipSuccess) return ::hydra::hip_fail(e__, #expr); \
  } while (0)
