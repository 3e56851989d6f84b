// reduce_kernels.h -- launcher declarations shared by the C-ABI (hydra_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace hydra {

constexpr int kBlock = 256;  // 4 waves of 64 lanes
constexpr int kMaxRanks = 16;  // P-way fold fan-in limit

enum Op { kSum = 0, kProduct = 1, kMax = 2, kMin = 3 };
enum DType { kI8 = 0, kU8, kI32, kU32, kI64, kU64, kF32, kF64, kF16, kBF16 };

inline size_t dtype_size(int d) {
  static const size_t sz[] = {1, 1, 4, 4, 8, 8, 4, 8, 2, 2};
  return (d >= 0 && d <= 9) ? sz[d] : 0;
}

// c[i] = op(a[i], b[i]); variant 0 = tuned default (see reduce_kernels.hip launch_variant)
hipError_t launch_reduce(int variant, int op, int dtype, void* c, const void* a, const void* b,
                         size_t n, hipStream_t s);
// dst = srcs[0] + (srcs[1] + (... + srcs[nsrc-1])) element-wise (reference ring fold order);
// acc32: bf16 data, fp32 accumulation, one rounding.  dst may equal srcs[0].
hipError_t launch_fold(int op, int dtype, bool acc32, void* dst, const void* const* srcs,
                       int nsrc, size_t n, hipStream_t s);
// K independent segments c_k = op(a_k, b_k) in as few launches as possible (kMaxBatch each)
constexpr int kMaxBatch = 32;
struct BatchSegDesc {
  void* c;
  const void* a;
  const void* b;
  size_t n;
};
hipError_t launch_reduce_batch(int op, int dtype, const BatchSegDesc* segs, size_t count,
                               hipStream_t s);
hipError_t launch_acc_bf16_f32(float* acc, const void* b_bf16, size_t n, hipStream_t s);
hipError_t launch_f32_to_bf16(void* out_bf16, const float* acc, size_t n, hipStream_t s);

}  // namespace hydra
