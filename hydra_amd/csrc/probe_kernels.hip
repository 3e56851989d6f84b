// probe_kernels.hip -- measurement-only kernels for bench.py (libhydra_probe.so, not part of
// the product library): the HBM streaming ceiling of the chip for the access mixes that bound
// the chunk-sum, so the bench line can state the chunk-sum's rate against what THIS HBM
// delivers in the same run, next to the 8 TB/s spec.
//   kind 0  read2 : read a and b (8 B per element), no stores (2R)
//   kind 1  copy  : c = a                      (8 B per element, 1R1W)
// float4 per lane, nontemporal loads, 256-thread blocks, one vector per lane (grid = n/1024
// blocks), the chunk-sum's own launch shape.  (scripts/probe_ceiling.hip is the standalone
// form with the plain c = a + b beside them.)
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace {
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read2(const f4* a, const f4* b, float* sink, size_t nv) {
  f4 acc = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
    acc += __builtin_nontemporal_load(a + i);
    acc += __builtin_nontemporal_load(b + i);
  }
  const float v = acc.x + acc.y + acc.z + acc.w;
  if (v == 12345.678f) sink[blockIdx.x] = v;  // keeps the loads live; (almost) never stores
}

__global__ __launch_bounds__(256) void k_copy(f4* c, const f4* a, size_t nv) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256)
    c[i] = __builtin_nontemporal_load(a + i);
}
}  // namespace

extern "C" {
// n: floats, a multiple of 1024 (bench.py's 64 Mi); sink: >= n / 1024 floats of device memory.
// Returns a hipError_t.
int hydra_probe_launch(int kind, void* c, const void* a, const void* b, void* sink, size_t n,
                       void* stream) {
  if ((n % 1024) != 0 || !a || (kind == 0 && (!b || !sink)) || (kind == 1 && !c))
    return (int)hipErrorInvalidValue;
  const size_t nv = n / 4;
  const unsigned grid = (unsigned)(nv / 256);
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (kind == 0)
    k_read2<<<grid, 256, 0, s>>>(static_cast<const f4*>(a), static_cast<const f4*>(b),
                                 static_cast<float*>(sink), nv);
  else if (kind == 1)
    k_copy<<<grid, 256, 0, s>>>(static_cast<f4*>(c), static_cast<const f4*>(a), nv);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
}
