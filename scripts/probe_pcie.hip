// probe_pcie.hip -- the PCIe ceiling of the host-resident path: what a gfx950
// kernel gets reading / writing pinned host memory in place (zero-copy), against the SDMA
// engines' hipMemcpyAsync rate on the same buffers.  Measurement only; not part of the library.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/probe_pcie scripts/probe_pcie.hip
//   ./scripts/probe_pcie            # JSON lines: test, bytes per operand, grid, median us, GB/s
//
// Every kernel is a bounded grid-stride loop over buffers this program allocated; stores are
// vector stores.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                             \
    }                                                                           \
  } while (0)

__global__ void k_read(const uint4* __restrict__ p, size_t n16, unsigned* out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) out[threadIdx.x] = acc;  // keeps the loads; practically never taken
}

__global__ void k_write(uint4* __restrict__ p, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(i, i, i, i);
}

__global__ void k_add(float4* __restrict__ c, const float4* __restrict__ a,
                      const float4* __restrict__ b, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const float4 x = a[i], y = b[i];
    c[i] = make_float4(x.x + y.x, x.y + y.y, x.z + y.z, x.w + y.w);
  }
}

template <typename F>
static double median_us(hipStream_t s, F&& run, int reps = 15) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  run();  // warm-up
  CK(hipStreamSynchronize(s));
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0, s));
    run();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms * 1000.f);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

static void line(const char* test, size_t bytes, int grid, double us, double moved) {
  std::printf("{\"test\": \"%s\", \"bytes_per_operand\": %zu, \"grid\": %d, \"us\": %.2f, "
              "\"GBps\": %.2f}\n",
              test, bytes, grid, us, moved / (us * 1e-6) / 1e9);
  std::fflush(stdout);
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t maxb = size_t(64) << 20;
  void *ha, *hb, *hc, *dd;
  CK(hipHostMalloc(&ha, maxb, hipHostMallocDefault));
  CK(hipHostMalloc(&hb, maxb, hipHostMallocDefault));
  CK(hipHostMalloc(&hc, maxb, hipHostMallocDefault));
  CK(hipMalloc(&dd, maxb));
  unsigned* sink;
  CK(hipMalloc(&sink, 1024 * sizeof(unsigned)));
  for (size_t i = 0; i < maxb / 4; i++) {
    static_cast<float*>(ha)[i] = float(i & 1023);
    static_cast<float*>(hb)[i] = 1.0f;
  }
  void *da, *db, *dc;
  CK(hipHostGetDevicePointer(&da, ha, 0));
  CK(hipHostGetDevicePointer(&db, hb, 0));
  CK(hipHostGetDevicePointer(&dc, hc, 0));
  const size_t sizes[] = {size_t(1) << 20, size_t(4) << 20, size_t(16) << 20, size_t(64) << 20};
  const int grids[] = {64, 128, 256, 512, 1024};
  for (size_t bytes : sizes) {
    const size_t n16 = bytes / 16;
    line("sdma_h2d", bytes, 0,
         median_us(s, [&] { CK(hipMemcpyAsync(dd, ha, bytes, hipMemcpyHostToDevice, s)); }),
         double(bytes));
    line("sdma_d2h", bytes, 0,
         median_us(s, [&] { CK(hipMemcpyAsync(hc, dd, bytes, hipMemcpyDeviceToHost, s)); }),
         double(bytes));
    for (int g : grids) {
      line("kernel_read", bytes, g, median_us(s, [&] {
             hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, s,
                                static_cast<const uint4*>(da), n16, sink);
           }), double(bytes));
      line("kernel_write", bytes, g, median_us(s, [&] {
             hipLaunchKernelGGL(k_write, dim3(g), dim3(256), 0, s, static_cast<uint4*>(dc), n16);
           }), double(bytes));
      line("kernel_add_2r1w", bytes, g, median_us(s, [&] {
             hipLaunchKernelGGL(k_add, dim3(g), dim3(256), 0, s, static_cast<float4*>(dc),
                                static_cast<const float4*>(da), static_cast<const float4*>(db),
                                n16);
           }), 3.0 * double(bytes));
      line("kernel_add_inplace", bytes, g, median_us(s, [&] {
             hipLaunchKernelGGL(k_add, dim3(g), dim3(256), 0, s, static_cast<float4*>(da),
                                static_cast<const float4*>(da), static_cast<const float4*>(db),
                                n16);
           }), 3.0 * double(bytes));
    }
    CK(hipGetLastError());
  }
  CK(hipStreamSynchronize(s));
  CK(hipHostFree(ha));
  CK(hipHostFree(hb));
  CK(hipHostFree(hc));
  CK(hipFree(dd));
  CK(hipFree(sink));
  CK(hipStreamDestroy(s));
  return 0;
}
