// probe_ceiling.hip -- the HBM streaming ceiling of this MI355X for the three access mixes that
// bound the chunk-sum, measured under the same HBM-resident condition as bench.py's headline
// (launch k works on buffer set k mod 4; 4 sets of 3 x 256 MiB = 3 GiB >> the 256 MiB MALL):
//   read   : 2 streams read, one float per workgroup written   (2R)
//   copy   : 1 stream read, 1 written                          (1R1W, the guide's float4 copy)
//   add    : 2 streams read, 1 written, c = a + b              (2R1W, what k_reduce does)
// Each kernel: float4 (16 B) per lane, grid-stride over contiguous tiles, nontemporal loads,
// 256-thread blocks, 8 x 256 workgroups per XCD-dealt wave of the dispatcher (grid = 65536
// blocks for 64 Mi floats).  Reported: TB/s of algorithmic bytes, median over 5 rounds of 40
// launches (event span / launches).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probe_ceiling scripts/probe_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const f4* a, const f4* b, float* out, size_t nv) {
  f4 acc = {0, 0, 0, 0};
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
    acc += __builtin_nontemporal_load(a + i);
    acc += __builtin_nontemporal_load(b + i);
  }
  float v = acc.x + acc.y + acc.z + acc.w;
  if (v == 12345.678f) out[blockIdx.x] = v;  // keeps the loads live, (almost) never stores
}

__global__ __launch_bounds__(256) void k_copy(f4* c, const f4* a, size_t nv) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256)
    c[i] = __builtin_nontemporal_load(a + i);
}

__global__ __launch_bounds__(256) void k_add(f4* c, const f4* a, const f4* b, size_t nv) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256)
    c[i] = __builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i);
}

int main() {
  const size_t n = size_t(64) << 20, nv = n / 4, bytes = n * 4;
  const int sets = 4, launches = 40, rounds = 5;
  const unsigned grid = (unsigned)(nv / 256);
  std::vector<f4*> A(sets), B(sets), C(sets);
  for (int s = 0; s < sets; s++) {
    CK(hipMalloc(&A[s], bytes));
    CK(hipMalloc(&B[s], bytes));
    CK(hipMalloc(&C[s], bytes));
    CK(hipMemset(A[s], 0, bytes));
    CK(hipMemset(B[s], 0, bytes));
    CK(hipMemset(C[s], 0, bytes));
  }
  float* out;
  CK(hipMalloc(&out, grid * sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[3] = {"read_2R", "copy_1R1W", "add_2R1W"};
  const double algo[3] = {8.0 * n, 8.0 * n, 12.0 * n};
  std::vector<double> res[3];
  for (int r = 0; r < rounds + 1; r++) {
    for (int m = 0; m < 3; m++) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < launches; k++) {
        const int s = k % sets;
        if (m == 0) k_read<<<grid, 256>>>(A[s], B[s], out, nv);
        else if (m == 1) k_copy<<<grid, 256>>>(C[s], A[s], nv);
        else k_add<<<grid, 256>>>(A[s], A[s], B[s], nv);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r > 0) res[m].push_back(algo[m] / (ms * 1e-3 / launches) / 1e12);
    }
  }
  CK(hipGetLastError());
  std::printf("{\"elements\": %zu, \"buffer_sets\": %d, \"launches_per_round\": %d", n, sets,
              launches);
  for (int m = 0; m < 3; m++) {
    std::sort(res[m].begin(), res[m].end());
    std::printf(", \"%s_TBps\": %.3f", names[m], res[m][res[m].size() / 2]);
  }
  std::printf("}\n");
  for (int s = 0; s < sets; s++) {
    CK(hipFree(A[s]));
    CK(hipFree(B[s]));
    CK(hipFree(C[s]));
  }
  CK(hipFree(out));
  return 0;
}
