// probe_sync.hip -- what a synchronous call pays to learn that its kernel finished
// (hydra_reduce_host and the Func shims are synchronous, as the reference's sum is).
// One small kernel per call, then one of:
//   stream_sync : hipStreamSynchronize
//   event_sync  : hipEventRecord + hipEventSynchronize
//   query_spin  : hipStreamQuery in a loop until it stops returning hipErrorNotReady
// Prints the mean microseconds per call for each, interleaved over several rounds.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/probe_sync scripts/probe_sync.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

__global__ void k_add(float* c, const float* a, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = c[i] + a[i];
}

int main() {
  const int n = 1024, iters = 2000, rounds = 5;
  float *c, *a;
  CK(hipMalloc(&c, n * sizeof(float)));
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMemset(c, 0, n * sizeof(float)));
  CK(hipMemset(a, 0, n * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  double tot[3] = {0, 0, 0};
  for (int r = 0; r < rounds; r++) {
    for (int m = 0; m < 3; m++) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; i++) {
        k_add<<<(n + 255) / 256, 256, 0, s>>>(c, a, n);
        if (m == 0) {
          CK(hipStreamSynchronize(s));
        } else if (m == 1) {
          CK(hipEventRecord(ev, s));
          CK(hipEventSynchronize(ev));
        } else {
          hipError_t q;
          while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
          }
          CK(q);
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      if (r > 0) tot[m] += std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    }
  }
  const char* names[3] = {"stream_sync", "event_sync", "query_spin"};
  std::printf("{");
  for (int m = 0; m < 3; m++)
    std::printf("\"%s_us\": %.2f%s", names[m], tot[m] / (rounds - 1), m < 2 ? ", " : "");
  std::printf("}\n");
  CK(hipEventDestroy(ev));
  CK(hipStreamDestroy(s));
  CK(hipFree(c));
  CK(hipFree(a));
  return 0;
}
