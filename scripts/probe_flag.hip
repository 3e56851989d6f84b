// probe_flag.hip -- can a synchronous chunk-sum call learn of its kernel's completion faster
// than the HIP runtime's own wait?  (probe_sync.hip measured the runtime's waits: a
// synchronous call of a trivial kernel costs ~11 us with hipStreamSynchronize.)
//
// One 1 MiB ring segment per call (262 144 fp32, c = a + b in place, device-resident), each
// call followed by one completion wait:
//   stream_sync : hipStreamSynchronize
//   flag_spin   : the kernel itself reports completion: every workgroup drains its stores,
//                 releases them (system scope) and adds to a device counter; the workgroup
//                 whose add came last resets the counter and stores the call's sequence number
//                 into a host-mapped coherent word (system-scope release); the host spins on
//                 that word (bounded: 1 s, then the probe fails).
//   launch_only : no wait at all (back-to-back enqueue rate, for reference)
// argv[1] = "spin" sets hipDeviceScheduleSpin before the runtime initialises the device.
// Prints one JSON line: mean us per call for each mode over interleaved rounds, and the grid.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/probe_flag scripts/probe_flag.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool kFlag>
__global__ __launch_bounds__(256) void k_sum(f4* c, const f4* b, size_t nv, unsigned* counter,
                                             unsigned* done, unsigned seq) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256)
    c[i] = c[i] + __builtin_nontemporal_load(b + i);
  if (!kFlag) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: this workgroup's stores out
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old =
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {  // last arrival: every workgroup's stores are released
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

int main(int argc, char** argv) {
  if (argc > 1 && !std::strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  const size_t n = 262144, nv = n / 4;
  const int iters = 2000, rounds = 5;
  const unsigned grid = argc > 2 ? (unsigned)std::atoi(argv[2]) : 256;
  f4 *c, *b;
  unsigned *counter, *done;
  CK(hipMalloc(&c, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMalloc(&counter, 64));
  CK(hipMemset(c, 0, n * sizeof(float)));
  CK(hipMemset(b, 0, n * sizeof(float)));
  CK(hipMemset(counter, 0, 64));
  CK(hipHostMalloc(reinterpret_cast<void**>(&done), 64, hipHostMallocMapped | hipHostMallocCoherent));
  *done = 0;
  unsigned* done_dev;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&done_dev), done, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipDeviceSynchronize());
  unsigned seq = 0;
  double tot[3] = {0, 0, 0};
  int failed = 0;
  for (int r = 0; r < rounds && !failed; r++) {
    for (int m = 0; m < 3 && !failed; m++) {
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; i++) {
        if (m == 0) {
          k_sum<false><<<grid, 256, 0, s>>>(c, b, nv, counter, done_dev, 0);
          CK(hipStreamSynchronize(s));
        } else if (m == 1) {
          ++seq;
          k_sum<true><<<grid, 256, 0, s>>>(c, b, nv, counter, done_dev, seq);
          const auto ts = std::chrono::steady_clock::now();
          while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != seq) {
            if (std::chrono::steady_clock::now() - ts > std::chrono::seconds(1)) {
              failed = 1;
              break;
            }
          }
          if (failed) break;
        } else {
          k_sum<false><<<grid, 256, 0, s>>>(c, b, nv, counter, done_dev, 0);
        }
      }
      CK(hipStreamSynchronize(s));
      auto t1 = std::chrono::steady_clock::now();
      if (r > 0) tot[m] += std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    }
  }
  CK(hipStreamSynchronize(s));
  std::printf("{\"sched\": \"%s\", \"grid\": %u, \"elements\": %zu, \"failed\": %d, "
              "\"stream_sync_us\": %.2f, \"flag_spin_us\": %.2f, \"launch_only_us\": %.2f}\n",
              argc > 1 ? argv[1] : "auto", grid, n, failed, tot[0] / (rounds - 1),
              tot[1] / (rounds - 1), tot[2] / (rounds - 1));
  CK(hipStreamDestroy(s));
  CK(hipHostFree(done));
  CK(hipFree(counter));
  CK(hipFree(b));
  CK(hipFree(c));
  return failed;
}
