// probe_doorbell.hip -- what would a synchronous chunk-sum call cost if no launch were needed?
// (probe_flag.hip: a fresh launch's dispatch-to-start latency dominates a synchronous call.)
//
// A persistent reducer: ONE launch of G workgroups stays resident; the host posts each call as a
// descriptor {c, a, b, n} plus a sequence number in host-mapped coherent memory and spins on a
// completion word the kernel writes there.
//   workgroup 0 / lane 0 polls the host doorbell (system-scope relaxed loads, s_sleep backoff),
//   copies the descriptor to device memory with write-through (sc1) stores, drains them, and
//   publishes the sequence number in a device word (sc1 store); the other workgroups poll that
//   word with sc1 loads; every workgroup sums its slice (c = a + b, float4, nontemporal loads),
//   drains its stores, releases them (agent scope) and adds to a device counter; the workgroup
//   whose add came last resets the counter and stores the sequence number into the host
//   completion word (system-scope release).
// Every spin is bounded (kTimeoutTicks of s_memrealtime, 100 MHz): a stuck kernel leaves by
// itself with an error code in the host word; the host also stops waiting after 1 s.
// Quit: the host posts sequence number kQuit.
// Prints one JSON line per grid size: mean us per synchronous call (262 144 fp32 elements,
// device-resident) for the persistent reducer and, interleaved, launch + hipStreamSynchronize.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/probe_doorbell scripts/probe_doorbell.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
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

constexpr uint32_t kQuit = 0xFFFFFFFFu;
constexpr uint64_t kTimeoutTicks = 200000000ull;  // 2 s at 100 MHz

struct Desc {  // one call
  f4* c;
  const f4* a;
  const f4* b;
  uint64_t nv;  // float4 count
};

struct HostCtl {       // host-mapped, coherent
  Desc desc;           // written by the host before it rings
  uint32_t seq;        // doorbell: the call's sequence number
  uint32_t pad0[15];
  uint32_t done;       // completion: the sequence number of the last finished call
  uint32_t err;        // non-zero: the kernel gave up (1 = doorbell wait timed out)
  uint32_t pad1[14];
};

struct DevCtl {  // device memory
  Desc desc;
  uint32_t seq;
  uint32_t pad0[15];
  uint32_t counter;
  uint32_t pad1[15];
};

__device__ __forceinline__ uint32_t ld_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(256) void k_persistent(HostCtl* h, DevCtl* d) {
  __shared__ uint32_t s_seq;
  __shared__ Desc s_desc;
  uint32_t last = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t s;
      if (blockIdx.x == 0) {
        while ((s = ld_sys(&h->seq)) == last) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            s = kQuit;
            __hip_atomic_store(&h->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the descriptor the host wrote first
        if (s != kQuit) {  // all four loads in flight at once (one host round trip), then store
          const uint64_t* src = reinterpret_cast<const uint64_t*>(&h->desc);
          uint64_t* dst = reinterpret_cast<uint64_t*>(&d->desc);
          uint64_t v[4];
          for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(src + k);
          for (int k = 0; k < 4; k++)
            __hip_atomic_store(dst + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&d->seq, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while ((s = ld_agent(&d->seq)) == last) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks) {
            s = kQuit;
            break;
          }
        }
      }
      s_seq = s;
      if (s != kQuit) {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&d->desc);
        uint64_t* dst = reinterpret_cast<uint64_t*>(&s_desc);
        for (int k = 0; k < 4; k++)
          dst[k] = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
    const uint32_t s = s_seq;
    if (s == kQuit) return;
    last = s;
    const Desc D = s_desc;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < D.nv;
         i += (uint64_t)gridDim.x * 256)
      D.c[i] = D.a[i] + __builtin_nontemporal_load(D.b + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t old =
          __hip_atomic_fetch_add(&d->counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (old == gridDim.x - 1) {
        __hip_atomic_store(&d->counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&h->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();  // s_seq / s_desc are rewritten by thread 0 next round
  }
}

__global__ __launch_bounds__(256) void k_sum(f4* c, const f4* a, const f4* b, uint64_t nv) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nv;
       i += (uint64_t)gridDim.x * 256)
    c[i] = a[i] + __builtin_nontemporal_load(b + i);
}

int main(int argc, char** argv) {
  const size_t n = 262144, nv = n / 4;
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  f4 *c, *a, *b;
  CK(hipMalloc(&c, n * sizeof(float)));
  CK(hipMalloc(&a, n * sizeof(float)));
  CK(hipMalloc(&b, n * sizeof(float)));
  CK(hipMemset(c, 0, n * sizeof(float)));
  CK(hipMemset(a, 0, n * sizeof(float)));
  CK(hipMemset(b, 0, n * sizeof(float)));
  HostCtl* h;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(HostCtl),
                   hipHostMallocMapped | hipHostMallocCoherent));
  HostCtl* h_dev;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_dev), h, 0));
  DevCtl* d;
  CK(hipMalloc(&d, sizeof(DevCtl)));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  int rc = 0;
  for (unsigned grid : {1u, 8u, 32u, 64u, 256u}) {
    std::memset(h, 0, sizeof(HostCtl));
    CK(hipMemset(d, 0, sizeof(DevCtl)));
    CK(hipDeviceSynchronize());
    k_persistent<<<grid, 256, 0, s>>>(h_dev, d);
    CK(hipGetLastError());
    uint32_t seq = 0;
    int failed = 0;
    double t_db = 0, t_sync = 0;
    for (int round = 0; round < 2 && !failed; round++) {  // round 0 warms up
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters && !failed; i++) {
        h->desc = Desc{c, a, b, nv};
        ++seq;
        __atomic_store_n(&h->seq, seq, __ATOMIC_RELEASE);
        const auto ts = std::chrono::steady_clock::now();
        while (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != seq) {
          if (__atomic_load_n(&h->err, __ATOMIC_RELAXED) ||
              std::chrono::steady_clock::now() - ts > std::chrono::seconds(1)) {
            failed = 1;
            break;
          }
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      if (round == 1) t_db = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    }
    // the same call as a fresh launch + hipStreamSynchronize, on another stream meanwhile
    // (the persistent grid holds `grid` CUs; the rest of the chip runs this)
    if (!failed) {
      for (int round = 0; round < 2; round++) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; i++) {
          k_sum<<<256, 256, 0, s2>>>(c, a, b, nv);
          CK(hipStreamSynchronize(s2));
        }
        auto t1 = std::chrono::steady_clock::now();
        if (round == 1) t_sync = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
      }
    }
    __atomic_store_n(&h->seq, kQuit, __ATOMIC_RELEASE);  // every workgroup leaves
    CK(hipStreamSynchronize(s));
    std::printf("{\"grid\": %u, \"elements\": %zu, \"failed\": %d, \"kernel_err\": %u, "
                "\"doorbell_us\": %.2f, \"launch_sync_us\": %.2f}\n",
                grid, n, failed, h->err, t_db, t_sync);
    std::fflush(stdout);
    if (failed) {
      rc = 1;
      break;
    }
  }
  CK(hipStreamDestroy(s));
  CK(hipStreamDestroy(s2));
  CK(hipFree(d));
  CK(hipHostFree(h));
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(c));
  return rc;
}
