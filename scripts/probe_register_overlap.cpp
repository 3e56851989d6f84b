// Probe (no kernel touches any memory): how HIP treats hipHostRegister of overlapping / nested
// ranges and what HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR / RANGE_SIZE report for registered
// host memory -- the facts an on-the-fly pinning policy in hydra_reduce_host rests on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

static void attrs(const char* tag, void* p) {
  hipPointerAttribute_t at{};
  hipError_t e = hipPointerGetAttributes(&at, p);
  void* start = nullptr;
  size_t size = 0;
  hipError_t e1 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                         reinterpret_cast<hipDeviceptr_t>(p));
  hipError_t e2 = hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                         reinterpret_cast<hipDeviceptr_t>(p));
  std::printf("%-28s attrs=%d type=%d host=%p dev=%p | range_start(e=%d)=%p range_size(e=%d)=%zu\n",
              tag, (int)e, (int)at.type, at.hostPointer, at.devicePointer, (int)e1, start, (int)e2,
              size);
  (void)hipGetLastError();
}

int main() {
  const size_t MiB = 1 << 20;
  char* p = static_cast<char*>(std::aligned_alloc(4096, 4 * MiB));
  std::printf("base %p\n", (void*)p);
  hipError_t r1 = hipHostRegister(p + 100, MiB, hipHostRegisterDefault);
  std::printf("register R1 [p+100, +1MiB): %d\n", (int)r1);
  attrs("p+100", p + 100);
  attrs("p+200", p + 200);
  attrs("p+1MiB+50 (past R1 end)", p + MiB + 50);
  hipError_t r2 = hipHostRegister(p + MiB + 50, MiB, hipHostRegisterDefault);
  std::printf("register R2 [p+1MiB+50, +1MiB) (shares a page with R1): %d\n", (int)r2);
  (void)hipGetLastError();
  attrs("p+1MiB+60", p + MiB + 60);
  hipError_t r3 = hipHostRegister(p + 4096, 8192, hipHostRegisterDefault);
  std::printf("register R3 [p+4096, +8KiB) (nested in R1): %d\n", (int)r3);
  (void)hipGetLastError();
  attrs("p+4096", p + 4096);
  hipError_t u1 = hipHostUnregister(p + 100);
  std::printf("unregister R1: %d\n", (int)u1);
  (void)hipGetLastError();
  attrs("p+200 after R1 unregister", p + 200);
  attrs("p+1MiB+60 after R1 unreg", p + MiB + 60);
  hipError_t u2 = hipHostUnregister(p + MiB + 50);
  std::printf("unregister R2: %d\n", (int)u2);
  hipError_t u3 = hipHostUnregister(p + 4096);
  std::printf("unregister R3: %d\n", (int)u3);
  (void)hipGetLastError();
  std::free(p);
  return 0;
}
