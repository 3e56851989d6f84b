// resource_cache.h -- process-wide caches of the HIP objects hydra creates per call or per
// algorithm object: device blocks, pinned host blocks, streams and events.
//
// A ring class built per bucket (the reference's CudaAllreduceRing allocates its scratch and
// streams in the constructor), a communicator per process group and the one-GPU simulator per
// call would otherwise pay hipMalloc / hipHostMalloc / stream creation every time, and every
// release would be a hipFree / hipStreamDestroy.  Like torch's caching allocator, released
// objects are kept and handed out again:
//   * blocks are matched by size class (64 KiB granules) and device; a release first drains the
//     device (hipFree's own implicit synchronisation, so a cached block is never handed out
//     while work enqueued before its release may still touch it); at most kMaxCachedDevice /
//     kMaxCachedHost bytes are kept, the rest is really freed;
//   * streams are synchronised and events waited on before they are kept (at most 64 each);
//   * pointers the caches did not hand out are freed / destroyed directly; releasing a kept
//     object again (a double free) fails with hipErrorInvalidValue instead of freeing memory
//     the cache would hand out later;
//   * trim_caches() really frees everything kept (hydra_cache_trim in the C-ABI).
// Every function returns the first HIP error it met (hipSuccess otherwise).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace hydra {

hipError_t cached_malloc(int device, size_t bytes, void** out);
hipError_t cached_free(void* p);
hipError_t cached_malloc_host(size_t bytes, void** out);
hipError_t cached_free_host(void* p);
hipError_t cached_stream(int device, hipStream_t* out);  // non-blocking
hipError_t release_stream(hipStream_t s);
hipError_t cached_event(int device, hipEvent_t* out);  // hipEventDisableTiming; -1: current device
hipError_t release_event(hipEvent_t e);
hipError_t trim_caches();

// Makes `device` current for a scope and restores the caller's device (every C-ABI entry that
// works on an object bound to a device opens one: the caller's current device is never changed).
struct DeviceScope {
  int old = -1;
  hipError_t err = hipSuccess;  // of switching to `device` (an invalid device fails here)
  explicit DeviceScope(int device) {
    if (hipGetDevice(&old) != hipSuccess) old = -1;
    if (device >= 0 && device != old) err = hipSetDevice(device);
  }
  ~DeviceScope() {
    if (old >= 0) (void)hipSetDevice(old);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

}  // namespace hydra
