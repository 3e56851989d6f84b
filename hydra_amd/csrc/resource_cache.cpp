// resource_cache.cpp -- see resource_cache.h.
#include "resource_cache.h"

#include "fault_report.h"
#include "host_map.h"
#include "resident.h"

#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace hydra {
namespace {

constexpr size_t kGranule = size_t(64) << 10;
constexpr size_t kMaxCachedDevice = size_t(4) << 30;  // per device
constexpr size_t kMaxCachedHost = size_t(2) << 30;
constexpr size_t kMaxCachedHandles = 64;  // streams / events per device

size_t size_class(size_t b) { return ((b ? b : 1) + kGranule - 1) / kGranule * kGranule; }

struct BlockKey {
  bool host;
  int device;  // -1 for pinned host blocks
  size_t bytes;
  bool operator<(const BlockKey& o) const {
    return std::tie(host, device, bytes) < std::tie(o.host, o.device, o.bytes);
  }
};

struct Caches {
  std::mutex m;
  std::unordered_map<void*, BlockKey> live_blocks;  // handed out, not yet released
  std::multimap<BlockKey, void*> blocks;            // kept for reuse
  std::unordered_set<void*> kept;                   // the pointers in `blocks`
  std::map<int, size_t> kept_bytes;                 // per device; -1 = pinned host
  std::unordered_map<hipStream_t, int> live_streams;
  std::multimap<int, hipStream_t> streams;
  std::unordered_set<hipStream_t> kept_streams;
  std::unordered_map<hipEvent_t, int> live_events;
  std::multimap<int, hipEvent_t> events;
  std::unordered_set<hipEvent_t> kept_events;
};

// Never destroyed: no HIP call may run from a static destructor after the runtime is gone.
Caches& C() {
  static Caches* c = new Caches;
  return *c;
}

// Devices hydra has created streams, events or blocks on (bit d), plus the caller's current one:
// the devices whose kernels may be reading a pinned block.  Touching any other device would
// create a context on it.
std::atomic<uint64_t> g_devices{0};
void note_device(int d) {
  if (d >= 0 && d < 64) g_devices.fetch_or(uint64_t(1) << d, std::memory_order_relaxed);
}

// Drains those devices; the caller's current device is left as it was.
hipError_t sync_all_devices() {
  ResidentPause pause_(-1);  // a serving resident reducer would hold the drain up indefinitely
  int cur = -1;
  if (hipGetDevice(&cur) == hipSuccess) note_device(cur);
  const uint64_t m = g_devices.load(std::memory_order_relaxed);
  hipError_t e = hipSuccess;
  for (int d = 0; d < 64 && e == hipSuccess; d++) {
    if (!(m >> d & 1)) continue;
    DeviceScope ds(d);
    e = ds.err != hipSuccess ? ds.err : hipDeviceSynchronize();
  }
  return e;
}

hipError_t take_block(const BlockKey& k, void** out) {
  Caches& c = C();
  {
    std::lock_guard<std::mutex> g(c.m);
    auto it = c.blocks.find(k);
    if (it != c.blocks.end()) {
      *out = it->second;
      c.blocks.erase(it);
      c.kept.erase(*out);
      c.kept_bytes[k.host ? -1 : k.device] -= k.bytes;
      c.live_blocks[*out] = k;
      return hipSuccess;
    }
  }
  void* p = nullptr;
  hipError_t e =
      k.host ? hipHostMalloc(&p, k.bytes, hipHostMallocDefault) : hipMalloc(&p, k.bytes);
  if (e != hipSuccess) return e;
  ledger_add(k.host ? kLedgerPinnedBlock : kLedgerDeviceBlock, p, k.bytes);
  if (k.host) host_map_add_block(p, k.bytes);  // zero-copy operands may lie in it
  std::lock_guard<std::mutex> g(c.m);
  c.live_blocks[p] = k;
  *out = p;
  return hipSuccess;
}

hipError_t give_block(void* p, bool host) {
  if (!p) return hipSuccess;
  Caches& c = C();
  BlockKey k{};
  {
    std::lock_guard<std::mutex> g(c.m);
    if (c.kept.count(p)) return hipErrorInvalidValue;  // released twice
    auto it = c.live_blocks.find(p);
    if (it == c.live_blocks.end() || it->second.host != host)  // not ours: release directly
      return host ? hipHostFree(p) : hipFree(p);
    k = it->second;
    c.live_blocks.erase(it);  // a second release of p now fails above or below, never twice
  }
  // hipFree's implicit synchronisation: work enqueued before the release may still use p (a
  // pinned block: on any device -- the kernels of every device can read it in place).  The
  // resident reducer is stopped for the drain and the free (both wait for every stream).
  ResidentPause pause_(-1);
  hipError_t e = k.host ? sync_all_devices() : hipSuccess;
  if (!k.host) {
    DeviceScope ds(k.device);
    e = hipDeviceSynchronize();
  }
  {
    std::lock_guard<std::mutex> g(c.m);
    size_t& kept = c.kept_bytes[k.host ? -1 : k.device];
    if (e == hipSuccess && kept + k.bytes <= (k.host ? kMaxCachedHost : kMaxCachedDevice)) {
      kept += k.bytes;
      c.blocks.emplace(k, p);
      c.kept.insert(p);
      return hipSuccess;
    }
  }
  DeviceScope ds(k.host ? -1 : k.device);
  if (k.host) host_map_remove_block(p);
  hipError_t f = k.host ? hipHostFree(p) : hipFree(p);
  ledger_release(k.host ? kLedgerPinnedBlock : kLedgerDeviceBlock, p);
  return e != hipSuccess ? e : f;
}

}  // namespace

hipError_t cached_malloc(int device, size_t bytes, void** out) {
  if (device < 0) return hipErrorInvalidDevice;
  DeviceScope ds(device);  // the caller's current device is left as it was
  if (ds.err != hipSuccess) return ds.err;
  note_device(device);
  return take_block(BlockKey{false, device, size_class(bytes)}, out);
}

hipError_t cached_free(void* p) { return give_block(p, false); }

hipError_t cached_malloc_host(size_t bytes, void** out) {
  return take_block(BlockKey{true, -1, size_class(bytes)}, out);
}

hipError_t cached_free_host(void* p) { return give_block(p, true); }

hipError_t cached_stream(int device, hipStream_t* out) {
  if (device < 0) return hipErrorInvalidDevice;
  DeviceScope ds(device);  // the caller's current device is left as it was
  if (ds.err != hipSuccess) return ds.err;
  note_device(device);
  Caches& c = C();
  {
    std::lock_guard<std::mutex> g(c.m);
    auto it = c.streams.find(device);
    if (it != c.streams.end()) {
      *out = it->second;
      c.streams.erase(it);
      c.kept_streams.erase(*out);
      c.live_streams[*out] = device;
      return hipSuccess;
    }
  }
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(c.m);
  c.live_streams[s] = device;
  *out = s;
  return hipSuccess;
}

hipError_t release_stream(hipStream_t s) {
  if (!s) return hipSuccess;
  Caches& c = C();
  int device;
  {
    std::lock_guard<std::mutex> g(c.m);
    if (c.kept_streams.count(s)) return hipErrorInvalidValue;  // released twice
    auto it = c.live_streams.find(s);
    if (it == c.live_streams.end()) return hipStreamDestroy(s);
    device = it->second;
    c.live_streams.erase(it);
  }
  hipError_t e = hipStreamSynchronize(s);
  {
    std::lock_guard<std::mutex> g(c.m);
    if (e == hipSuccess && c.streams.count(device) < kMaxCachedHandles) {
      c.streams.emplace(device, s);
      c.kept_streams.insert(s);
      return hipSuccess;
    }
  }
  DeviceScope ds(device);
  hipError_t f = hipStreamDestroy(s);
  return e != hipSuccess ? e : f;
}

hipError_t cached_event(int device, hipEvent_t* out) {
  hipError_t e = hipSuccess;
  if (device < 0) e = hipGetDevice(&device);
  if (e != hipSuccess) return e;
  DeviceScope ds(device);  // created on `device`; the caller's current device is left as it was
  if (ds.err != hipSuccess) return ds.err;
  note_device(device);
  Caches& c = C();
  {
    std::lock_guard<std::mutex> g(c.m);
    auto it = c.events.find(device);
    if (it != c.events.end()) {
      *out = it->second;
      c.events.erase(it);
      c.kept_events.erase(*out);
      c.live_events[*out] = device;
      return hipSuccess;
    }
  }
  hipEvent_t ev = nullptr;
  e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(c.m);
  c.live_events[ev] = device;
  *out = ev;
  return hipSuccess;
}

hipError_t release_event(hipEvent_t ev) {
  if (!ev) return hipSuccess;
  Caches& c = C();
  int device;
  {
    std::lock_guard<std::mutex> g(c.m);
    if (c.kept_events.count(ev)) return hipErrorInvalidValue;  // released twice
    auto it = c.live_events.find(ev);
    if (it == c.live_events.end()) return hipEventDestroy(ev);
    device = it->second;
    c.live_events.erase(it);
  }
  hipError_t e = hipEventSynchronize(ev);  // its last record (if any) has completed
  {
    std::lock_guard<std::mutex> g(c.m);
    if (e == hipSuccess && c.events.count(device) < kMaxCachedHandles) {
      c.events.emplace(device, ev);
      c.kept_events.insert(ev);
      return hipSuccess;
    }
  }
  DeviceScope ds(device);
  hipError_t f = hipEventDestroy(ev);
  return e != hipSuccess ? e : f;
}

hipError_t trim_caches() {
  Caches& c = C();
  std::multimap<BlockKey, void*> blocks;
  std::multimap<int, hipStream_t> streams;
  std::multimap<int, hipEvent_t> events;
  {
    std::lock_guard<std::mutex> g(c.m);
    blocks.swap(c.blocks);
    streams.swap(c.streams);
    events.swap(c.events);
    c.kept.clear();
    c.kept_streams.clear();
    c.kept_events.clear();
    c.kept_bytes.clear();
  }
  ResidentPause pause_(-1);  // hipFree / hipHostFree synchronise the device
  hipError_t first = hipSuccess;
  auto note = [&first](hipError_t e) {
    if (e != hipSuccess && first == hipSuccess) first = e;
  };
  for (auto& kv : events) {
    DeviceScope ds(kv.first);
    note(hipEventDestroy(kv.second));
  }
  for (auto& kv : streams) {
    DeviceScope ds(kv.first);
    note(hipStreamDestroy(kv.second));
  }
  for (auto& kv : blocks) {
    DeviceScope ds(kv.first.host ? -1 : kv.first.device);
    if (kv.first.host) host_map_remove_block(kv.second);
    note(kv.first.host ? hipHostFree(kv.second) : hipFree(kv.second));
    ledger_release(kv.first.host ? kLedgerPinnedBlock : kLedgerDeviceBlock, kv.second);
  }
  return first;
}

}  // namespace hydra
