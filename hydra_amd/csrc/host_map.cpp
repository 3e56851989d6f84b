// host_map.cpp -- see host_map.h.
#include "host_map.h"

#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <utility>
#include <vector>
#include <mutex>

#include "../../include/hydra_hip.h"
#include "fault_report.h"

namespace hydra {

size_t page_size() {
  static const size_t ps = [] {
    const long v = sysconf(_SC_PAGESIZE);
    return v > 0 ? size_t(v) : size_t(4096);
  }();
  return ps;
}

void page_interior(uintptr_t p, size_t bytes, uintptr_t* lo, uintptr_t* hi) {
  const uintptr_t ps = page_size();
  const uintptr_t end = p + bytes;
  uintptr_t l = (p + ps - 1) / ps * ps;
  uintptr_t h = end / ps * ps;
  if (end < p || l >= h) l = h = 0;  // wrapped, or no whole page inside
  *lo = l;
  *hi = h;
}

namespace {

struct Entry {
  uintptr_t hi;
  char* dev;  // device address of the entry's first byte
  int kind;
  int owners;  // hydra_host_register callers sharing the entry
  int users;   // windows held by in-flight calls
  bool pending = false;  // hipHostRegister in progress (outside the lock)
  bool dying = false;    // hipHostUnregister in progress (outside the lock)
  uintptr_t owner_lo, owner_hi;
};

struct Caller {
  size_t bytes;
  int count;
  uintptr_t key;  // entry holding the interior pages (0: nothing registered for it)
};

struct Registry {
  std::mutex m;
  std::map<uintptr_t, Entry> entries;  // by first byte; never overlapping
  std::map<void*, Caller> callers;     // hydra_host_register, by the caller's start address
  uint64_t registrations = 0;
  uint64_t outside = 0;
};

Registry& R() {
  static Registry* r = new Registry;  // never destroyed (no HIP call from a static destructor)
  return *r;
}

// The registry entry with the lowest address that intersects [lo, hi), or end().
std::map<uintptr_t, Entry>::iterator first_intersecting(Registry& r, uintptr_t lo, uintptr_t hi) {
  auto it = r.entries.upper_bound(lo);
  if (it != r.entries.begin()) {
    auto prev = std::prev(it);
    if (prev->second.hi > lo) return prev;
  }
  if (it != r.entries.end() && it->first < hi) return it;
  return r.entries.end();
}

// A mapping of p's page the caller made (hipHostRegister / hipHostMalloc): its host range and
// device address.  Called with the registry lock held and only where no registry entry
// intersects, so it can never return one of hydra's own registrations.
bool caller_mapping(uintptr_t p, uintptr_t* start, size_t* size, char** dev_at_p,
                    bool* device = nullptr) {
  hipPointerAttribute_t at{};
  const void* q = reinterpret_cast<const void*>(p);
  if (hipPointerGetAttributes(&at, q) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (device) *device = at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeArray;
  if ((at.type != hipMemoryTypeHost && at.type != hipMemoryTypeManaged) || !at.devicePointer)
    return false;
  void* s = nullptr;
  size_t sz = 0;
  hipDeviceptr_t dq = reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(q));
  if (hipPointerGetAttribute(&s, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, dq) != hipSuccess ||
      hipPointerGetAttribute(&sz, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, dq) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t s0 = reinterpret_cast<uintptr_t>(s);
  if (p < s0 || p - s0 >= sz) return false;
  *start = s0;
  *size = sz;
  const uintptr_t hp = at.hostPointer ? reinterpret_cast<uintptr_t>(at.hostPointer) : p;
  *dev_at_p = static_cast<char*>(at.devicePointer) + (p - hp);
  return true;
}

// hipHostRegister of [lo, hi) for the reserved (pending) entry `lo`; the lock is NOT held.
hipError_t do_register(uintptr_t lo, uintptr_t hi, char** dev) {
  void* p = reinterpret_cast<void*>(lo);
  hipError_t e = hipHostRegister(p, hi - lo, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return e;
  }
  void* d = nullptr;
  e = hipHostGetDevicePointer(&d, p, 0);
  if (e != hipSuccess || !d) {
    (void)hipGetLastError();
    (void)hipHostUnregister(p);
    return e != hipSuccess ? e : hipErrorInvalidValue;
  }
  *dev = static_cast<char*>(d);
  return hipSuccess;
}

// Finish a pending registration (lock held): keep the entry or drop it.
void settle(Registry& r, uintptr_t lo, hipError_t e, char* dev, LedgerKind lk) {
  auto it = r.entries.find(lo);
  if (it == r.entries.end()) return;
  if (e != hipSuccess) {
    r.entries.erase(it);
    return;
  }
  Entry& x = it->second;
  x.pending = false;
  x.dev = dev;
  r.registrations++;
  if (lo < x.owner_lo || x.hi > x.owner_hi) r.outside++;
  ledger_add(lk, reinterpret_cast<void*>(lo), x.hi - lo);
}

// Unregister and erase entry `it` (lock held on entry via `g`, released around the HIP call).
void retire(Registry& r, std::unique_lock<std::mutex>& g, std::map<uintptr_t, Entry>::iterator it) {
  const uintptr_t lo = it->first;
  const LedgerKind lk = kLedgerHostRegister;
  it->second.dying = true;  // still intersects: nobody maps or registers these pages meanwhile
  g.unlock();
  (void)hipHostUnregister(reinterpret_cast<void*>(lo));
  (void)hipGetLastError();
  ledger_release(lk, reinterpret_cast<void*>(lo));
  g.lock();
  r.entries.erase(lo);
}

}  // namespace

void host_windows_acquire(const void* ptr, size_t bytes, HostWindows* out) {
  *out = HostWindows{};
  if (!ptr || !bytes) return;
  Registry& r = R();
  const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
  const uintptr_t end = p + bytes;
  std::unique_lock<std::mutex> g(r.m);
  auto add = [&](uintptr_t lo, uintptr_t hi, char* dev, int kind, uintptr_t key,
                 size_t entry_bytes) {
    HostWindow& w = out->w[out->count++];
    w.lo = reinterpret_cast<const char*>(lo);
    w.hi = reinterpret_cast<const char*>(hi);
    w.dev = dev;
    w.kind = kind;
    w.key = key;
    w.entry_bytes = entry_bytes;
  };
  // hydra's own mappings inside the operand (one being (un)registered meanwhile is not used:
  // its bytes are staged)
  bool any = false;
  for (auto it = first_intersecting(r, p, end); it != r.entries.end() && it->first < end; ++it) {
    Entry& x = it->second;
    any = true;
    if (x.pending || x.dying || out->count == kMaxWindows) continue;
    const uintptr_t lo = std::max(p, it->first), hi = std::min(end, x.hi);
    x.users++;
    add(lo, hi, x.dev + (lo - it->first), x.kind, it->first, x.hi - it->first);
  }
  if (any) return;
  // none: a mapping the caller made (no reference: the caller keeps it for the call)
  uintptr_t s = 0;
  size_t sz = 0;
  char* d = nullptr;
  if (caller_mapping(p, &s, &sz, &d, &out->device))
    add(p, std::min(end, s + sz), d, kMapCaller, 0, sz);
}

void host_windows_release(HostWindows* ws) {
  if (!ws) return;
  Registry& r = R();
  std::unique_lock<std::mutex> g(r.m, std::defer_lock);
  for (int i = 0; i < ws->count; i++) {
    const uintptr_t key = ws->w[i].key;
    ws->w[i] = HostWindow{};
    if (!key) continue;
    if (!g.owns_lock()) g.lock();
    auto it = r.entries.find(key);
    if (it == r.entries.end()) continue;
    Entry& x = it->second;
    if (--x.users > 0) continue;
    if (x.kind == kMapRegister && x.owners == 0) retire(r, g, it);
  }
  ws->count = 0;
}

int host_register(void* ptr, size_t bytes, const char** what) {
  *what = "";
  if (!ptr || !bytes) {
    *what = "null/empty range";
    return HYDRA_ERR_INVALID;
  }
  Registry& r = R();
  std::unique_lock<std::mutex> g(r.m);
  auto ci = r.callers.find(ptr);
  if (ci != r.callers.end()) {
    if (bytes > ci->second.bytes) {
      *what = "already registered with a shorter range: unregister it first";
      return HYDRA_ERR_INVALID;
    }
    ci->second.count++;
    if (ci->second.key) {
      auto it = r.entries.find(ci->second.key);
      if (it != r.entries.end()) it->second.owners++;
    }
    return HYDRA_OK;
  }
  const uintptr_t p = reinterpret_cast<uintptr_t>(ptr);
  uintptr_t lo, hi;
  page_interior(p, bytes, &lo, &hi);
  Caller c{bytes, 1, 0};
  if (lo >= hi) {  // no whole page inside: nothing to register, the operand is staged
    r.callers.emplace(ptr, c);
    return HYDRA_OK;
  }
  auto it = first_intersecting(r, lo, hi);
  if (it != r.entries.end()) {
    // shares the pages of a live registration of another owner: reference it; anything else
    // (a pinned block -- mapped already --, a partial overlap, one in flight) registers nothing
    Entry& x = it->second;
    if (x.kind == kMapRegister && !x.pending && !x.dying && it->first <= lo && hi <= x.hi) {
      x.owners++;
      c.key = it->first;
    }
    r.callers.emplace(ptr, c);
    return HYDRA_OK;
  }
  uintptr_t s;
  size_t sz;
  char* d;
  if (caller_mapping(lo, &s, &sz, &d) || caller_mapping(hi - 1, &s, &sz, &d)) {
    r.callers.emplace(ptr, c);  // mapped by its owner: used as it is, never released here
    return HYDRA_OK;
  }
  Entry x{};
  x.hi = hi;
  x.kind = kMapRegister;
  x.owners = 1;
  x.pending = true;
  x.owner_lo = p;
  x.owner_hi = p + bytes;
  r.entries.emplace(lo, x);
  c.key = lo;
  r.callers.emplace(ptr, c);
  g.unlock();
  char* dev = nullptr;
  const hipError_t e = do_register(lo, hi, &dev);
  g.lock();
  settle(r, lo, e, dev, kLedgerHostRegister);
  if (e == hipSuccess) {
    auto it2 = r.entries.find(lo);  // every owner unregistered while the registration ran
    if (it2 != r.entries.end() && it2->second.owners <= 0 && it2->second.users <= 0)
      retire(r, g, it2);
    return HYDRA_OK;
  }
  if (e == hipErrorHostMemoryAlreadyRegistered) {  // registered by its owner: used as it is
    auto c2 = r.callers.find(ptr);
    if (c2 != r.callers.end()) c2->second.key = 0;
    return HYDRA_OK;
  }
  auto c2 = r.callers.find(ptr);
  if (c2 != r.callers.end() && --c2->second.count <= 0) r.callers.erase(c2);
  else if (c2 != r.callers.end()) c2->second.key = 0;
  *what = hipGetErrorString(e);
  return HYDRA_ERR_HIP;
}

int host_unregister(void* ptr, const char** what) {
  *what = "";
  Registry& r = R();
  std::unique_lock<std::mutex> g(r.m);
  auto ci = r.callers.find(ptr);
  if (ci == r.callers.end()) return HYDRA_OK;  // not registered here (or already released)
  const uintptr_t key = ci->second.key;
  if (--ci->second.count <= 0) r.callers.erase(ci);
  if (!key) return HYDRA_OK;
  auto it = r.entries.find(key);
  if (it == r.entries.end()) return HYDRA_OK;
  Entry& x = it->second;
  if (--x.owners > 0 || x.users > 0 || x.pending) return HYDRA_OK;  // the last user retires it
  retire(r, g, it);
  return HYDRA_OK;
}

void host_map_add_block(void* p, size_t bytes) {
  Registry& r = R();
  std::lock_guard<std::mutex> g(r.m);
  Entry x{};
  x.hi = reinterpret_cast<uintptr_t>(p) + bytes;
  x.dev = static_cast<char*>(p);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess && d) x.dev = static_cast<char*>(d);
  (void)hipGetLastError();
  x.kind = kMapPinnedBlock;
  x.owners = 1;
  x.owner_lo = reinterpret_cast<uintptr_t>(p);
  x.owner_hi = x.hi;
  r.entries[reinterpret_cast<uintptr_t>(p)] = x;
}

void host_map_remove_block(void* p) {
  Registry& r = R();
  std::lock_guard<std::mutex> g(r.m);
  r.entries.erase(reinterpret_cast<uintptr_t>(p));
}

size_t host_map_snapshot(HostMapEntry* out, size_t cap) {
  Registry& r = R();
  std::lock_guard<std::mutex> g(r.m);
  size_t k = 0;
  for (auto& kv : r.entries) {
    if (out && k < cap)
      out[k] = HostMapEntry{kv.first, kv.second.hi, kv.second.kind, kv.second.owners,
                            kv.second.users, kv.second.owner_lo, kv.second.owner_hi};
    k++;
  }
  return k;
}

void host_map_counters(uint64_t* registrations, uint64_t* outside) {
  Registry& r = R();
  std::lock_guard<std::mutex> g(r.m);
  if (registrations) *registrations = r.registrations;
  if (outside) *outside = r.outside;
}

}  // namespace hydra
