// host_map.h -- which caller host memory a kernel may touch in place (zero-copy), and for how long.
//
// hydra_reduce_host lets the chunk-sum kernel read and write host operands over PCIe when they
// are mapped for the GPU.  A mapping the kernel uses must stay mapped until the kernel is done.
//
// Round 3 found what the late device faults of rounds 1-2 were (DESIGN.md §10,
// profiles/r03_fault_report.txt): host pages that hydra had hipHostRegister'ed and
// hipHostUnregister'ed -- per-call pins of pageable operands, or test buffers registered with
// hydra_host_register -- were later freed, reused by the allocator, and copied by the HIP
// runtime's own pageable copy path (above 1 MiB it locks the caller's pages); that copy faulted
// on the GPU, seconds after hydra had released the range.  So:
//
//   * hydra never registers host memory on its own: a pageable operand is read and written by
//     the CPU only (memcpy through the context's pinned staging), never pinned for a call and
//     never handed to a HIP copy;
//   * hydra_host_register (an explicit, long-lived registration the caller asks for) covers only
//     the WHOLE PAGES strictly inside the caller's range, never a page shared with other
//     objects; the ragged head / tail bytes are staged;
//   * hydra's registrations never overlap each other: one registry (an interval map) holds them,
//     plus the pinned blocks of the block cache; a call that finds its operand inside a registry
//     entry takes a reference on it, so the entry outlives the call's kernel whatever its owner
//     does meanwhile (the case round 2's advisor raised: one thread's operand inside another's
//     mapping);
//   * a mapping hydra did not make (the caller's own hipHostRegister / hipHostMalloc, e.g. torch
//     pinned tensors) is looked up with the registry lock held, so no hydra registration can
//     appear or vanish between the lookup and its use; the caller keeps it alive for the call,
//     as for any asynchronous copy from it.
//
// Windows are byte ranges [lo, hi) inside the operand; the rest of the operand is staged by the
// CPU.
#pragma once

#include <cstddef>
#include <cstdint>

namespace hydra {

size_t page_size();

// Whole pages strictly inside [p, p + bytes): [*lo, *hi) (empty: *lo == *hi).
void page_interior(uintptr_t p, size_t bytes, uintptr_t* lo, uintptr_t* hi);

enum HostMapKind : int {
  kMapNone = 0,
  kMapRegister = 1,     // hydra_host_register (whole interior pages)
  kMapPin = 2,          // (retired in round 3: pageable operands are no longer pinned per call)
  kMapPinnedBlock = 3,  // hipHostMalloc block of the cache (hydra_malloc_host)
  kMapCaller = 4,       // mapped by the caller, not by hydra (no reference taken)
};

struct HostWindow {
  const char* lo = nullptr;  // [lo, hi) of the operand is mapped; dev is lo's device address
  const char* hi = nullptr;
  char* dev = nullptr;
  int kind = kMapNone;
  uintptr_t key = 0;  // registry entry referenced by this window (0: none)
  size_t entry_bytes = 0;  // the whole mapping's size (registry entry / caller mapping)
  bool empty() const { return lo >= hi; }
};

// The mapped windows of the operand [p, p + bytes), in address order, each referenced until
// host_windows_release: every hydra registry entry intersecting the operand (at most
// kMaxWindows) or, if there is none, the caller's own mapping of p's page.  The bytes outside
// the windows are the caller's pageable memory: hydra only ever reads / writes them with CPU
// loads and stores.  `device` is set (and no window returned) when the operand is device memory.
constexpr int kMaxWindows = 4;
struct HostWindows {
  HostWindow w[kMaxWindows];
  int count = 0;
  bool device = false;
};
void host_windows_acquire(const void* p, size_t bytes, HostWindows* out);
void host_windows_release(HostWindows* ws);

// hydra_host_register / hydra_host_unregister (C-ABI semantics in include/hydra_hip.h).
// Return a hydra status; *what names the failing step.
int host_register(void* p, size_t bytes, const char** what);
int host_unregister(void* p, const char** what);

// The block cache's pinned blocks (whole allocations; never registered, never unregistered here).
void host_map_add_block(void* p, size_t bytes);
void host_map_remove_block(void* p);

// Test hook: the registry's live entries.
struct HostMapEntry {
  uintptr_t lo, hi;
  int kind;
  int owners;  // hydra_host_register owners of the entry
  int users;   // calls holding a window on it
  uintptr_t owner_lo, owner_hi;  // the caller range that created it (kMapRegister / kMapPin)
};
size_t host_map_snapshot(HostMapEntry* out, size_t cap);
// Registrations (hipHostRegister calls) hydra has made so far, and how many of them covered a
// byte outside the caller range they were made for (must stay 0).
void host_map_counters(uint64_t* registrations, uint64_t* outside);

}  // namespace hydra
