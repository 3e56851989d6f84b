// resident_host.cpp -- the host side of the resident reducer (resident.h): one server per
// device per process (control block, device record, its own hardware queue), slots leased by
// host contexts, launches on demand.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/hydra_hip.h"
#include "errors.h"
#include "options.h"
#include "resident.h"
#include "resource_cache.h"

namespace hydra {

struct ResidentServer {
  int device = 0;
  ResCtl* h = nullptr;      // host address of the control block
  ResCtl* h_dev = nullptr;  // its device address
  ResDev* d = nullptr;
  hipStream_t s = nullptr;
  std::mutex mu;  // launches and slot leases
  std::condition_variable resumed;  // paused dropped to 0
  uint64_t gen = 0;
  uint32_t leased = 0;  // bit i: slot i has a holder
  int paused = 0;       // resident_pause holders: no launch meanwhile (under mu)
  std::atomic<bool> poisoned{false};  // an instance could not be confirmed gone: never used again
  std::atomic<uint64_t> launches{0};
};

struct ResidentLease {
  ResidentServer* srv;
  int slot;
  uint64_t seq;    // the slot's last sequence number rung
  uint64_t calls;  // calls submitted through this lease
  uint64_t seen;   // the highest completion word a wait saw (a lower one later: a regression)
};

namespace {
static_assert(kResidentSlots <= 32, "leased is a 32-bit mask");

constexpr int kMaxDevices = 64;
std::mutex g_mu;
std::atomic<ResidentServer*> g_srv[kMaxDevices] = {};  // set once each (under g_mu)
std::atomic<bool> g_exiting{false};

// Settings of an instance, read at each launch (hydra_set_option, options.h; s_memrealtime
// ticks run at 100 MHz): leave after HYDRA_OPT_RESIDENT_IDLE_US without a call (2 ms); bound
// every wait inside the grid by HYDRA_OPT_RESIDENT_GRACE_US (10 s).
uint64_t idle_ticks() { return (uint64_t)opt(HYDRA_OPT_RESIDENT_IDLE_US) * 100; }
uint64_t grace_ticks() { return (uint64_t)opt(HYDRA_OPT_RESIDENT_GRACE_US) * 100; }

ResidentShape shape() {  // HYDRA_OPT_RESIDENT_BLOCKS / _BATCH / _SOLO / _TILES
  ResidentShape r;
  r.blocks = (int)std::min<int64_t>(opt(HYDRA_OPT_RESIDENT_BLOCKS), kResidentMaxBlocks);
  const int64_t u = opt(HYDRA_OPT_RESIDENT_BATCH);
  r.batch = u >= 4 ? 4 : u >= 2 ? 2 : 1;
  r.solo = (uint32_t)opt(HYDRA_OPT_RESIDENT_SOLO);
  r.tiles_per_block = (uint32_t)opt(HYDRA_OPT_RESIDENT_TILES);
  return r;
}

template <typename T>
volatile T& vol(T& x) {
  return reinterpret_cast<volatile T&>(x);
}

// At process exit every running instance is told to leave, so each grid has drained before
// the runtime tears down (registered after the runtime initialised: runs before its teardown).
void quit_all() {
  g_exiting.store(true);
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& x : g_srv)
    if (ResidentServer* v = x.load()) vol(v->h->quit) = 1u;
  for (auto& x : g_srv) {  // bounded: an instance leaves within microseconds
    ResidentServer* v = x.load();
    if (!v) continue;
    const auto t0 = std::chrono::steady_clock::now();
    while (vol(v->h->alive) != 0u &&
           std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(200))
      std::this_thread::yield();
  }
}

// The instance's stream must not hold anything else up behind the persistent grid:
//  * non-blocking, or every kernel on the legacy default stream (torch's default stream) waits
//    for the grid to leave;
//  * on a hardware queue no other stream uses: the runtime shares its GPU_MAX_HW_QUEUES queues
//    per priority level among a process's streams, so a plain stream can land behind the grid.
//    The greatest-priority level has a pool of its own, which ordinary code (torch's default
//    and pool streams, RCCL) does not use.
// HYDRA_OPT_RESIDENT_QUEUE 1 (a plain non-blocking stream) and 2 (a CU-masked stream: a queue
// of its own, but blocking) are A/B settings only (scripts/probe_queue_block.py).
hipError_t make_stream(int device, hipStream_t* out) {
  const int64_t q = opt(HYDRA_OPT_RESIDENT_QUEUE);
  if (q == 1) return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
  if (q == 2) {
    hipDeviceProp_t p;
    hipError_t e = hipGetDeviceProperties(&p, device);
    if (e != hipSuccess) return e;
    const int cus = std::max(1, p.multiProcessorCount);
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int i = 0; i < cus; i++) mask[i / 32] |= 1u << (i % 32);
    return hipExtStreamCreateWithCUMask(out, (uint32_t)mask.size(), mask.data());
  }
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(out, hipStreamNonBlocking, greatest);
}

int server(int device, ResidentServer** out) {
  *out = nullptr;
  if (device < 0 || device >= kMaxDevices) return fail(HYDRA_ERR_INVALID, "device out of range");
  std::lock_guard<std::mutex> g(g_mu);
  if (ResidentServer* have = g_srv[device].load()) {
    *out = have;
    return HYDRA_OK;
  }
  int prev = -1;
  (void)hipGetDevice(&prev);
  auto* v = new ResidentServer();
  v->device = device;
  void* p = nullptr;
  void* q = nullptr;
  void* hd = nullptr;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = cached_malloc_host(sizeof(ResCtl), &p);
  if (e == hipSuccess) {
    std::memset(p, 0, sizeof(ResCtl));
    e = hipHostGetDevicePointer(&hd, p, 0);
  }
  if (e == hipSuccess) e = cached_malloc(device, sizeof(ResDev), &q);
  if (e == hipSuccess) e = hipMemset(q, 0, sizeof(ResDev));
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = make_stream(device, &v->s);
  if (prev >= 0) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    if (p) (void)cached_free_host(p);
    if (q) (void)cached_free(q);
    delete v;
    return hip_fail(e, "resident reducer setup");
  }
  v->h = static_cast<ResCtl*>(p);
  v->h_dev = static_cast<ResCtl*>(hd);
  v->d = static_cast<ResDev*>(q);
  static bool registered = false;
  if (!registered) {
    std::atexit(quit_all);
    registered = true;
  }
  g_srv[device] = v;  // lives for the process
  *out = v;
  return HYDRA_OK;
}

// Tell the running instance (if any) to leave and wait, bounded, until it has: true when no
// instance of this server is running any more.
bool stop_instance(ResidentServer* v, std::chrono::milliseconds bound) {
  vol(v->h->quit) = 1u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const auto t0 = std::chrono::steady_clock::now();
  while (vol(v->h->alive) != 0u) {
    if (std::chrono::steady_clock::now() - t0 > bound) return false;
    std::this_thread::yield();
  }
  return true;
}

// A new instance unless one is running (alive); `alive` is set before the launch, cleared by
// the kernel as it leaves.  While a drain holds the server paused (resident_pause), a caller
// whose call is pending waits here (bounded) for the drain to finish, then launches.
int ensure_running(ResidentServer* v) {
  if (vol(v->h->alive) != 0u) return HYDRA_OK;
  std::unique_lock<std::mutex> g(v->mu);
  if (vol(v->h->alive) != 0u) return HYDRA_OK;
  if (v->paused > 0 &&
      !v->resumed.wait_for(g, std::chrono::seconds(20), [v] { return v->paused == 0; }))
    return fail(HYDRA_ERR_TIMEOUT, "Timed out waiting 20000ms for a device drain to finish");
  if (g_exiting.load()) return fail(HYDRA_ERR_INVALID, "resident reducer: process is exiting");
  if (v->poisoned.load()) return fail(HYDRA_ERR_HIP, "resident reducer: disabled after a fault");
  vol(v->h->quit) = 0u;
  vol(v->h->alive) = 1u;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != v->device) (void)hipSetDevice(v->device);
  // Every instance starts from a zeroed device record, ordered after the last instance on the
  // same stream: no job word, `finished` word or arrival count an earlier instance left behind
  // can reach this one's workers, whatever its generation tag (the job word keeps 16 bits of the
  // generation, which wraps after 65536 launches).  After an expired wait
  // this also discards the partial arrival count that instance left.
  hipError_t e = hipMemsetAsync(v->d, 0, sizeof(ResDev), v->s);
  vol(v->h->err) = 0u;
  // (test switch HYDRA_TEST_RESIDENT_GEN_STRIDE: wrap the tag on every launch)
  const int64_t stride = test_value(HYDRA_TEST_RESIDENT_GEN_STRIDE);
  v->gen += stride > 0 ? (uint64_t)stride : 1u;
  if (e == hipSuccess)
    e = launch_resident(v->h_dev, v->d, v->gen, idle_ticks(), grace_ticks(), shape(), v->s);
  if (prev >= 0 && prev != v->device) (void)hipSetDevice(prev);
  if (e != hipSuccess) {
    vol(v->h->alive) = 0u;
    return hip_fail(e, "resident reducer launch");
  }
  v->launches.fetch_add(1);
  return HYDRA_OK;
}

// Lock-free (g_mu may be held by a caller that releases a block: server()'s error path).
ResidentServer* find_server(int device) {
  if (device < 0 || device >= kMaxDevices) return nullptr;
  return g_srv[device].load();
}
}  // namespace

int resident_lease(int device, ResidentLease** out) {
  *out = nullptr;
  ResidentServer* v = nullptr;
  if (int rc = server(device, &v)) return rc;
  std::lock_guard<std::mutex> g(v->mu);
  for (int k = 0; k < kResidentSlots; k++) {
    if (v->leased & (1u << k)) continue;
    v->leased |= 1u << k;
    // numbering continues from the slot's last doorbell (a slot is reused by later contexts)
    *out = new ResidentLease{v, k, vol(v->h->slot[k].doorbell), 0, vol(v->h->slot[k].done)};
    return HYDRA_OK;
  }
  return HYDRA_OK;  // every slot leased: this context launches
}

void resident_release(ResidentLease* l) {
  if (!l) return;
  {
    std::lock_guard<std::mutex> g(l->srv->mu);
    l->srv->leased &= ~(1u << l->slot);
  }
  delete l;
}

int resident_submit(ResidentLease* l, int op, int dtype, size_t es, const BatchSegDesc* segs,
                    size_t count) {
  if (count == 0 || count > (size_t)kResidentSegs)
    return fail(HYDRA_ERR_INVALID, "resident reducer: 1..16 segments per call");
  ResidentServer* v = l->srv;
  ResSlot& S = v->h->slot[l->slot];
  ResDesc& D = S.desc;
  const size_t N = 16 / es;
  uint32_t tiles = 0;
  int k = 0;
  for (size_t i = 0; i < count; i++) {
    const BatchSegDesc& g = segs[i];
    if (g.n == 0) continue;
    const uintptr_t cp = reinterpret_cast<uintptr_t>(g.c);
    size_t head = ((16 - (cp & 15)) & 15) / es;
    if (head > g.n) head = g.n;
    const size_t nvec = (g.n - head) / N;
    ResSeg& r = D.s[k++];
    r.c = static_cast<char*>(g.c) + head * es;
    r.a = static_cast<const char*>(g.a) + head * es;
    r.b = static_cast<const char*>(g.b) + head * es;
    r.nvec = nvec;
    r.head = (int32_t)head;
    r.tail = (int32_t)(g.n - head - nvec * N);
    r.tile0 = tiles;
    r.c_old = (dtype == HYDRA_FLOAT16 && g.c != g.a) ? 1u : 0u;
    tiles += (uint32_t)std::max<size_t>(1, (nvec + kBlock - 1) / kBlock);
  }
  if (k == 0) return fail(HYDRA_ERR_INVALID, "resident reducer: empty call");
  D.op = op;
  D.dtype = dtype;
  D.count = k;
  D.tiles = tiles;
  std::atomic_thread_fence(std::memory_order_release);  // the descriptor before the doorbell
  vol(S.doorbell) = ++l->seq;
  l->calls++;
  return ensure_running(v);
}

// A failed wait (an expired wait inside the grid, or this bound) must not return while the
// grid may still touch the caller's buffers: the instance is told to leave and waited for; if it
// cannot be confirmed gone, the server is poisoned (every later call launches instead) and
// *poisoned tells the caller to keep its windows mapped.
int resident_wait(ResidentLease* l, bool* poisoned) {
  ResidentServer* v = l->srv;
  if (poisoned) *poisoned = false;
  volatile uint64_t& done = vol(v->h->slot[l->slot].done);
  const uint64_t seq = l->seq;
  const auto t0 = std::chrono::steady_clock::now();
  // the call is abandoned: with relaunches held, stop the instance, then retire the doorbell
  // (done = seq) so that no later instance serves this descriptor after the caller returned
  auto give_up = [&](int code, const char* msg) {
    {
      std::lock_guard<std::mutex> g(v->mu);
      v->paused++;
    }
    if (stop_instance(v, std::chrono::seconds(2))) {
      done = seq;
      l->seen = std::max(l->seen, seq);
    } else {
      v->poisoned.store(true);
      if (poisoned) *poisoned = true;
    }
    {
      std::lock_guard<std::mutex> g(v->mu);
      v->paused--;
    }
    v->resumed.notify_all();
    return fail(code, msg);
  };
  for (uint32_t spins = 0;; spins++) {
    const uint64_t now_done = done;
    if (now_done < l->seen) test_count(HYDRA_TEST_RESIDENT_REGRESSIONS);  // (never, by design)
    l->seen = std::max(l->seen, now_done);
    if (now_done >= seq) break;
    if (vol(v->h->alive) == 0u && done < seq) {  // it left without serving us: a new instance
      if (vol(v->h->err))  // (it left on an expired wait: report that, do not relaunch)
        return give_up(HYDRA_ERR_HIP, "resident reducer: a wait inside the grid expired");
      if (int rc = ensure_running(v)) return rc;
      continue;
    }
    if ((spins & 1023) == 0) {
      if (vol(v->h->err))
        return give_up(HYDRA_ERR_HIP, "resident reducer: a wait inside the grid expired");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(20))
        return give_up(HYDRA_ERR_TIMEOUT, "Timed out waiting 20000ms for the resident reducer");
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);  // the results after `done`
  return HYDRA_OK;
}

bool resident_usable(const ResidentLease* l) { return l && !l->srv->poisoned.load(); }

void resident_pause(int device) {
  for (int d = 0; d < kMaxDevices; d++) {
    if (device >= 0 && d != device) continue;
    ResidentServer* v = find_server(d);
    if (!v) continue;
    {
      std::lock_guard<std::mutex> g(v->mu);
      v->paused++;
    }
    // bounded: an instance finishes the call it is serving, then leaves (quit is checked before
    // the doorbells); past the bound the caller's drain simply waits for it as before
    (void)stop_instance(v, std::chrono::milliseconds(500));
  }
}

void resident_resume(int device) {
  for (int d = 0; d < kMaxDevices; d++) {
    if (device >= 0 && d != device) continue;
    ResidentServer* v = find_server(d);
    if (!v) continue;
    {
      std::lock_guard<std::mutex> g(v->mu);
      if (v->paused > 0) v->paused--;
    }
    v->resumed.notify_all();
  }
}

hipError_t drain_device(int device) {
  ResidentPause p(device);
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  hipError_t e = device >= 0 && device != prev ? hipSetDevice(device) : hipSuccess;
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (prev >= 0 && device >= 0 && device != prev) (void)hipSetDevice(prev);
  return e;
}

uint64_t resident_calls(const ResidentLease* l) { return l ? l->calls : 0; }

uint64_t resident_launches(int device) {
  if (device < 0 || device >= kMaxDevices) return 0;
  ResidentServer* v = g_srv[device].load();
  return v ? v->launches.load() : 0;
}

}  // namespace hydra
