// hydra_capi.cpp -- the extern "C" boundary of libhydra_hip.so (declared in include/hydra_hip.h).
//
// Argument checking, error reporting (thread-local message + status code), the host-resident
// staging context, and the ring geometry.  Kernels live in reduce_kernels.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hydra_hip.h"
#include "copy_pool.h"
#include "errors.h"
#include "fault_report.h"
#include "host_map.h"
#include "options.h"
#include "resource_cache.h"
#include "reduce_kernels.h"
#include "resident.h"
#include "trace.h"

namespace {
thread_local std::string g_err;
#ifdef HYDRA_MEASURE
std::atomic<int> g_variant{0};
#endif
}  // namespace

namespace hydra {
int ok() {
  g_err.clear();
  return HYDRA_OK;
}
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(HYDRA_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
#ifdef HYDRA_MEASURE
int current_variant() { return g_variant.load(std::memory_order_relaxed); }
#endif

namespace {
constexpr int kTestKeys = 4;  // hydra_test_key_t values 1..3
std::atomic<int64_t> g_test[kTestKeys] = {};
}  // namespace
int64_t test_value(int key) {
  return key > 0 && key < kTestKeys ? g_test[key].load(std::memory_order_relaxed) : 0;
}
void test_count(int key) {
  if (key > 0 && key < kTestKeys) g_test[key].fetch_add(1, std::memory_order_relaxed);
}
}  // namespace hydra

using hydra::fail;
using hydra::hip_fail;
using hydra::ok;

namespace {

bool overlaps(const void* x, const void* y, size_t bytes) {
  const char* a = static_cast<const char*>(x);
  const char* b = static_cast<const char*>(y);
  return a < b + bytes && b < a + bytes;
}

// Shared argument contract of hydra_reduce / hydra_reduce_host.
int check_args(int op, int dtype, const void* c, const void* a, const void* b, size_t n) {
  if (op < HYDRA_SUM || op > HYDRA_MIN) return fail(HYDRA_ERR_INVALID, "invalid op");
  const size_t es = hydra::dtype_size(dtype);
  if (!es) return fail(HYDRA_ERR_INVALID, "invalid dtype " + std::to_string(dtype));
  if (n == 0) return HYDRA_OK;
  if (!c || !a || !b) return fail(HYDRA_ERR_INVALID, "null pointer");
  const uintptr_t m = es - 1;
  if ((reinterpret_cast<uintptr_t>(c) | reinterpret_cast<uintptr_t>(a) |
       reinterpret_cast<uintptr_t>(b)) & m)
    return fail(HYDRA_ERR_INVALID, "pointer not aligned to the element size");
  const size_t bytes = n * es;
  if (c != a && overlaps(c, a, bytes))
    return fail(HYDRA_ERR_INVALID, "c partially overlaps a (only c == a is allowed)");
  if (c != b && overlaps(c, b, bytes))
    return fail(HYDRA_ERR_INVALID, "c partially overlaps b (only c == b is allowed)");
  return HYDRA_OK;
}

}  // namespace

// ---- host staging context ----------------------------------------------------------------
// A stream, two completion events and two pinned staging buffers (hipHostMalloc blocks of the
// cache).  Operand bytes the kernel cannot reach in place (hydra_reduce_host) are copied into
// a staging buffer by the CPU and read / written by the kernel there over PCIe; the two
// buffers alternate, so the CPU fills round r + 1 while the GPU reduces round r.
struct hydra_ctx {
  int device = 0;
  hydra::CtxOpts opts;  // the [ctx] options (hydra_ctx_set_option), from the process-wide values
  hipStream_t stream = nullptr;
  hipEvent_t done[2] = {nullptr, nullptr};
  char* stage[2] = {nullptr, nullptr};      // host address
  char* stage_dev[2] = {nullptr, nullptr};  // its device address
  // a slot of the device's resident reducer (resident.h); null: off, or every slot leased
  hydra::ResidentLease* lease = nullptr;
};

namespace {
// hydra_host_trace: per-call records of hydra_reduce_host (measurement only)
std::atomic<bool> g_trace_on{false};
std::mutex g_trace_mu;
std::vector<hydra_host_call_t>* g_trace = new std::vector<hydra_host_call_t>;  // never freed
constexpr size_t kTraceCap = size_t(1) << 20;

using Clock = std::chrono::steady_clock;
double us_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
}

constexpr size_t kSlotBytes = 4u << 20;  // per operand and staging buffer (3 slots: a, b, c)
// (the smallest staging round per operand, HYDRA_OPT_ROUND_MIN, defaults to 512 KiB:
// scripts/probe_stage_split.cc's A/B)

// Staged RESULT where c is mapped: the kernel writes the pinned staging and the CPU copies it
// into c, which leaves c's lines in the CPU's cache for the caller's next read of them (a
// zero-copy write from the GPU invalidates them).  Measured inside the reference's ring
// (profiles/r04d_dropin_sweep.json): it pays while the registered bucket fits the CPU's cache
// (4 MiB: 0.669 vs 0.714 ms per allreduce) and costs once it does not (16 MiB and up: the
// zero-copy write wins, 2.94 vs 3.11 ms).  So a result goes through the staging when c lies in a
// hydra_host_register'ed range of at most HYDRA_OPT_STAGE_RESULT_REG_MAX bytes (default 8 MiB),
// or when the call itself is at most HYDRA_OPT_STAGE_RESULT_MAX bytes per operand (default 0,
// A/B).  Not for float16 (its store quirk reads c's old bits).

void ctx_release(hydra_ctx* x) {
  if (x->stream) (void)hydra::release_stream(x->stream);
  for (int i = 0; i < 2; i++) {
    if (x->done[i]) (void)hydra::release_event(x->done[i]);
    if (x->stage[i]) (void)hydra::cached_free_host(x->stage[i]);
  }
  hydra::resident_release(x->lease);
  x->lease = nullptr;
}

}  // namespace

extern "C" {

int hydra_abi_version(void) { return HYDRA_ABI_VERSION; }

const char* hydra_last_error(void) { return g_err.c_str(); }

int hydra_device_count(int* count) {
  if (!count) return fail(HYDRA_ERR_INVALID, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = c;
  return ok();
}

int hydra_device_arch(int device, char* buf, size_t len) {
  hipDeviceProp_t p;
  HIP_TRY(hipGetDeviceProperties(&p, device));
  if (buf && len) {
    std::strncpy(buf, p.gcnArchName, len - 1);
    buf[len - 1] = 0;
  }
  return ok();
}

int hydra_device_check(int device) {
  hydra::DeviceScope ds(device);  // the caller's current device is left as it was
  HIP_TRY(ds.err);
  // surfaces an asynchronous fault of any enqueued work (the resident reducer is stopped first,
  // so the drain does not wait on other threads' host calls)
  HIP_TRY(hydra::drain_device(device));
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hydra::hip_fail(e, "sticky device error");
  return ok();
}

#ifdef HYDRA_MEASURE  // libhydra_measure.so only (include/hydra_measure.h)
int hydra_set_variant(int variant) { return g_variant.exchange(variant); }
#endif

int hydra_set_option(int key, long long value) {
  if (key <= 0 || key >= hydra::kOptCount)
    return fail(HYDRA_ERR_INVALID, "hydra_set_option: unknown key " + std::to_string(key));
  const hydra::OptSpec& sp = hydra::opt_spec(key);
  if (value < sp.lo || value > sp.hi)
    return fail(HYDRA_ERR_INVALID, "hydra_set_option: value " + std::to_string(value) +
                                       " of key " + std::to_string(key) + " outside [" +
                                       std::to_string(sp.lo) + ", " + std::to_string(sp.hi) + "]");
  hydra::opt_set(key, value);
  return ok();
}

int hydra_get_option(int key, long long* value) {
  if (!value) return fail(HYDRA_ERR_INVALID, "null value");
  if (key <= 0 || key >= hydra::kOptCount)
    return fail(HYDRA_ERR_INVALID, "hydra_get_option: unknown key " + std::to_string(key));
  *value = hydra::opt(key);
  return ok();
}

int hydra_test_set(int key, int64_t value, int64_t* prev) {
  if (key != HYDRA_TEST_LOCAL_STAGE && key != HYDRA_TEST_RESIDENT_GEN_STRIDE)
    return fail(HYDRA_ERR_INVALID, "hydra_test_set: unknown or read-only key " + std::to_string(key));
  const int64_t old = hydra::g_test[key].exchange(value);
  if (prev) *prev = old;
  return ok();
}

int hydra_test_get(int key, int64_t* value) {
  if (!value) return fail(HYDRA_ERR_INVALID, "null value");
  if (key < HYDRA_TEST_LOCAL_STAGE || key > HYDRA_TEST_RESIDENT_REGRESSIONS)
    return fail(HYDRA_ERR_INVALID, "hydra_test_get: unknown key " + std::to_string(key));
  *value = hydra::test_value(key);
  return ok();
}

int hydra_reduce(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                 hydra_stream_t stream) {
  int rc = check_args(op, dtype, c, a, b, n);
  if (rc) return rc;
  if (n == 0) return ok();
  hipError_t e = hydra::launch_reduce(hydra::current_variant(), op, dtype, c, a,
                                      b, n, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "reduce kernel launch");
  return ok();
}

int hydra_chunk_sum(int dtype, void* c, const void* a, const void* b, size_t n,
                    hydra_stream_t stream) {
  return hydra_reduce(HYDRA_SUM, dtype, c, a, b, n, stream);
}

int hydra_reduce_batch(int op, int dtype, const hydra_segment_t* segs, size_t count,
                       hydra_stream_t stream) {
  if (count && !segs) return fail(HYDRA_ERR_INVALID, "null segment list");
  static_assert(sizeof(hydra_segment_t) == sizeof(hydra::BatchSegDesc), "layout");
  for (size_t i = 0; i < count; i++) {  // every segment obeys hydra_reduce's contract
    int rc = check_args(op, dtype, segs[i].c, segs[i].a, segs[i].b, segs[i].n);
    if (rc) return fail(rc, "segment " + std::to_string(i) + ": " + hydra_last_error());
  }
  if (op < HYDRA_SUM || op > HYDRA_MIN || !hydra::dtype_size(dtype))
    return fail(HYDRA_ERR_INVALID, "invalid op/dtype");
  hipError_t e = hydra::launch_reduce_batch(op, dtype,
                                            reinterpret_cast<const hydra::BatchSegDesc*>(segs),
                                            count, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "batched reduce kernel launch");
  return ok();
}

int hydra_fold(int op, int dtype, int flags, void* dst, const void* const* srcs, int nsrc,
               size_t n, hydra_stream_t stream) {
  if (op < HYDRA_SUM || op > HYDRA_MIN) return fail(HYDRA_ERR_INVALID, "invalid op");
  const size_t es = hydra::dtype_size(dtype);
  if (!es) return fail(HYDRA_ERR_INVALID, "invalid dtype");
  if (nsrc < 1 || nsrc > hydra::kMaxRanks || !srcs || !dst)
    return fail(HYDRA_ERR_INVALID, "need 1..16 sources and a destination");
  const bool acc32 = (flags & HYDRA_ACC_F32) != 0;
  if (acc32 && dtype != HYDRA_BFLOAT16)
    return fail(HYDRA_ERR_UNSUPPORTED, "HYDRA_ACC_F32 needs bf16 data");
  if (n == 0) return ok();
  for (int j = 0; j < nsrc; j++) {
    if (!srcs[j] || reinterpret_cast<uintptr_t>(srcs[j]) % es)
      return fail(HYDRA_ERR_INVALID, "source null or not element-aligned");
    if (srcs[j] != dst && overlaps(dst, srcs[j], n * es))
      return fail(HYDRA_ERR_INVALID, "dst partially overlaps a source");
  }
  if (reinterpret_cast<uintptr_t>(dst) % es) return fail(HYDRA_ERR_INVALID, "dst not aligned");
  hipError_t e = hydra::launch_fold(op, dtype, acc32, dst, srcs, nsrc, n,
                                    static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "fold kernel launch");
  return ok();
}

int hydra_acc_bf16_f32(float* acc, const void* b_bf16, size_t n, hydra_stream_t stream) {
  if (n == 0) return ok();
  if (!acc || !b_bf16) return fail(HYDRA_ERR_INVALID, "null pointer");
  if ((reinterpret_cast<uintptr_t>(acc) & 15) || (reinterpret_cast<uintptr_t>(b_bf16) & 1))
    return fail(HYDRA_ERR_INVALID, "acc must be 16-B aligned, b 2-B aligned");
  hipError_t e = hydra::launch_acc_bf16_f32(acc, b_bf16, n, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "acc_bf16 kernel launch");
  return ok();
}

int hydra_f32_to_bf16(void* out_bf16, const float* acc, size_t n, hydra_stream_t stream) {
  if (n == 0) return ok();
  if (!acc || !out_bf16) return fail(HYDRA_ERR_INVALID, "null pointer");
  hipError_t e = hydra::launch_f32_to_bf16(out_bf16, acc, n, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "f32_to_bf16 kernel launch");
  return ok();
}

// ---- host-resident ------------------------------------------------------------------------
int hydra_ctx_create(int device, hydra_ctx_t* out) {
  if (!out) return fail(HYDRA_ERR_INVALID, "null out");
  *out = nullptr;
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (device < 0 || device >= count) return fail(HYDRA_ERR_NO_DEVICE, "no such device");
  hydra::DeviceScope ds(device);  // the caller's current device is left as it was
  auto* x = new hydra_ctx();
  x->device = device;
  x->opts.load();
  hipError_t e = ds.err;
  if (e == hipSuccess) e = hydra::cached_stream(device, &x->stream);
  for (int i = 0; i < 2 && e == hipSuccess; i++) {
    e = hydra::cached_event(device, &x->done[i]);
    void* p = nullptr;
    if (e == hipSuccess) e = hydra::cached_malloc_host(3 * kSlotBytes, &p);
    x->stage[i] = static_cast<char*>(p);
    void* d = nullptr;
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d, p, 0);
    x->stage_dev[i] = static_cast<char*>(d);
  }
  if (e != hipSuccess) {
    ctx_release(x);
    delete x;
    return hip_fail(e, "hydra_ctx_create");
  }
  if (x->opts[HYDRA_OPT_RESIDENT] == 0) {
    // no slot of the resident reducer: every round is one launch on the context's stream
  } else if (int rc = hydra::resident_lease(device, &x->lease)) {
    ctx_release(x);
    delete x;
    return rc;
  }
  *out = x;
  return ok();
}

int hydra_ctx_set_option(hydra_ctx_t ctx, int key, long long value) {
  if (!ctx) return fail(HYDRA_ERR_INVALID, "null context");
  if (key <= 0 || key >= hydra::kOptCount || !hydra::opt_spec(key).per_ctx)
    return fail(HYDRA_ERR_INVALID, "hydra_ctx_set_option: not a per-context key " + std::to_string(key));
  const hydra::OptSpec& sp = hydra::opt_spec(key);
  if (value < sp.lo || value > sp.hi)
    return fail(HYDRA_ERR_INVALID, "hydra_ctx_set_option: value out of range");
  if (key == HYDRA_OPT_RESIDENT) {
    if (value == 0 && ctx->lease) {  // its calls were synchronous: the slot holds nothing
      hydra::resident_release(ctx->lease);
      ctx->lease = nullptr;
    } else if (value != 0 && !ctx->lease) {
      if (int rc = hydra::resident_lease(ctx->device, &ctx->lease)) return rc;
    }
  }
  ctx->opts.v[key] = value;
  return ok();
}

int hydra_ctx_destroy(hydra_ctx_t ctx) {
  if (!ctx) return ok();
  hydra::DeviceScope ds(ctx->device);
  // (its calls were synchronous: nothing of this context is left on the resident reducer,
  // whose instance leaves by itself when idle)
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  ctx_release(ctx);
  delete ctx;
  return ok();
}

namespace {
// One operand of a host call: its mapped windows (host_map.h) in element units.
struct Operand {
  const char* base = nullptr;
  hydra::HostWindows win;
  size_t lo[hydra::kMaxWindows] = {}, hi[hydra::kMaxWindows] = {};
  int n = 0;
  // the window [i, j) lies in, or -1
  int window_of(size_t i, size_t j) const {
    for (int k = 0; k < n; k++)
      if (lo[k] <= i && j <= hi[k]) return k;
    return -1;
  }
  // device address of element i if [i, j) lies in one window, else null
  char* dev(size_t i, size_t j, size_t es) const {
    const int k = window_of(i, j);
    return k >= 0 ? win.w[k].dev + (base + i * es - win.w[k].lo) : nullptr;
  }
};

void set_ranges(Operand* o, size_t es, size_t n) {
  o->n = 0;
  for (int k = 0; k < o->win.count; k++) {
    const hydra::HostWindow& w = o->win.w[k];
    size_t l = (size_t(w.lo - o->base) + es - 1) / es;
    size_t h = std::min(n, size_t(w.hi - o->base) / es);
    if (l < h) {
      o->lo[o->n] = l;
      o->hi[o->n] = h;
      if (o->n != k) o->win.w[o->n] = o->win.w[k];  // (keys stay in win for the release)
      o->n++;
    }
  }
}

// Releases the windows of a call when it returns -- declared before the drain, so any work
// still enqueued is drained first.
struct WindowsGuard {
  hydra::HostWindows* w[3];
  int k = 0;
  ~WindowsGuard() {
    for (int i = 0; i < k; i++) hydra::host_windows_release(w[i]);
  }
};

}  // namespace

int hydra_reduce_host(hydra_ctx_t ctx, int op, int dtype, void* c, const void* a, const void* b,
                      size_t n) {
  hydra::TraceRange trace_("hydra_reduce_host");
  if (!ctx) return fail(HYDRA_ERR_INVALID, "null context");
  int rc = check_args(op, dtype, c, a, b, n);
  if (rc) return rc;
  if (n == 0) return ok();
  const size_t es = hydra::dtype_size(dtype);
  const hydra::CtxOpts& opts = ctx->opts;
  const size_t nbytes = n * es;
  const bool tracing = g_trace_on.load(std::memory_order_relaxed);
  const Clock::time_point t_call = tracing ? Clock::now() : Clock::time_point();
  hydra_host_call_t rec{};
  rec.n = n;
  rec.elem_bytes = es;
  // Each operand's mapped windows (host_map.h): the parts the kernel reads / writes in place
  // over PCIe -- a registered bucket (hydra_host_register), a pinned block (hydra_malloc_host,
  // e.g. the ring's receive slots after setScratchAllocator(pinnedAlloc)) or the caller's own
  // pinned / registered memory.  Everything else -- pageable memory, the ragged first / last
  // page of a registered range -- is copied by the CPU into the context's pinned staging and
  // reduced there (pageable memory is never pinned for a call: DESIGN.md §10).  The whole call
  // is one batched kernel launch per staging round (one round unless more than kSlotBytes per
  // operand must be staged).  HYDRA_OPT_FORCE_STAGING stages everything (A/B).
  Operand oc, oa, ob;
  oc.base = static_cast<const char*>(c);
  oa.base = static_cast<const char*>(a);
  ob.base = static_cast<const char*>(b);
  Operand* A = a == c ? &oc : &oa;
  Operand* B = b == c ? &oc : b == a ? A : &ob;
  WindowsGuard guard_;
  if (opts[HYDRA_OPT_FORCE_STAGING] == 0) {
    for (Operand* o : {&oc, A, B}) {
      bool seen = false;
      for (int i = 0; i < guard_.k; i++) seen = seen || guard_.w[i] == &o->win;
      if (seen) continue;
      hydra::host_windows_acquire(o->base, nbytes, &o->win);
      guard_.w[guard_.k++] = &o->win;
      if (o->win.device)
        return fail(HYDRA_ERR_INVALID,
                    "hydra_reduce_host: an operand is device memory (use hydra_reduce)");
      set_ranges(o, es, n);
    }
  }
  // intervals between window edges: inside one, every operand is either mapped throughout or
  // staged throughout
  std::vector<size_t> cut{0, n};
  for (const Operand* o : {&oc, A, B})
    for (int k = 0; k < o->n; k++) cut.insert(cut.end(), {o->lo[k], o->hi[k]});
  std::sort(cut.begin(), cut.end());
  cut.erase(std::unique(cut.begin(), cut.end()), cut.end());

  const bool c_old_bits = dtype == HYDRA_FLOAT16 && c != a && c != b;  // store quirk: read c
  const bool stage_result_all =
      dtype != HYDRA_FLOAT16 && nbytes <= (size_t)opts[HYDRA_OPT_STAGE_RESULT_MAX];
  // per interval: its result goes through the staging when the window holding that interval of
  // c is a small (cache-resident) registration; a large registration or a caller mapping keeps
  // the zero-copy write
  auto stage_result_in = [&](size_t i, size_t j) {
    if (dtype == HYDRA_FLOAT16) return false;
    if (stage_result_all) return true;
    const int k = oc.window_of(i, j);
    return k >= 0 && oc.win.w[k].kind == hydra::kMapRegister &&
           oc.win.w[k].entry_bytes <= (size_t)opts[HYDRA_OPT_STAGE_RESULT_REG_MAX];
  };
  // Rounds: a round is one batched call over at most kResidentSegs intervals and one staging
  // buffer's slots.  Round r is submitted once round r - 1 is done; its staged results go back
  // to c while round r runs, and the CPU fills the other buffer meanwhile.  Submitted to the
  // resident reducer when the context holds a slot, else launched on the context's stream.
  hydra::ResidentLease* const lease = hydra::resident_usable(ctx->lease) ? ctx->lease : nullptr;
  bool poisoned = false;  // a failed resident wait could not confirm the grid gone: keep windows
  std::vector<hydra::BatchSegDesc> segs;
  segs.reserve(hydra::kResidentSegs);
  std::vector<hydra::CopyJob> ins;      // the current round's copies into the staging
  std::vector<hydra::CopyJob> outs[2];  // each buffer's staged results, back to c
  size_t used[3] = {0, 0, 0};  // bytes of the current buffer's a, b, c slots
  int buf = 0;
  bool pending = false;  // the other buffer's round is in flight
  auto timed = [&](double* acc, auto&& f) {  // f's wall time into *acc while tracing
    if (!tracing) return f();
    const Clock::time_point t0 = Clock::now();
    f();
    *acc += us_since(t0);
  };
  struct Drain {  // an early return waits for the round in flight before the windows go
    std::function<void()> f;
    ~Drain() {
      if (f) f();
    }
  } drain_;
  auto wait_round = [&](int k) -> int {
    const Clock::time_point t0 = tracing ? Clock::now() : Clock::time_point();
    struct Acc {
      bool on;
      Clock::time_point t0;
      double* acc;
      ~Acc() {
        if (on) *acc += us_since(t0);
      }
    } acc_{tracing, t0, &rec.wait_us};
    if (lease) {
      if (int r = hydra::resident_wait(lease, &poisoned)) {
        if (poisoned) guard_.k = 0;  // the grid may still touch them: they stay mapped
        // the failed wait already stopped the instance (or poisoned the server): there is no
        // round left to drain, so an early return must not wait for it a second time
        drain_.f = nullptr;
        return r;
      }
    } else {
      HIP_TRY(hipEventSynchronize(ctx->done[k]));
    }
    return HYDRA_OK;
  };
  auto flush = [&]() -> int {  // submit the current buffer's round
    if (segs.empty() && outs[buf].empty()) return HYDRA_OK;
    const int other = buf ^ 1;
    // the staged operands (fanned out when large)
    timed(&rec.copy_in_us, [&] { hydra::copy_all(ins.data(), ins.size()); });
    ins.clear();
    if (pending) {
      if (int r = wait_round(other)) return r;
      pending = false;
    }
    if (!segs.empty()) {
      if (lease) {
        if (int r = hydra::resident_submit(lease, op, dtype, es, segs.data(), segs.size()))
          return r;
      } else {
        hipError_t e =
            hydra::launch_reduce_batch(op, dtype, segs.data(), segs.size(), ctx->stream);
        if (e != hipSuccess) return hip_fail(e, "batched reduce kernel launch (host)");
        HIP_TRY(hipEventRecord(ctx->done[buf], ctx->stream));
      }
      pending = true;
      rec.rounds++;
      if (!drain_.f) {
        drain_.f = lease ? std::function<void()>([lease, &guard_] {
                             bool p = false;
                             (void)hydra::resident_wait(lease, &p);
                             if (p) guard_.k = 0;
                           })
                         : std::function<void()>([st = ctx->stream] {
                             (void)hipStreamSynchronize(st);
                           });
      }
    }
    // the previous round is done: its staged results back to c (overlapping this round)
    timed(&rec.copy_out_us, [&] { hydra::copy_all(outs[other].data(), outs[other].size()); });
    outs[other].clear();
    segs.clear();
    used[0] = used[1] = used[2] = 0;
    buf = other;
    return HYDRA_OK;
  };
  hydra::DeviceScope ds(lease ? -1 : ctx->device);  // launches go to the context's device
  HIP_TRY(ds.err);
  // A staged call is cut into about HYDRA_OPT_STAGE_SPLIT rounds (>= HYDRA_OPT_ROUND_MIN bytes
  // per operand, at most a slot), so its copies overlap the GPU's rounds: in at round r + 1 and
  // out at round r - 1 while round r runs.
  const size_t round_min = std::min<size_t>((size_t)opts[HYDRA_OPT_ROUND_MIN], kSlotBytes);
  const size_t round_cap = std::min(
      kSlotBytes,
      std::max(round_min, (nbytes / (size_t)opts[HYDRA_OPT_STAGE_SPLIT] + 255) / 256 * 256));
  for (size_t q = 0; q + 1 < cut.size(); q++) {
    size_t off = cut[q];
    const size_t end = cut[q + 1];
    while (off < end) {
      if (segs.size() == (size_t)hydra::kResidentSegs) {
        if ((rc = flush())) return rc;
      }
      char* dc = stage_result_in(off, end) ? nullptr : oc.dev(off, end, es);
      char* da = A->dev(off, end, es);
      char* db = B->dev(off, end, es);
      if (dc && da && db) {  // in place over PCIe
        segs.push_back({dc, da, db, end - off});
        for (int k = 0; k < 3; k++) rec.zero_copy_bytes[k] += (end - off) * es;
        off = end;
        continue;
      }
      // staged: as much of [off, end) as the current buffer's slots still hold
      const size_t room = round_cap - std::min(round_cap, std::max({used[0], used[1], used[2]}));
      if (room < 64 * es) {
        if ((rc = flush())) return rc;
        continue;
      }
      const size_t cnt = std::min(end - off, room / es);
      const size_t bytes = cnt * es;
      const size_t ob = off * es;
      if (tracing) {  // which operands of this interval the kernel touches in place
        const bool m[3] = {dc != nullptr, da != nullptr, db != nullptr};
        for (int k = 0; k < 3; k++) (m[k] ? rec.zero_copy_bytes[k] : rec.staged_bytes[k]) += bytes;
      }
      char* host_st = ctx->stage[buf];
      char* dev_st = ctx->stage_dev[buf];
      auto slot = [&](int k, const char* src, bool fill) -> char* {  // k: 0 a, 1 b, 2 c
        const size_t at = size_t(k) * kSlotBytes + used[k];
        if (fill) ins.push_back({host_st + at, src, bytes});
        used[k] += (bytes + 255) / 256 * 256;
        return dev_st + at;
      };
      const size_t mark_a = size_t(0) * kSlotBytes + used[0];
      const bool a_staged = !da, b_staged = !db;
      if (!da) da = slot(0, oa.base + ob, true);
      if (!db) {
        if (B == A)
          db = da;
        else
          db = slot(1, B->base + ob, true);
      }
      if (!dc) {  // (c == a / c == b: in the staged copy of that operand, if it is staged)
        if (c == a && a_staged) {
          dc = da;
          outs[buf].push_back({static_cast<char*>(c) + ob, host_st + mark_a, bytes});
        } else if (c == b && b_staged) {
          dc = db;
          outs[buf].push_back({static_cast<char*>(c) + ob,
                               host_st + (size_t(dc - dev_st)), bytes});
        } else {
          const size_t at = size_t(2) * kSlotBytes + used[2];
          dc = slot(2, oc.base + ob, c_old_bits);
          outs[buf].push_back({static_cast<char*>(c) + ob, host_st + at, bytes});
        }
      }
      segs.push_back({dc, da, db, cnt});
      off += cnt;
    }
  }
  if ((rc = flush())) return rc;
  if (pending) {  // the last round: done, results back
    if ((rc = wait_round(buf ^ 1))) return rc;
    pending = false;
    timed(&rec.copy_out_us,
          [&] { hydra::copy_all(outs[buf ^ 1].data(), outs[buf ^ 1].size()); });
  }
  drain_.f = nullptr;
  if (tracing) {
    rec.intervals = (uint32_t)(cut.size() - 1);
    rec.resident = lease ? 1u : 0u;
    rec.total_us = us_since(t_call);
    std::lock_guard<std::mutex> g(g_trace_mu);
    if (g_trace->size() < kTraceCap) g_trace->push_back(rec);
  }
  return ok();  // the windows are released here, after every round finished
}

int hydra_host_trace(int enable) {
  std::lock_guard<std::mutex> g(g_trace_mu);
  if (enable) g_trace->clear();
  g_trace_on.store(enable != 0);
  return ok();
}

int hydra_host_trace_read(hydra_host_call_t* out, size_t cap, size_t* count) {
  std::lock_guard<std::mutex> g(g_trace_mu);
  if (count) *count = g_trace->size();
  if (out)
    std::memcpy(out, g_trace->data(), std::min(cap, g_trace->size()) * sizeof(hydra_host_call_t));
  return ok();
}

int hydra_ctx_stats(hydra_ctx_t ctx, uint64_t* resident_calls, uint64_t* resident_launches) {
  if (!ctx) return fail(HYDRA_ERR_INVALID, "null context");
  if (resident_calls) *resident_calls = hydra::resident_calls(ctx->lease);
  if (resident_launches) *resident_launches = hydra::resident_launches(ctx->device);
  return ok();
}

int hydra_chunk_sum_host(hydra_ctx_t ctx, int dtype, void* c, const void* a, const void* b,
                         size_t n) {
  return hydra_reduce_host(ctx, HYDRA_SUM, dtype, c, a, b, n);
}

int hydra_host_register(void* ptr, size_t bytes) {
  const char* what = "";
  const int rc = hydra::host_register(ptr, bytes, &what);
  if (rc != HYDRA_OK) return fail(rc, std::string("hydra_host_register: ") + what);
  return ok();
}

int hydra_host_unregister(void* ptr) {
  const char* what = "";
  const int rc = hydra::host_unregister(ptr, &what);
  if (rc != HYDRA_OK) return fail(rc, std::string("hydra_host_unregister: ") + what);
  return ok();
}

int hydra_host_mappings(hydra_host_mapping_t* out, size_t cap, size_t* count,
                        uint64_t* registrations, uint64_t* outside) {
  std::vector<hydra::HostMapEntry> v(cap);
  const size_t k = hydra::host_map_snapshot(v.data(), cap);
  for (size_t i = 0; i < std::min(k, cap) && out; i++)
    out[i] = hydra_host_mapping_t{v[i].lo, v[i].hi, v[i].kind, v[i].owners, v[i].users,
                                  v[i].owner_lo, v[i].owner_hi};
  if (count) *count = k;
  hydra::host_map_counters(registrations, outside);
  return ok();
}

void hydra_page_interior(uint64_t ptr, size_t bytes, uint64_t* lo, uint64_t* hi) {
  uintptr_t l = 0, h = 0;
  hydra::page_interior(static_cast<uintptr_t>(ptr), bytes, &l, &h);
  if (lo) *lo = l;
  if (hi) *hi = h;
}

// ---- helpers --------------------------------------------------------------------------------
int hydra_stream_create(int device, hydra_stream_t* out) {
  if (!out) return fail(HYDRA_ERR_INVALID, "null out");
  hipStream_t s = nullptr;
  HIP_TRY(hydra::cached_stream(device, &s));
  *out = s;
  return ok();
}

int hydra_stream_destroy(hydra_stream_t s) {
  if (s) HIP_TRY(hydra::release_stream(static_cast<hipStream_t>(s)));
  return ok();
}

int hydra_stream_synchronize(hydra_stream_t s) {
  HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(s)));
  return ok();
}

int hydra_event_create(hydra_event_t* out) { return hydra_event_create_on(-1, out); }

int hydra_event_create_on(int device, hydra_event_t* out) {
  if (!out) return fail(HYDRA_ERR_INVALID, "null out");
  hipEvent_t e = nullptr;
  HIP_TRY(hydra::cached_event(device, &e));
  *out = e;
  return ok();
}

int hydra_event_record(hydra_event_t e, hydra_stream_t s) {
  if (!e) return fail(HYDRA_ERR_INVALID, "null event");
  HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(e), static_cast<hipStream_t>(s)));
  return ok();
}

int hydra_event_synchronize(hydra_event_t e) {
  if (!e) return fail(HYDRA_ERR_INVALID, "null event");
  HIP_TRY(hipEventSynchronize(static_cast<hipEvent_t>(e)));
  return ok();
}

int hydra_event_destroy(hydra_event_t e) {
  if (e) HIP_TRY(hydra::release_event(static_cast<hipEvent_t>(e)));
  return ok();
}

int hydra_stream_wait_event(hydra_stream_t s, hydra_event_t e) {
  if (!e) return fail(HYDRA_ERR_INVALID, "null event");
  HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(s), static_cast<hipEvent_t>(e), 0));
  return ok();
}

int hydra_device_peer_access(int device, int peer, int* can) {
  if (!can) return fail(HYDRA_ERR_INVALID, "null out");
  *can = 0;
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (device < 0 || device >= count || peer < 0 || peer >= count)
    return fail(HYDRA_ERR_NO_DEVICE, "no such device");
  if (device == peer) {
    *can = 1;
    return ok();
  }
  int c = 0;
  HIP_TRY(hipDeviceCanAccessPeer(&c, device, peer));
  if (!c) return ok();
  hydra::DeviceScope ds(device);
  HIP_TRY(ds.err);
  const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hip_fail(e, "hipDeviceEnablePeerAccess");
  (void)hipGetLastError();  // (already enabled is not an error here)
  *can = 1;
  return ok();
}

int hydra_device_link(int device, int peer, int* link, int* hops, int* can_peer) {
  if (!link || !hops || !can_peer) return fail(HYDRA_ERR_INVALID, "null out");
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));
  if (device < 0 || device >= count || peer < 0 || peer >= count || device == peer)
    return fail(HYDRA_ERR_INVALID, "need two distinct visible devices");
  uint32_t t = 0, h = 0;
  HIP_TRY(hipExtGetLinkTypeAndHopCount(device, peer, &t, &h));
  int c = 0;
  HIP_TRY(hipDeviceCanAccessPeer(&c, device, peer));
  *link = (int)t;
  *hops = (int)h;
  *can_peer = c;
  return ok();
}

int hydra_malloc(int device, size_t bytes, void** out) {
  if (!out) return fail(HYDRA_ERR_INVALID, "null out");
  HIP_TRY(hydra::cached_malloc(device, bytes, out));
  return ok();
}

int hydra_free(void* p) {
  if (p) HIP_TRY(hydra::cached_free(p));
  return ok();
}

int hydra_cache_trim(void) {
  HIP_TRY(hydra::trim_caches());
  return ok();
}

int hydra_memcpy(void* dst, const void* src, size_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
  return ok();
}

int hydra_memcpy_async(void* dst, const void* src, size_t bytes, hydra_stream_t stream) {
  if (!bytes) return ok();
  if (!dst || !src) return fail(HYDRA_ERR_INVALID, "null pointer");
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
  return ok();
}

int hydra_malloc_host(size_t bytes, void** out) {
  if (!out) return fail(HYDRA_ERR_INVALID, "null out");
  HIP_TRY(hydra::cached_malloc_host(bytes, out));
  return ok();
}

int hydra_free_host(void* p) {
  if (p) HIP_TRY(hydra::cached_free_host(p));
  return ok();
}

// CudaDevicePointer<T>::create's device lookup (cuda.cu:175-188): device of a device (or
// managed) allocation; -1 for host memory, registered or not.
int hydra_pointer_device(const void* p, int* device) {
  if (!p || !device) return fail(HYDRA_ERR_INVALID, "null pointer");
  hipPointerAttribute_t a{};
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {  // plain pageable host memory is unknown to the runtime
    (void)hipGetLastError();
    *device = -1;
    return ok();
  }
  *device = (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) ? a.device : -1;
  return ok();
}

// allreduce.cc:199-221 -- identical integer arithmetic.
void hydra_ring_plan(int P, size_t n, size_t esize, size_t max_segment, size_t* num_segments,
                     size_t* segment_bytes, size_t* segments_per_rank) {
  auto round_up = [](size_t v, size_t m) {
    const size_t r = v % m;
    return r ? v + m - r : v;
  };
  const size_t total = n * esize;
  const size_t max_seg_bytes = esize * std::max<size_t>(1, max_segment / esize);
  const size_t ns = round_up(std::max((total + max_seg_bytes - 1) / max_seg_bytes,
                                      (size_t)P * 2),
                             (size_t)P);
  if (num_segments) *num_segments = ns;
  if (segments_per_rank) *segments_per_rank = ns / (size_t)P;
  if (segment_bytes) *segment_bytes = round_up((total + ns - 1) / ns, esize);
}

}  // extern "C"
