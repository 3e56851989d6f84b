// hydra_capi.cpp -- the extern "C" boundary of libhydra_hip.so (declared in include/hydra_hip.h).
//
// Argument checking, error reporting (thread-local message + status code), the host-resident
// staging context, and the ring geometry.  Kernels live in reduce_kernels.hip.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hydra_hip.h"
#include "errors.h"
#include "fault_report.h"
#include "host_map.h"
#include "resource_cache.h"
#include "reduce_kernels.h"
#include "trace.h"

namespace {
thread_local std::string g_err;
std::atomic<int> g_variant{0};
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
int current_variant() { return g_variant.load(std::memory_order_relaxed); }
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
// Two streams ping-pong over fixed-size chunks: H2D(a,b) -> reduce -> D2H(c) on stream k%2, so
// chunk k+1's copies overlap chunk k's kernel and copy-back.
struct hydra_ctx {
  int device = 0;
  hipStream_t stream[2] = {nullptr, nullptr};
  void* da[2] = {nullptr, nullptr};
  void* db[2] = {nullptr, nullptr};
  void* dc[2] = {nullptr, nullptr};  // only for float16 with c != a
  size_t chunk_bytes = 0;
};

namespace {
constexpr size_t kChunkBytes = 8u << 20;
constexpr int kVariantForceStaging = 1000;  // hydra_set_variant value: host path always stages
constexpr int kVariantNoPinOnTheFly = 1001;  // pageable operands staged, not pinned per call

void ctx_release(hydra_ctx* x) {
  for (int i = 0; i < 2; i++) {
    if (x->stream[i]) (void)hydra::release_stream(x->stream[i]);
    if (x->da[i]) (void)hydra::cached_free(x->da[i]);
    if (x->db[i]) (void)hydra::cached_free(x->db[i]);
    if (x->dc[i]) (void)hydra::cached_free(x->dc[i]);
  }
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
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  struct Restore {  // the caller's current device is left as it was
    int d;
    ~Restore() {
      if (d >= 0) (void)hipSetDevice(d);
    }
  } restore_{prev};
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());  // surfaces an asynchronous fault of any enqueued work
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hydra::hip_fail(e, "sticky device error");
  return ok();
}

int hydra_set_variant(int variant) { return g_variant.exchange(variant); }

int hydra_reduce(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                 hydra_stream_t stream) {
  int rc = check_args(op, dtype, c, a, b, n);
  if (rc) return rc;
  if (n == 0) return ok();
  hipError_t e = hydra::launch_reduce(g_variant.load(std::memory_order_relaxed), op, dtype, c, a,
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
  auto* x = new hydra_ctx();
  x->device = device;
  x->chunk_bytes = kChunkBytes;
  hipError_t e = hipSetDevice(device);
  for (int i = 0; i < 2 && e == hipSuccess; i++) {
    e = hydra::cached_stream(device, &x->stream[i]);
    if (e == hipSuccess) e = hydra::cached_malloc(device, kChunkBytes, &x->da[i]);
    if (e == hipSuccess) e = hydra::cached_malloc(device, kChunkBytes, &x->db[i]);
  }
  if (e != hipSuccess) {
    ctx_release(x);
    delete x;
    return hip_fail(e, "hydra_ctx_create");
  }
  *out = x;
  return ok();
}

int hydra_ctx_destroy(hydra_ctx_t ctx) {
  if (!ctx) return ok();
  (void)hipSetDevice(ctx->device);
  for (int i = 0; i < 2; i++)
    if (ctx->stream[i]) (void)hipStreamSynchronize(ctx->stream[i]);
  ctx_release(ctx);
  delete ctx;
  return ok();
}

namespace {
// Host copies of pageable memory go in pieces of at most 1 MiB: up to that size the HIP runtime
// copies through its own staging buffers, above it it locks the caller's pages for the copy --
// page-rounded, so the lock's edge pages hold the operand's neighbours.  hydra
// never asks the runtime to lock memory outside an operand.
constexpr size_t kCopyPiece = 1u << 20;

hipError_t copy_pieces(void* dst, const void* src, size_t bytes, hipMemcpyKind kind,
                       hipStream_t st) {
  for (size_t off = 0; off < bytes; off += kCopyPiece) {
    const size_t b = std::min(kCopyPiece, bytes - off);
    hipError_t e = hipMemcpyAsync(static_cast<char*>(dst) + off,
                                  static_cast<const char*>(src) + off, b, kind, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The mapped windows of one call's operands, released (after the call's kernels finished)
// when the call returns.
struct Windows {
  hydra::HostWindow w[3];
  ~Windows() {
    for (auto& x : w) hydra::host_window_release(&x);
  }
};

// An operand's window in elements: [lo, hi) of [0, n) (empty: lo == hi == 0).
struct ElemRange {
  size_t lo = 0, hi = 0;
  bool covers(size_t a, size_t b) const { return lo <= a && b <= hi && a < b; }
  static ElemRange of(const hydra::HostWindow& w, const void* base, size_t es, size_t n) {
    ElemRange r;
    if (w.empty()) return r;
    const char* b = static_cast<const char*>(base);
    r.lo = (size_t(w.lo - b) + es - 1) / es;
    r.hi = std::min(n, size_t(w.hi - b) / es);
    if (r.lo >= r.hi) r = ElemRange{};
    return r;
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
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t es = hydra::dtype_size(dtype);
  const size_t per = ctx->chunk_bytes / es;
  const int variant = g_variant.load(std::memory_order_relaxed);
  const size_t nbytes = n * es;
  // Each operand's mapped window (host_map.h): the part of it the kernel may read / write in
  // place over PCIe -- a registered bucket (hydra_host_register), a pinned block
  // (hydra_malloc_host, e.g. the ring's receive slots after setScratchAllocator(pinnedAlloc)),
  // the caller's own pinned / registered memory, or, for a pageable operand, the whole pages
  // inside it pinned for this call.  Elements inside all three windows are reduced in one
  // zero-copy pass; the rest (the ragged edge pages of pageable operands, anything unmapped) is
  // staged through device buffers, per operand.  kVariantForceStaging stages everything;
  // kVariantNoPinOnTheFly maps only memory that is already mapped (A/B).
  Windows win;  // declared before the drain: released only after every stream is drained
  struct DrainOnError {
    hipStream_t* st;
    bool armed = true;
    ~DrainOnError() {
      if (armed)
        for (int i = 0; i < 2; i++)
          if (st[i]) (void)hipStreamSynchronize(st[i]);
    }
  } drain_{ctx->stream};
  ElemRange rc_, ra_, rb_;
  if (variant != kVariantForceStaging) {
    const bool pin = variant != kVariantNoPinOnTheFly;
    win.w[0] = hydra::host_window_acquire(c, nbytes, pin);
    rc_ = ElemRange::of(win.w[0], c, es, n);
    if (a == c) {
      ra_ = rc_;
    } else {
      win.w[1] = hydra::host_window_acquire(a, nbytes, pin);
      ra_ = ElemRange::of(win.w[1], a, es, n);
    }
    if (b == c) {
      rb_ = rc_;
    } else if (b == a) {
      rb_ = ra_;
    } else {
      win.w[2] = hydra::host_window_acquire(b, nbytes, pin);
      rb_ = ElemRange::of(win.w[2], b, es, n);
    }
  }
  const hydra::HostWindow& wc = win.w[0];
  const hydra::HostWindow& wa = a == c ? win.w[0] : win.w[1];
  const hydra::HostWindow& wb = b == c ? win.w[0] : b == a ? wa : win.w[2];
  // device address of element i of an operand inside its window
  auto dev = [es](const hydra::HostWindow& w, const void* base, size_t i) -> char* {
    return w.dev + (static_cast<const char*>(base) + i * es - w.lo);
  };
  // zero-copy region: inside all three windows
  const size_t z0 = std::max({rc_.lo, ra_.lo, rb_.lo});
  const size_t z1 = std::min({rc_.hi, ra_.hi, rb_.hi});
  const bool zero = z0 < z1;
  if (zero) {
    hipError_t e = hydra::launch_reduce(0, op, dtype, dev(wc, c, z0), dev(wa, a, z0),
                                        dev(wb, b, z0), z1 - z0, ctx->stream[0]);
    if (e != hipSuccess) return hip_fail(e, "reduce kernel launch (zero-copy)");
  }
  // the rest, staged per operand in chunks over both streams
  struct Span {
    size_t lo, hi;
  };
  Span spans[2] = {{0, zero ? z0 : n}, {zero ? z1 : n, n}};
  size_t k = zero ? 1 : 0;  // the zero-copy pass ran on stream 0
  for (const Span& sp : spans) {
    for (size_t off = sp.lo; off < sp.hi; off += per, k++) {
      const size_t cnt = std::min(per, sp.hi - off);
      const size_t bytes = cnt * es;
      const int s = (int)(k & 1);
      hipStream_t st = ctx->stream[s];
      const size_t ob = off * es;
      const char* pa = static_cast<const char*>(a) + ob;
      const char* pb = static_cast<const char*>(b) + ob;
      char* pc = static_cast<char*>(c) + ob;
      const bool ma = ra_.covers(off, off + cnt);
      const bool mb = rb_.covers(off, off + cnt);
      const bool mc = rc_.covers(off, off + cnt);
      // operand a: mapped in place, else staged
      const void* ka = ma ? static_cast<const void*>(dev(wa, a, off)) : ctx->da[s];
      if (!ma) HIP_TRY(copy_pieces(ctx->da[s], pa, bytes, hipMemcpyHostToDevice, st));
      const void* kb;
      if (b == a) {
        kb = ka;
      } else if (mb) {
        kb = dev(wb, b, off);
      } else {
        HIP_TRY(copy_pieces(ctx->db[s], pb, bytes, hipMemcpyHostToDevice, st));
        kb = ctx->db[s];
      }
      // destination: mapped in place; else in place on the staged a (c == a, the ring's form)
      // or a staging buffer of its own -- which must hold c's old bits for float16's store quirk
      void* kc;
      bool copy_back = false;
      if (mc) {
        kc = dev(wc, c, off);
      } else if (c == a && !ma) {
        kc = ctx->da[s];
        copy_back = true;
      } else {
        if (!ctx->dc[s]) HIP_TRY(hydra::cached_malloc(ctx->device, ctx->chunk_bytes, &ctx->dc[s]));
        kc = ctx->dc[s];
        if (dtype == HYDRA_FLOAT16) HIP_TRY(copy_pieces(kc, pc, bytes, hipMemcpyHostToDevice, st));
        copy_back = true;
      }
      hipError_t e = hydra::launch_reduce(variant >= 1000 ? 0 : variant, op, dtype, kc, ka, kb,
                                          cnt, st);
      if (e != hipSuccess) return hip_fail(e, "reduce kernel launch");
      if (copy_back) HIP_TRY(copy_pieces(pc, kc, bytes, hipMemcpyDeviceToHost, st));
    }
  }
  HIP_TRY(hipStreamSynchronize(ctx->stream[0]));
  HIP_TRY(hipStreamSynchronize(ctx->stream[1]));
  drain_.armed = false;
  return ok();  // the windows are released here, after every kernel finished
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
