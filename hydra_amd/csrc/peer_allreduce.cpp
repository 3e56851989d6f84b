// peer_allreduce.cpp -- host side of the peer-access bucket allreduce (peer_kernels.hip).
//
// One process per GPU.  Buckets and the per-rank signal area are shared by hipIpc handles;
// the handles travel through whatever channel the caller has (the reference's rendezvous store,
// torch.distributed, a pipe): this file only produces and consumes opaque byte blobs.  After
// that, hydra_peer_allreduce is ONE kernel launch on the caller's stream -- no host
// synchronisation, no RCCL, graph-capturable (barrier epochs are kept on the device) -- whose
// reads of the peers' blocks travel over xGMI.  Geometry and fold order are the reference ring's (xgmi_plan.h make_geom), so results
// equal gloo::allreduce RING (allreduce.cc:147-422) bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "fault_report.h"
#include "../../include/hydra_hip.h"
#include "errors.h"
#include "peer_kernels.h"
#include "reduce_kernels.h"
#include "resident.h"
#include "resource_cache.h"
#include "trace.h"
#include "xgmi_plan.h"

using hydra::fail;
using hydra::ok;

namespace {

constexpr uint64_t kMagic = 0x3152505241445948ull;  // "HYDRAPR1"
constexpr size_t kIpcBytes = sizeof(hipIpcMemHandle_t);
static_assert(kIpcBytes <= 64, "hipIpcMemHandle_t larger than the blob slot");

// Blob layout (HYDRA_PEER_HANDLE_BYTES): [0,64) hipIpcMemHandle_t of the allocation base,
// [64,72) offset of the buffer in it, [72,80) buffer bytes, [80,88) magic, [88,92) rank,
// [96,104) the exporter's allocation id (HIP_POINTER_ATTRIBUTE_BUFFER_ID: unique per
// allocation, so a freed-and-reallocated bucket whose IPC handle bytes repeat is a NEW mapping),
// [104,116) the exporter's GPU (PCI domain, bus, device: ranks on the same GPU share its CUs),
// [116,120) its compute units.
struct Blob {
  unsigned char ipc[64];
  uint64_t offset, bytes, magic;
  int32_t rank, pad;
  uint64_t alloc_id;
  int32_t pci[3];
  int32_t cus;
};
static_assert(sizeof(Blob) <= HYDRA_PEER_HANDLE_BYTES, "blob too large");

struct Mapping {
  void* base = nullptr;
  int refs = 0;
};

}  // namespace

struct hydra_peer {
  int P = 1, rank = 0, device = 0;
  int pci[3] = {0, 0, 0};  // this rank's GPU (PCI domain, bus, device)
  int cus = 0;             // its compute units
  // (connect) the most ranks of the group on any one GPU, and the fewest CUs of the group's
  // GPUs: the same on every rank, so every rank derives the same grid
  int colocated = 1, group_cus = 0;
  hydra::PeerSignals* sig = nullptr;  // own signal area (uncached device memory)
  hydra::PeerSigPtrs sigs{};          // every rank's, mapped
  uint32_t* err_host = nullptr;       // host-mapped error word the kernels write
  uint32_t* err_dev = nullptr;
  uint64_t timeout_ticks = 20ull * 100000000ull;  // 20 s at 100 MHz
  int blocks = 0;                                 // 0 = derived from the bucket
  // AUTO: ONE_SHOT up to this many bytes -- 0 since round 6: the push is as fast or faster at
  // every size measured, 1 KiB up (profiles/r06z), so ONE_SHOT is an explicit choice
  size_t one_shot_max = 0;
  char* scratch = nullptr;
  size_t scratch_bytes = 0;
  struct Reg {
    char* base;
    size_t bytes;
    const void* alloc_base;  // base of the device allocation holding it (its export record)
    char* peer[hydra::kPeerMaxRanks];
    std::string key[hydra::kPeerMaxRanks];
  };
  std::vector<Reg> regs;
  std::map<std::string, Mapping> opened;  // (rank, allocation id, ipc bytes) -> mapping
  std::map<const void*, uint64_t> exported;  // own allocation base -> allocation id exported
  bool detached = false;                  // hydra_peer_detach ran: no mappings left
  // the last call's completion: the next call's kernel waits for it, so two calls issued on
  // different streams never run at once (their workgroups share the barrier epochs and the
  // one-shot scratch)
  hipEvent_t last = nullptr;
  bool last_valid = false;
#ifdef HYDRA_MEASURE
  uint64_t* stamps = nullptr;  // hydra_measure_peer_stamps: per-workgroup phase clocks
  size_t stamps_cap = 0;       // workgroups it holds
#endif
};

namespace {

int export_blob(hydra_peer* p, void* ptr, size_t bytes, void* out) {
  void* base = nullptr;
  size_t size = 0;
  HIP_TRY(hipMemGetAddressRange(&base, &size, ptr));
  const char* b = static_cast<const char*>(base);
  const char* q = static_cast<const char*>(ptr);
  if (q < b || q + bytes > b + size)
    return fail(HYDRA_ERR_INVALID, "buffer is not inside one device allocation");
  unsigned long long id = 0;
  HIP_TRY(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                 reinterpret_cast<hipDeviceptr_t>(base)));
  // Register once: an allocation base with an OPEN registration in this group must still be
  // the SAME allocation.  Freeing a registered bucket and exporting a new allocation there
  // while peers may still map the old one (round 1: peers read zeros/garbage after free +
  // re-register) is refused; hydra_peer_close the old registration on every rank first.
  auto ex = p->exported.find(base);
  if (ex != p->exported.end() && ex->second != (uint64_t)id)
    return fail(HYDRA_ERR_INVALID,
                "allocation at this address changed since it was exported to the peer group "
                "(register a bucket once; hydra_peer_close it on every rank before freeing it)");
  hipIpcMemHandle_t h;
  HIP_TRY(hipIpcGetMemHandle(&h, base));
  Blob blob{};
  std::memcpy(blob.ipc, &h, kIpcBytes);
  blob.offset = (uint64_t)(q - b);
  blob.bytes = bytes;
  blob.magic = kMagic;
  blob.rank = p->rank;
  blob.alloc_id = (uint64_t)id;
  std::memcpy(blob.pci, p->pci, sizeof(blob.pci));
  blob.cus = p->cus;
  std::memset(out, 0, HYDRA_PEER_HANDLE_BYTES);
  std::memcpy(out, &blob, sizeof(blob));
  return HYDRA_OK;
}

int parse_blob(const void* in, int expect_rank, Blob* blob) {
  std::memcpy(blob, in, sizeof(Blob));
  if (blob->magic != kMagic) return fail(HYDRA_ERR_INVALID, "not a hydra peer handle");
  if (blob->rank != expect_rank)
    return fail(HYDRA_ERR_INVALID, "peer handles out of rank order");
  return HYDRA_OK;
}

// Map a peer allocation (cached: several buffers may share one allocation).
int open_mapping(hydra_peer* p, const Blob& b, std::string* key, char** base) {
  // keyed by exporter rank + allocation id + handle bytes, never by the handle bytes alone
  *key = std::to_string(b.rank) + ":" + std::to_string(b.alloc_id) + ":" +
         std::string(reinterpret_cast<const char*>(b.ipc), kIpcBytes);
  auto it = p->opened.find(*key);
  if (it == p->opened.end()) {
    hipIpcMemHandle_t h;
    std::memcpy(&h, b.ipc, kIpcBytes);
    void* m = nullptr;
    HIP_TRY(hipIpcOpenMemHandle(&m, h, hipIpcMemLazyEnablePeerAccess));
    {
      void* mb = nullptr;
      size_t msz = 0;
      if (hipMemGetAddressRange(&mb, &msz, m) != hipSuccess || mb != m) {
        (void)hipGetLastError();
        msz = b.offset + b.bytes;  // at least what this registration reads
      }
      hydra::ledger_add(hydra::kLedgerPeerMapping, m, msz);
    }
    it = p->opened.emplace(*key, Mapping{m, 0}).first;
  }
  it->second.refs++;
  *base = static_cast<char*>(it->second.base);
  return HYDRA_OK;
}

void close_mapping(hydra_peer* p, const std::string& key) {
  auto it = p->opened.find(key);
  if (it == p->opened.end()) return;
  if (--it->second.refs <= 0) {
    (void)hipIpcCloseMemHandle(it->second.base);
    hydra::ledger_release(hydra::kLedgerPeerMapping, it->second.base);
    p->opened.erase(it);
  }
}

// Workgroups of one peer kernel each rank may launch: when ranks of the group share a GPU, every
// rank's whole grid must be resident at once (workgroup b of one rank waits for workgroup b of
// the others, so a grid that fills the CUs while a peer's waits behind it never finishes), so
// colocated x grid <= CUs x (workgroups of that kernel per CU).  0 = no limit (a GPU per rank).
int colocated_cap(const hydra_peer* p, int algo, int op, int dtype, bool acc32) {
  if (p->colocated <= 1) return 0;
  int per_cu = 0;
  if (hydra::peer_occupancy(algo, op, dtype, acc32, &per_cu) != hipSuccess || per_cu < 1)
    per_cu = 1;
  return std::max(1, p->group_cus * per_cu / p->colocated);
}

const hydra_peer::Reg* find_reg(const hydra_peer* p, const void* buf, size_t bytes) {
  const char* b = static_cast<const char*>(buf);
  for (const auto& r : p->regs)
    if (b >= r.base && b + bytes <= r.base + r.bytes) return &r;
  return nullptr;
}

}  // namespace

extern "C" {

int hydra_peer_create(int nranks, int rank, int device, hydra_peer_t* out, void* sig_handle) {
  if (!out || !sig_handle) return fail(HYDRA_ERR_INVALID, "null argument");
  *out = nullptr;
  if (nranks < 1 || nranks > hydra::kPeerMaxRanks || rank < 0 || rank >= nranks)
    return fail(HYDRA_ERR_INVALID, "bad rank/nranks (peer allreduce: 1..8 ranks)");
  hydra::DeviceScope ds(device);
  HIP_TRY(ds.err);
  auto* p = new hydra_peer();
  p->P = nranks;
  p->rank = rank;
  p->device = device;
  hipError_t e = hipDeviceGetAttribute(&p->pci[0], hipDeviceAttributePciDomainID, device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&p->pci[1], hipDeviceAttributePciBusId, device);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&p->pci[2], hipDeviceAttributePciDeviceId, device);
  if (e == hipSuccess)
    e = hipDeviceGetAttribute(&p->cus, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = hipExtMallocWithFlags(reinterpret_cast<void**>(&p->sig),
                                       sizeof(hydra::PeerSignals), hipDeviceMallocUncached);
  if (e == hipSuccess) hydra::ledger_add(hydra::kLedgerPeerLocal, p->sig, sizeof(hydra::PeerSignals));
  if (e == hipSuccess) e = hipMemset(p->sig, 0, sizeof(hydra::PeerSignals));
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void**>(&p->err_host), sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    *p->err_host = 0;
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&p->err_dev), p->err_host, 0);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&p->last, hipEventDisableTiming);
  if (e == hipSuccess) e = hydra::drain_device(device);
  if (e != hipSuccess) {
    hydra_peer_destroy(p);
    return hydra::hip_fail(e, "hydra_peer_create");
  }
  p->sigs.p[rank] = p->sig;
  int rc = export_blob(p, p->sig, sizeof(hydra::PeerSignals), sig_handle);
  if (rc) {
    hydra_peer_destroy(p);
    return rc;
  }
  *out = p;
  return ok();
}

int hydra_peer_connect(hydra_peer_t p, const void* sig_handles) {
  if (!p || !sig_handles) return fail(HYDRA_ERR_INVALID, "null argument");
  hydra::DeviceScope ds_(p->device);  // IPC mappings and drains on the group's device
  const char* h = static_cast<const char*>(sig_handles);
  // every rank sees the same blobs: the busiest GPU's rank count and the smallest CU count
  // decide the co-resident grid alike everywhere (a rank with a GPU of its own in a group
  // where others share one must still launch the same grid: workgroup b meets workgroup b)
  int colocated = 1, group_cus = p->cus;
  for (int q = 0; q < p->P; q++) {
    Blob bq;
    int rc = parse_blob(h + (size_t)q * HYDRA_PEER_HANDLE_BYTES, q, &bq);
    if (rc) return rc;
    int same = 0;
    for (int j = 0; j < p->P; j++) {
      Blob bj;
      std::memcpy(&bj, h + (size_t)j * HYDRA_PEER_HANDLE_BYTES, sizeof(Blob));
      if (std::memcmp(bj.pci, bq.pci, sizeof(bq.pci)) == 0) same++;
    }
    colocated = std::max(colocated, same);
    if (bq.cus > 0) group_cus = std::min(group_cus, (int)bq.cus);
  }
  for (int q = 0; q < p->P; q++) {
    Blob b;
    int rc = parse_blob(h + (size_t)q * HYDRA_PEER_HANDLE_BYTES, q, &b);
    if (rc) return rc;
    if (q == p->rank || p->sigs.p[q]) continue;
    std::string key;
    char* base = nullptr;
    rc = open_mapping(p, b, &key, &base);
    if (rc) return rc;
    p->sigs.p[q] = reinterpret_cast<hydra::PeerSignals*>(base + b.offset);
  }
  p->colocated = colocated;
  p->group_cus = group_cus;
  return ok();
}

int hydra_peer_register(hydra_peer_t p, void* buf, size_t bytes, void* handle) {
  if (!p || !buf || !handle) return fail(HYDRA_ERR_INVALID, "null argument");
  hydra::DeviceScope ds_(p->device);  // IPC mappings and drains on the group's device
  const int rc = export_blob(p, buf, bytes, handle);
  return rc ? rc : ok();
}

int hydra_peer_open(hydra_peer_t p, void* buf, size_t bytes, const void* handles) {
  if (!p || !buf || !handles) return fail(HYDRA_ERR_INVALID, "null argument");
  hydra::DeviceScope ds_(p->device);  // IPC mappings and drains on the group's device
  const char* h = static_cast<const char*>(handles);
  hydra_peer::Reg reg{};
  reg.base = static_cast<char*>(buf);
  reg.bytes = bytes;
  unsigned long long alloc_id = 0;
  {
    void* ab = nullptr;
    size_t asz = 0;
    HIP_TRY(hipMemGetAddressRange(&ab, &asz, buf));
    HIP_TRY(hipPointerGetAttribute(&alloc_id, HIP_POINTER_ATTRIBUTE_BUFFER_ID,
                                   reinterpret_cast<hipDeviceptr_t>(ab)));
    reg.alloc_base = ab;
  }
  reg.peer[p->rank] = reg.base;
  for (int q = 0; q < p->P; q++) {
    Blob b;
    int rc = parse_blob(h + (size_t)q * HYDRA_PEER_HANDLE_BYTES, q, &b);
    if (!rc && b.bytes != bytes) rc = fail(HYDRA_ERR_INVALID, "ranks registered different sizes");
    if (!rc && q != p->rank) {
      char* base = nullptr;
      rc = open_mapping(p, b, &reg.key[q], &base);
      if (!rc) reg.peer[q] = base + b.offset;
    }
    if (rc) {
      for (int j = 0; j < q; j++)
        if (j != p->rank && !reg.key[j].empty()) close_mapping(p, reg.key[j]);
      return rc;
    }
  }
  // the export record starts once the registration is open on this rank (peers may map it
  // from now on); hydra_peer_close ends it.  An export that never got opened (a collective
  // register that failed elsewhere) leaves no record behind.
  p->exported[reg.alloc_base] = (uint64_t)alloc_id;
  p->regs.push_back(reg);
  return ok();
}

int hydra_peer_close(hydra_peer_t p, void* buf) {
  if (!p) return fail(HYDRA_ERR_INVALID, "null peer");
  hydra::DeviceScope ds_(p->device);  // IPC mappings and drains on the group's device
  for (size_t i = 0; i < p->regs.size(); i++) {
    if (p->regs[i].base != buf) continue;
    (void)hydra::drain_device(p->device);  // no kernel may still read through the mappings
    for (int q = 0; q < p->P; q++)
      if (q != p->rank) close_mapping(p, p->regs[i].key[q]);
    bool shared = false;  // another open registration in the same allocation keeps its record
    for (size_t j = 0; j < p->regs.size(); j++)
      if (j != i && p->regs[j].alloc_base == p->regs[i].alloc_base) shared = true;
    if (!shared) p->exported.erase(p->regs[i].alloc_base);
    p->regs.erase(p->regs.begin() + (long)i);
    return ok();
  }
  return fail(HYDRA_ERR_INVALID, "buffer was not opened on this peer group");
}

int hydra_peer_set_option(hydra_peer_t p, int key, long long value) {
  if (!p) return fail(HYDRA_ERR_INVALID, "null peer");
  switch (key) {
    case HYDRA_PEER_OPT_TIMEOUT_MS:
      if (value <= 0) return fail(HYDRA_ERR_INVALID, "timeout must be positive");
      p->timeout_ticks = (uint64_t)value * 100000ull;
      return ok();
    case HYDRA_PEER_OPT_BLOCKS: {
      if (value < 0 || value > hydra::kPeerMaxBlocks)
        return fail(HYDRA_ERR_INVALID, "blocks out of range");
      // ranks sharing this GPU: refuse a grid that none of the schedules' kernels could hold
      // at once on it (each call checks again for the kernel it launches) instead of a barrier
      // timeout later
      int cap = 0;
      for (int k : {hydra::kPeerTwoShotPush, hydra::kPeerTwoShot, hydra::kPeerOneShot})
        cap = std::max(cap, colocated_cap(p, k, HYDRA_SUM, HYDRA_FLOAT32, false));
      if (cap && value > cap)
        return fail(HYDRA_ERR_INVALID,
                    "blocks " + std::to_string(value) + " x " + std::to_string(p->colocated) +
                        " ranks sharing this GPU exceeds its resident capacity (at most " +
                        std::to_string(cap) + " workgroups per rank)");
      p->blocks = (int)value;
      return ok();
    }
    case HYDRA_PEER_OPT_ONE_SHOT_MAX:
      if (value < 0) return fail(HYDRA_ERR_INVALID, "negative size");
      p->one_shot_max = (size_t)value;
      return ok();
  }
  return fail(HYDRA_ERR_INVALID, "unknown option");
}

int hydra_peer_error(hydra_peer_t p, int* code) {
  if (!p || !code) return fail(HYDRA_ERR_INVALID, "null argument");
  *code = (int)__atomic_load_n(p->err_host, __ATOMIC_ACQUIRE);
  return ok();
}

int hydra_peer_allreduce(hydra_peer_t p, int algo, int op, int dtype, int flags, void* buf,
                         size_t n, size_t max_segment, hydra_stream_t stream) {
  hydra::TraceRange trace_("hydra_peer_allreduce");
  if (!p) return fail(HYDRA_ERR_INVALID, "null peer");
  hydra::DeviceScope ds_(p->device);  // the group's device, restored on return
  if (p->detached) return fail(HYDRA_ERR_INVALID, "peer group detached");
  const size_t es = hydra::dtype_size(dtype);
  if (!es) return fail(HYDRA_ERR_INVALID, "invalid dtype");
  if (op < HYDRA_SUM || op > HYDRA_MIN) return fail(HYDRA_ERR_INVALID, "invalid op");
  if (algo < HYDRA_PEER_AUTO || algo > HYDRA_PEER_TWO_SHOT_PUSH)
    return fail(HYDRA_ERR_INVALID, "invalid peer algorithm");
  const bool acc32 = (flags & HYDRA_ACC_F32) != 0;
  if (acc32 && dtype != HYDRA_BFLOAT16)
    return fail(HYDRA_ERR_UNSUPPORTED, "HYDRA_ACC_F32 needs a bf16 bucket");
  if (*p->err_host)
    return fail(HYDRA_ERR_HIP, "peer group is broken: an earlier barrier timed out (code " +
                                   std::to_string(*p->err_host) + ")");
  if (n == 0 || p->P == 1) return ok();  // allreduce.cc:129-133
  if (!buf) return fail(HYDRA_ERR_INVALID, "null buffer");
  if (reinterpret_cast<uintptr_t>(buf) % es)
    return fail(HYDRA_ERR_INVALID, "buffer not aligned to the element size");
  for (int q = 0; q < p->P; q++)
    if (!p->sigs.p[q]) return fail(HYDRA_ERR_INVALID, "hydra_peer_connect has not run");
  const hydra_peer::Reg* reg = find_reg(p, buf, n * es);
  if (!reg) return fail(HYDRA_ERR_INVALID, "bucket is not inside a buffer opened by hydra_peer_open");
  if (algo == HYDRA_PEER_AUTO)
    algo = n * es <= p->one_shot_max ? HYDRA_PEER_ONE_SHOT : HYDRA_PEER_TWO_SHOT_PUSH;

  const hydra::PlanGeom g =
      hydra::make_geom(p->P, n, es, max_segment ? max_segment : (1u << 20), 0);
  hydra::PeerLaunch A{};
  const size_t off = static_cast<const char*>(buf) - reg->base;
  for (int q = 0; q < p->P; q++) {
    A.x[q] = reg->peer[q] + off;
    A.sync.sig.p[q] = p->sigs.p[q];
    A.lo[q] = g.block_begin(q) / es;
  }
  A.lo[p->P] = n;
  A.sync.err = p->err_dev;
  A.sync.timeout_ticks = p->timeout_ticks;
  A.sync.P = p->P;
  A.sync.rank = p->rank;
  // work unit: 64 KiB slabs for big buckets; smaller (down to 4 KiB) so that a small bucket
  // still spreads over ~256 workgroups.  Depends on (P, n, dtype) only: identical on all ranks.
  const size_t span = algo == HYDRA_PEER_ONE_SHOT ? n * es : g.max_block();
  size_t slab = hydra::kPeerSlabBytes;
  while (slab > hydra::kPeerMinSlabBytes && span / slab < 256) slab >>= 1;
  A.slab_bytes = slab;
  size_t work = 0;  // slabs of the largest block (two-shot) / of the bucket (one-shot)
  if (algo == HYDRA_PEER_ONE_SHOT)
    for (int q = 0; q < p->P; q++) work += (g.block_bytes(q) + slab - 1) / slab;
  else
    work = (g.max_block() + slab - 1) / slab;
  // grid: one workgroup per slab, at most 256 (one per CU).  The deep fold holds ~250 VGPRs,
  // so a CU runs two of these workgroups at once: every workgroup of the grid is resident, with
  // room for the same grid of a second rank when ranks share a GPU (the one-GPU tests); the
  // depth comes from each wave (peer_kernels.hip slab_fold_n), not from more workgroups, which
  // measured no faster (profiles/r05h, r05m)
  size_t grid =
      p->blocks > 0 ? (size_t)p->blocks : std::min<size_t>(std::max<size_t>(work, 1), 256);
  if (algo == HYDRA_PEER_TWO_SHOT_PUSH) {
    // the push stores the folded vectors into every bucket at the local bucket's alignment:
    // every rank's bucket must sit at the same address mod 16 (true for the usual 256-B aligned
    // allocations); otherwise TWO_SHOT, which every rank decides alike (congruence is shared)
    for (int q = 0; q < p->P; q++)
      if ((reinterpret_cast<uintptr_t>(A.x[q]) & 15) != (reinterpret_cast<uintptr_t>(A.x[p->rank]) & 15))
        algo = HYDRA_PEER_TWO_SHOT;
  }
  const int kalgo = algo == HYDRA_PEER_ONE_SHOT        ? hydra::kPeerOneShot
                    : algo == HYDRA_PEER_TWO_SHOT_PUSH ? hydra::kPeerTwoShotPush
                                                       : hydra::kPeerTwoShot;
  if (const int cap = colocated_cap(p, kalgo, op, dtype, acc32)) {
    if (p->blocks > 0 && grid > (size_t)cap)
      return fail(HYDRA_ERR_INVALID,
                  "blocks " + std::to_string(grid) + " x " + std::to_string(p->colocated) +
                      " ranks sharing this GPU exceeds its resident capacity for this kernel (at "
                      "most " + std::to_string(cap) + " workgroups per rank)");
    grid = std::min(grid, (size_t)cap);  // the derived grid shrinks to fit
  }
  if (algo == HYDRA_PEER_ONE_SHOT) {
    if (p->scratch_bytes < n * es) {
      HIP_TRY(hydra::drain_device(p->device));  // first call at a new size: outside any capture
      if (p->scratch) {
        HIP_TRY(hipFree(p->scratch));
        hydra::ledger_release(hydra::kLedgerPeerLocal, p->scratch);
      }
      p->scratch = nullptr;
      p->scratch_bytes = 0;
      HIP_TRY(hipMalloc(reinterpret_cast<void**>(&p->scratch), n * es));
      hydra::ledger_add(hydra::kLedgerPeerLocal, p->scratch, n * es);
      p->scratch_bytes = n * es;
    }
    A.scratch = p->scratch;
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  // Calls on one group run one after another on the device whatever streams they are issued
  // on: each EAGER call waits for the group's completion marker and records it.  A call being
  // captured neither waits (a capture may not wait on an outside event) nor records (an event
  // recorded inside a capture is a graph node, not a marker an eager call can wait on), so a
  // graph's replays must be ordered by the caller against each other and against eager calls
  // on other streams (hydra_hip.h).
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(st, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (!capturing && p->last_valid) HIP_TRY(hipStreamWaitEvent(st, p->last, 0));
#ifdef HYDRA_MEASURE
  if (p->stamps && grid > p->stamps_cap)
    return fail(HYDRA_ERR_INVALID, "stamp buffer smaller than the grid");
  A.stamps = p->stamps;
#endif
  const hipError_t e = hydra::launch_peer(kalgo, op, dtype, acc32, A, (unsigned)grid, st);
  if (e != hipSuccess) return hydra::hip_fail(e, "peer allreduce kernel launch");
  if (!capturing) {
    HIP_TRY(hipEventRecord(p->last, st));
    p->last_valid = true;
  }
  return ok();
}

#ifdef HYDRA_MEASURE  // libhydra_measure.so only (include/hydra_measure.h)
int hydra_measure_peer_stamps(hydra_peer_t p, void* dev_buf, size_t max_workgroups) {
  if (!p) return fail(HYDRA_ERR_INVALID, "null peer");
  p->stamps = static_cast<uint64_t*>(dev_buf);
  p->stamps_cap = dev_buf ? max_workgroups : 0;
  return ok();
}
#endif

int hydra_peer_detach(hydra_peer_t p) {
  if (!p) return fail(HYDRA_ERR_INVALID, "null peer");
  hydra::DeviceScope ds_(p->device);  // the group's device, restored on return
  if (p->detached) return ok();
  (void)hydra::drain_device(p->device);  // no kernel of ours may still read through the mappings
  for (auto& kv : p->opened) {
    (void)hipIpcCloseMemHandle(kv.second.base);
    hydra::ledger_release(hydra::kLedgerPeerMapping, kv.second.base);
  }
  p->opened.clear();
  p->regs.clear();
  for (int q = 0; q < p->P; q++)
    if (q != p->rank) p->sigs.p[q] = nullptr;
  p->detached = true;
  return ok();
}

int hydra_peer_destroy(hydra_peer_t p) {
  if (!p) return ok();
  hydra::DeviceScope ds_(p->device);  // the group's device, restored on return
  (void)hydra_peer_detach(p);  // local; callers detach + barrier first (hydra_hip.h)
  if (p->scratch) {
    (void)hipFree(p->scratch);
    hydra::ledger_release(hydra::kLedgerPeerLocal, p->scratch);
  }
  if (p->sig) {
    (void)hipFree(p->sig);
    hydra::ledger_release(hydra::kLedgerPeerLocal, p->sig);
  }
  if (p->err_host) (void)hipHostFree(p->err_host);
  if (p->last) (void)hipEventDestroy(p->last);
  delete p;
  return ok();
}

}  // extern "C"
