// xgmi_allreduce.cpp -- multi-GPU bucket allreduce: RCCL p2p over xGMI + fused HIP reductions.
//
// The schedule is data (xgmi_plan.h).  This file interprets it:
//   * run_plan_rccl   one rank: SEND/RECV groups -> ncclGroupStart/ncclSend/ncclRecv/ncclGroupEnd
//                     on the comm stream; REDUCE/FOLD -> HIP kernels on the compute stream; the
//                     plan's cross-stream wait0/wait1 edges -> hipEventRecord /
//                     hipStreamWaitEvent.  No host synchronisation: the whole allreduce is
//                     enqueued asynchronously on the caller's stream.  The fork/join, events,
//                     kernels and RCCL collectives capture into hipGraphs (tested); RCCL p2p
//                     capture is untested (RCCL faults on send-to-self under capture).
//   * simulate        every rank's plan on one GPU in lock-step, device copies on a "fabric"
//                     stream standing in for xGMI -- the multi-GPU path's test bench.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <deque>
#include <iterator>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/hydra_hip.h"
#include "errors.h"
#include "resident.h"
#include "resource_cache.h"
#include "reduce_kernels.h"
#include "split_table.h"
#include "trace.h"
#include "xgmi_plan.h"

using hydra::fail;
using hydra::ok;

namespace {

int nccl_fail(ncclResult_t r, const char* what) {
  return fail(HYDRA_ERR_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}

#define NCCL_TRY(expr)                                 \
  do {                                                 \
    ncclResult_t r__ = (expr);                         \
    if (r__ != ncclSuccess) return nccl_fail(r__, #expr); \
  } while (0)

ncclDataType_t nccl_type(int dtype) {
  switch (dtype) {
    case HYDRA_INT8: return ncclInt8;
    case HYDRA_UINT8: return ncclUint8;
    case HYDRA_INT32: return ncclInt32;
    case HYDRA_UINT32: return ncclUint32;
    case HYDRA_INT64: return ncclInt64;
    case HYDRA_UINT64: return ncclUint64;
    case HYDRA_FLOAT32: return ncclFloat32;
    case HYDRA_FLOAT64: return ncclFloat64;
    case HYDRA_FLOAT16: return ncclFloat16;
    case HYDRA_BFLOAT16: return ncclBfloat16;
  }
  return ncclUint8;
}

ncclRedOp_t nccl_op(int op) {
  switch (op) {
    case HYDRA_PRODUCT: return ncclProd;
    case HYDRA_MAX: return ncclMax;
    case HYDRA_MIN: return ncclMin;
  }
  return ncclSum;
}

int check_plan_args(int algo, int op, int dtype, int flags, size_t* esize) {
  *esize = hydra::dtype_size(dtype);
  if (!*esize) return fail(HYDRA_ERR_INVALID, "invalid dtype");
  if (op < HYDRA_SUM || op > HYDRA_MIN) return fail(HYDRA_ERR_INVALID, "invalid op");
  if (algo < HYDRA_ALGO_AUTO || algo > HYDRA_ALGO_RCCL_RS_AG)
    return fail(HYDRA_ERR_INVALID, "invalid algorithm");
  if (flags & HYDRA_ACC_F32) {
    if (dtype != HYDRA_BFLOAT16)
      return fail(HYDRA_ERR_UNSUPPORTED, "HYDRA_ACC_F32 needs a bf16 bucket");
    if (algo == HYDRA_ALGO_RING || algo == HYDRA_ALGO_RING_OLD ||
        algo == HYDRA_ALGO_RING_CHUNKED || algo == HYDRA_ALGO_BCUBE ||
        algo == HYDRA_ALGO_HALVING_DOUBLING)
      return fail(HYDRA_ERR_UNSUPPORTED, "HYDRA_ACC_F32 runs on the DIRECT/A2A algorithms");
  }
  return HYDRA_OK;
}

// HYDRA_ALGO_AUTO: A2A when the reference geometry gives P equal blocks (three launches per
// allreduce -- ncclAllToAll, one fold, ncclAllGather -- so the host enqueue is independent of the
// bucket size), else DIRECT.  Both are bit-identical to the reference ring.
int resolve_algo(int algo, int P, size_t n, size_t es, size_t max_segment) {
  if (algo != HYDRA_ALGO_AUTO) return algo;
  const hydra::PlanGeom g =
      hydra::make_geom(P, n, es, max_segment ? max_segment : (1u << 20), 0);
  return P > 1 && hydra::blocks_equal(g) ? HYDRA_ALGO_A2A : HYDRA_ALGO_DIRECT;
}

int check_geometry(int algo, const hydra::PlanGeom& g) {
  if (algo == HYDRA_ALGO_A2A && !hydra::blocks_equal(g))
    return fail(HYDRA_ERR_UNSUPPORTED,
                "A2A needs equal blocks (n*esize a multiple of P*S*segmentBytes)");
  return HYDRA_OK;
}

// ops that another op waits on need an event
std::vector<char> waited_set(const std::vector<hydra::PlanOp>& ops) {
  std::vector<char> w(ops.size(), 0);
  for (const auto& o : ops) {
    if (o.wait0 >= 0) w[o.wait0] = 1;
    if (o.wait1 >= 0) w[o.wait1] = 1;
  }
  return w;
}

hipError_t launch_compute(const hydra::PlanOp& o, int op, int dtype, bool acc32, char* user,
                          char* scratch, size_t esize, hipStream_t st) {
  if (o.kind == hydra::kOpReduce)
    return hydra::launch_reduce(0, op, dtype, user + o.off, user + o.off, scratch + o.src_off,
                                (size_t)o.bytes / esize, st);
  const void* srcs[hydra::kMaxRanks];
  srcs[0] = user + o.off;
  for (int j = 1; j < o.nsrc; j++) srcs[j] = scratch + hydra::fold_slot(o, j);
  return hydra::launch_fold(op, dtype, acc32, user + o.off, srcs, o.nsrc, (size_t)o.bytes / esize,
                            st);
}

// Every access of a plan must stay inside the rank's user bucket (buf_bytes) and scratch
// (scratch_bytes): a bad plan fails here with HYDRA_ERR_INVALID instead of faulting the GPU.
// One check for all three executors (RCCL, simulator, the run_plan test hook).
int validate_plan(const std::vector<hydra::PlanOp>& plan, int nranks, size_t es, size_t buf_bytes,
                  size_t scratch_bytes) {
  auto inside = [](int64_t off, int64_t len, size_t cap) {
    return off >= 0 && len >= 0 && (size_t)off <= cap && (size_t)len <= cap - (size_t)off;
  };
  bool open = false;  // a SEND/RECV not yet closed by a GROUP
  for (size_t i = 0; i < plan.size(); i++) {
    const hydra::PlanOp& o = plan[i];
    if (o.wait0 >= (int)i || o.wait1 >= (int)i)
      return fail(HYDRA_ERR_INVALID, "plan: wait on a later op");
    if (o.wait0 < -1 || o.wait1 < -1) return fail(HYDRA_ERR_INVALID, "plan: bad wait index");
    switch (o.kind) {
      case hydra::kOpSend:
      case hydra::kOpRecv: {
        if (o.buf != hydra::kBufUser && o.buf != hydra::kBufScratch)
          return fail(HYDRA_ERR_INVALID, "plan: bad p2p buffer");
        const size_t cap = o.buf == hydra::kBufUser ? buf_bytes : scratch_bytes;
        if (o.peer < 0 || o.peer >= nranks || !inside(o.off, o.bytes, cap))
          return fail(HYDRA_ERR_INVALID, "plan: bad p2p op");
        open = true;
        break;
      }
      case hydra::kOpGroup:
        open = false;
        break;
      case hydra::kOpReduce:
        if (open) return fail(HYDRA_ERR_INVALID, "plan: compute op inside a p2p group");
        if (o.bytes % (int64_t)es || !inside(o.off, o.bytes, buf_bytes) ||
            !inside(o.src_off, o.bytes, scratch_bytes))
          return fail(HYDRA_ERR_INVALID, "plan: bad reduce");
        break;
      case hydra::kOpFold:
        if (open) return fail(HYDRA_ERR_INVALID, "plan: compute op inside a p2p group");
        if (o.nsrc < 1 || o.nsrc > hydra::kMaxRanks || o.bytes % (int64_t)es ||
            !inside(o.off, o.bytes, buf_bytes))
          return fail(HYDRA_ERR_INVALID, "plan: bad fold");
        for (int j = 1; j < o.nsrc; j++)
          if (!inside(hydra::fold_slot(o, j), o.bytes, scratch_bytes))
            return fail(HYDRA_ERR_INVALID, "plan: fold slot outside scratch");
        break;
      case hydra::kOpAllToAll:
        if (open) return fail(HYDRA_ERR_INVALID, "plan: collective inside a p2p group");
        if (o.bytes < 0 || !inside(o.off, o.bytes * nranks, buf_bytes) ||
            !inside(o.src_off, o.bytes * nranks, scratch_bytes))
          return fail(HYDRA_ERR_INVALID, "plan: bad all-to-all");
        break;
      case hydra::kOpAllGather:
        if (open) return fail(HYDRA_ERR_INVALID, "plan: collective inside a p2p group");
        if (o.bytes < 0 || !inside(o.off, o.bytes * nranks, buf_bytes))
          return fail(HYDRA_ERR_INVALID, "plan: bad all-gather");
        break;
      default:
        return fail(HYDRA_ERR_INVALID, "plan: unknown op kind");
    }
  }
  if (open) return fail(HYDRA_ERR_INVALID, "plan: unterminated p2p group");
  return HYDRA_OK;
}

}  // namespace

// ---- communicator ----------------------------------------------------------------------------
struct hydra_comm {
  int rank = 0, nranks = 1, device = 0;
  bool aborted = false;  // hydra_comm_wait timed out: nccl was aborted
  // the end of the last EAGER call's folds on ks (ev_mark, recorded only outside a capture, so a
  // captured call in between never clears it: ADVICE r05)
  bool marked = false;
  ncclComm_t nccl = nullptr;
  hipStream_t cs = nullptr, ks = nullptr;  // comm stream, compute stream
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  std::vector<hipEvent_t> events;
  hipEvent_t ev_start = nullptr, ev_cs = nullptr, ev_ks = nullptr, ev_mark = nullptr;
  // plan cache
  int key_algo = -1;
  size_t key_n = 0, key_es = 0, key_ms = 0, key_chunk = 0;
  int key_root = -1;
  std::vector<hydra::PlanOp> plan;
  std::vector<char> waited;
  // per-phase timing (hydra_comm_profile): timing events around every op, read back lazily
  struct ProfRec {
    bool comm;
    hipEvent_t s, e;
    uint64_t sent, recv, hbm;
  };
  struct ProfCall {
    hipEvent_t t0;
    std::vector<ProfRec> ops;
  };
  bool profile = false;
  bool prof_active = false;  // the call being enqueued is recorded
  std::vector<ProfCall> prof_calls;
  std::vector<hipEvent_t> prof_pool;  // timing events (created on `device`)
  hydra_comm_phases_t prof{};
  std::set<int> prof_peers;
};

namespace {

int ensure_events(hydra_comm* c, size_t n) {
  while (c->events.size() < n) {
    hipEvent_t e;
    HIP_TRY(hydra::cached_event(c->device, &e));  // the communicator's device, not the caller's
    c->events.push_back(e);
  }
  return HYDRA_OK;
}

// ---- phase profiling -------------------------------------------------------------------------
hipError_t prof_event(hydra_comm* c, hipEvent_t* out) {
  if (!c->prof_pool.empty()) {
    *out = c->prof_pool.back();
    c->prof_pool.pop_back();
    return hipSuccess;
  }
  return hipEventCreate(out);  // timing enabled; the caller holds a DeviceScope(c->device)
}

// Opens a profiled call: its start on the caller's stream.  No-op unless profiling is on; at
// most kProfMaxCalls calls are held until hydra_comm_phases reads them (later ones go unrecorded,
// so a caller that never reads cannot grow the event pool without bound).
constexpr size_t kProfMaxCalls = 256;
int prof_begin(hydra_comm* c, hipStream_t user_st) {
  c->prof_active = c->profile && c->prof_calls.size() < kProfMaxCalls;
  if (!c->prof_active) return HYDRA_OK;
  hydra_comm::ProfCall call{};
  HIP_TRY(prof_event(c, &call.t0));
  if (hipError_t e = hipEventRecord(call.t0, user_st); e != hipSuccess) {
    c->prof_pool.push_back(call.t0);  // never recorded: back to the pool
    c->prof_active = false;
    return hydra::hip_fail(e, "hipEventRecord (profiled call start)");
  }
  c->prof_calls.push_back(std::move(call));
  return HYDRA_OK;
}

// Brackets one op: `start` recorded before it is enqueued on st, the end after.
struct ProfOp {
  hydra_comm* c;
  hipStream_t st;
  hydra_comm::ProfRec r{};
  bool on = false;
  ProfOp(hydra_comm* c_, hipStream_t st_, bool comm, uint64_t sent, uint64_t recv, uint64_t hbm)
      : c(c_), st(st_) {
    if (!c->profile || !c->prof_active || c->prof_calls.empty()) return;
    r.comm = comm;
    r.sent = sent;
    r.recv = recv;
    r.hbm = hbm;
    if (prof_event(c, &r.s) != hipSuccess) return;
    on = hipEventRecord(r.s, st) == hipSuccess;
    if (!on) c->prof_pool.push_back(r.s);
  }
  // an op that returned before end() (a failed enqueue): its start event is not in any profiled
  // call, so it goes back to the pool rather than leaking
  ~ProfOp() {
    if (on) c->prof_pool.push_back(r.s);
  }
  ProfOp(const ProfOp&) = delete;
  ProfOp& operator=(const ProfOp&) = delete;
  hipError_t end() {
    if (!on) return hipSuccess;
    on = false;
    hipError_t e = prof_event(c, &r.e);
    if (e != hipSuccess) {
      c->prof_pool.push_back(r.s);
      return e;
    }
    e = hipEventRecord(r.e, st);
    if (e == hipSuccess) {
      c->prof_calls.back().ops.push_back(r);
    } else {
      c->prof_pool.push_back(r.s);
      c->prof_pool.push_back(r.e);
    }
    return e;
  }
};

// Reads back every finished profiled call into the totals and recycles its events.  A call is
// read whole before anything of it is counted or recycled: on an error it stays (with the calls
// after it) in prof_calls, so no event is ever both pending and pooled (teardown destroys each
// once).
int prof_collect(hydra_comm* c) {
  std::vector<hydra_comm::ProfCall> calls;
  calls.swap(c->prof_calls);
  for (size_t i = 0; i < calls.size(); i++) {
    const hydra_comm::ProfCall& call = calls[i];
    std::vector<std::pair<float, float>> t(call.ops.size());  // (duration, end after t0)
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < call.ops.size() && e == hipSuccess; k++) {
      const hydra_comm::ProfRec& r = call.ops[k];
      e = hipEventSynchronize(r.e);
      if (e == hipSuccess) e = hipEventElapsedTime(&t[k].first, r.s, r.e);
      if (e == hipSuccess) e = hipEventElapsedTime(&t[k].second, call.t0, r.e);
    }
    if (e != hipSuccess) {
      c->prof_calls.assign(std::make_move_iterator(calls.begin() + i),
                           std::make_move_iterator(calls.end()));
      return hydra::hip_fail(e, "hydra_comm_phases: reading a profiled call's events");
    }
    float last = 0.f;
    for (size_t k = 0; k < call.ops.size(); k++) {
      const hydra_comm::ProfRec& r = call.ops[k];
      (r.comm ? c->prof.link_ms : c->prof.fold_ms) += t[k].first;
      (r.comm ? c->prof.link_ops : c->prof.fold_ops) += 1;
      c->prof.sent_bytes += r.sent;
      c->prof.recv_bytes += r.recv;
      c->prof.fold_hbm_bytes += r.hbm;
      last = std::max(last, t[k].second);
      c->prof_pool.push_back(r.s);
      c->prof_pool.push_back(r.e);
    }
    c->prof.span_ms += last;
    c->prof.calls += 1;
    c->prof_pool.push_back(call.t0);
  }
  c->prof.peers = (int32_t)c->prof_peers.size();
  return HYDRA_OK;
}

// Enqueueing a multi-rank schedule while the caller's stream is being captured: refused unless
// the caller opted in (HYDRA_ALLOW_CAPTURE).  RCCL's own collectives segfault in
// hipStreamEndCapture on the socket-linked ranks of the test box.
int capture_guard(const hydra_comm* c, int flags, hipStream_t st) {
  if (c->nranks <= 1 || (flags & HYDRA_ALLOW_CAPTURE)) return HYDRA_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(st, &cs));
  if (cs != hipStreamCaptureStatusNone)
    return fail(HYDRA_ERR_UNSUPPORTED,
                "multi-rank allreduce under hipGraph capture: ending the capture of RCCL's own "
                "collectives segfaulted on this transport (profiles/r03g2_graph_ranks_rccl.log); "
                "pass HYDRA_ALLOW_CAPTURE on a node whose RCCL captures");
  return HYDRA_OK;
}

// Which executor stream an op runs on: p2p groups and collectives on the comm stream, the
// fused reductions on the compute stream.
bool on_comm_stream(int32_t kind) {
  return kind != hydra::kOpReduce && kind != hydra::kOpFold;
}

// Cross-stream edges only: an op waiting on an earlier op of its OWN stream is already
// ordered behind it, and HIP graph capture faults on a wait for an event recorded on the
// capturing stream itself (scripts/probe_graph.py "fold_wait").
void wait_on(hipStream_t st, const hydra::PlanOp& o, const std::vector<hydra::PlanOp>& ops,
             const std::vector<hipEvent_t>& ev) {
  const bool comm = on_comm_stream(o.kind);
  for (int32_t w : {o.wait0, o.wait1})
    if (w >= 0 && on_comm_stream(ops[w].kind) != comm) (void)hipStreamWaitEvent(st, ev[w], 0);
}

// Enqueue the cached plan after `start` (recorded on the caller's stream); the caller joins
// with join_streams().  Two communicators forked from one event run concurrently (apipe).
int run_plan_rccl(hydra_comm* c, int op, int dtype, bool acc32, char* user, hipEvent_t start,
                  hipStream_t user_st) {
  const auto& ops = c->plan;
  const size_t es = hydra::dtype_size(dtype);
  char* scratch = static_cast<char*>(c->scratch);
  HIP_TRY(hipStreamWaitEvent(c->cs, start, 0));
  HIP_TRY(hipStreamWaitEvent(c->ks, start, 0));
  // The scratch belongs to the communicator: this call's first receive into it (comm stream)
  // must not overtake the previous call's folds still reading it (compute stream, ended by
  // ev_ks) -- also when the caller issues consecutive calls on different streams, which the
  // join onto one caller stream would otherwise be the only thing to order.  (Not under
  // capture: a captured graph orders its own nodes, and may not wait on an outside event.)
  hipStreamCaptureStatus cs_state = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(user_st, &cs_state));
  const bool capturing = cs_state != hipStreamCaptureStatusNone;
  if (c->marked && !capturing) HIP_TRY(hipStreamWaitEvent(c->cs, c->ev_mark, 0));
  size_t i = 0;
  while (i < ops.size()) {
    const hydra::PlanOp& o = ops[i];
    if (o.kind == hydra::kOpAllToAll || o.kind == hydra::kOpAllGather) {
      wait_on(c->cs, o, ops, c->events);
      const uint64_t off_rank = (uint64_t)o.bytes * (uint64_t)(c->nranks - 1);
      if (c->profile)
        for (int q = 0; q < c->nranks; q++)
          if (q != c->rank) c->prof_peers.insert(q);
      ProfOp pr(c, c->cs, true, off_rank, off_rank, 0);
      if (o.kind == hydra::kOpAllToAll)
        NCCL_TRY(ncclAllToAll(user + o.off, scratch + o.src_off, (size_t)o.bytes, ncclUint8,
                              c->nccl, c->cs));
      else
        NCCL_TRY(ncclAllGather(user + o.off + (int64_t)c->rank * o.bytes, user + o.off,
                               (size_t)o.bytes, ncclUint8, c->nccl, c->cs));
      HIP_TRY(pr.end());
      if (c->waited[i]) HIP_TRY(hipEventRecord(c->events[i], c->cs));
      i++;
      continue;
    }
    if (o.kind == hydra::kOpSend || o.kind == hydra::kOpRecv || o.kind == hydra::kOpGroup) {
      size_t g = i;
      while (g < ops.size() && ops[g].kind != hydra::kOpGroup) g++;
      if (g == ops.size()) return fail(HYDRA_ERR_INVALID, "plan: unterminated p2p group");
      wait_on(c->cs, ops[g], ops, c->events);
      uint64_t sent = 0, recv = 0;
      for (size_t j = i; j < g; j++) {
        if (ops[j].kind == hydra::kOpSend) {
          sent += (uint64_t)ops[j].bytes;
          if (c->profile) c->prof_peers.insert(ops[j].peer);
        } else {
          recv += (uint64_t)ops[j].bytes;
        }
      }
      ProfOp pr(c, c->cs, true, sent, recv, 0);
      NCCL_TRY(ncclGroupStart());
      ncclResult_t r = ncclSuccess;
      for (size_t j = i; j < g && r == ncclSuccess; j++) {
        const hydra::PlanOp& p = ops[j];
        char* base = (p.buf == hydra::kBufUser ? user : scratch) + p.off;
        r = p.kind == hydra::kOpSend
                ? ncclSend(base, (size_t)p.bytes, ncclUint8, p.peer, c->nccl, c->cs)
                : ncclRecv(base, (size_t)p.bytes, ncclUint8, p.peer, c->nccl, c->cs);
      }
      const ncclResult_t e = ncclGroupEnd();  // always close the group, even after a failure
      if (r != ncclSuccess) return nccl_fail(r, "ncclSend/ncclRecv");
      if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
      HIP_TRY(pr.end());
      if (c->waited[g]) HIP_TRY(hipEventRecord(c->events[g], c->cs));
      i = g + 1;
    } else {
      wait_on(c->ks, o, ops, c->events);
      const uint64_t hbm = (uint64_t)o.bytes * (o.kind == hydra::kOpReduce ? 3u : (uint64_t)o.nsrc + 1);
      ProfOp pr(c, c->ks, false, 0, 0, hbm);
      hipError_t e = launch_compute(o, op, dtype, acc32, user, scratch, es, c->ks);
      if (e != hipSuccess) return hydra::hip_fail(e, "fused reduction kernel");
      HIP_TRY(pr.end());
      if (c->waited[i]) HIP_TRY(hipEventRecord(c->events[i], c->ks));
      i++;
    }
  }
  HIP_TRY(hipEventRecord(c->ev_cs, c->cs));
  HIP_TRY(hipEventRecord(c->ev_ks, c->ks));
  if (!capturing) {  // (an event recorded inside a capture is a graph node, not a marker)
    HIP_TRY(hipEventRecord(c->ev_mark, c->ks));
    c->marked = true;
  }
  return HYDRA_OK;
}

int join_streams(hydra_comm* c, hipStream_t user_st) {
  HIP_TRY(hipStreamWaitEvent(user_st, c->ev_cs, 0));
  HIP_TRY(hipStreamWaitEvent(user_st, c->ev_ks, 0));
  return HYDRA_OK;
}

}  // namespace

extern "C" {

int hydra_comm_get_unique_id(void* id) {
  if (!id) return fail(HYDRA_ERR_INVALID, "null id");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return ok();
}

int hydra_comm_init(hydra_comm_t* out, int nranks, int rank, const void* id, int device) {
  if (!out || !id) return fail(HYDRA_ERR_INVALID, "null argument");
  if (nranks < 1 || nranks > hydra::kMaxRanks || rank < 0 || rank >= nranks)
    return fail(HYDRA_ERR_INVALID, "bad rank/nranks");
  *out = nullptr;
  hydra::DeviceScope ds(device);  // RCCL binds the communicator to the current device
  HIP_TRY(ds.err);
  auto* c = new hydra_comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  hipError_t e = hydra::cached_stream(device, &c->cs);
  if (e == hipSuccess) e = hydra::cached_stream(device, &c->ks);
  if (e == hipSuccess) e = hydra::cached_event(device, &c->ev_start);
  if (e == hipSuccess) e = hydra::cached_event(device, &c->ev_cs);
  if (e == hipSuccess) e = hydra::cached_event(device, &c->ev_ks);
  if (e == hipSuccess) e = hydra::cached_event(device, &c->ev_mark);
  if (e != hipSuccess) {
    hydra_comm_destroy(c);
    return hydra::hip_fail(e, "hydra_comm_init streams");
  }
  *out = c;
  return ok();
}

int hydra_comm_wait(hydra_comm_t c, hydra_stream_t stream, int64_t timeout_ms) {
  if (!c) return fail(HYDRA_ERR_INVALID, "null comm");
  if (c->aborted) return fail(HYDRA_ERR_TIMEOUT, "communicator was aborted by an earlier timeout");
  hydra::DeviceScope ds(c->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; spin++) {
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) return ok();
    if (q != hipErrorNotReady) return hydra::hip_fail(q, "hipStreamQuery");
    ncclResult_t ae = ncclSuccess;
    NCCL_TRY(ncclCommGetAsyncError(c->nccl, &ae));
    const auto waited = std::chrono::duration_cast<std::chrono::milliseconds>(
                            std::chrono::steady_clock::now() - t0).count();
    if (ae != ncclSuccess || waited > timeout_ms) {
      (void)ncclCommAbort(c->nccl);  // unblocks this rank's RCCL kernels
      c->nccl = nullptr;
      c->aborted = true;
      if (ae != ncclSuccess) return nccl_fail(ae, "RCCL asynchronous error");
      return fail(HYDRA_ERR_TIMEOUT, "Timed out waiting " + std::to_string(timeout_ms) +
                                         "ms for allreduce to complete");
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

int hydra_comm_info(hydra_comm_t c, int* nranks, int* rank, int* device) {
  if (!c || !c->nccl) return fail(HYDRA_ERR_INVALID, "null communicator");
  int cnt = 0, r = 0, d = 0;
  ncclResult_t e = ncclCommCount(c->nccl, &cnt);
  if (e == ncclSuccess) e = ncclCommUserRank(c->nccl, &r);
  if (e == ncclSuccess) e = ncclCommCuDevice(c->nccl, &d);
  if (e != ncclSuccess) return fail(HYDRA_ERR_HIP, std::string("ncclCommCount: ") + ncclGetErrorString(e));
  if (nranks) *nranks = cnt;
  if (rank) *rank = r;
  if (device) *device = d;
  return ok();
}

int hydra_comm_profile(hydra_comm_t c, int enable) {
  if (!c) return fail(HYDRA_ERR_INVALID, "null comm");
  hydra::DeviceScope ds(c->device);
  // recycle what an earlier session left; the switch applies whatever that gives:
  // calls whose events cannot be read are dropped -- after a drain of the communicator's
  // streams, nothing pending records them any more -- so profiling can always be turned off
  const int rc = prof_collect(c);
  if (rc) {
    (void)hipStreamSynchronize(c->cs);
    (void)hipStreamSynchronize(c->ks);
    for (auto& call : c->prof_calls) {
      (void)hipEventDestroy(call.t0);
      for (auto& r : call.ops) {
        (void)hipEventDestroy(r.s);
        (void)hipEventDestroy(r.e);
      }
    }
    c->prof_calls.clear();
  }
  c->profile = enable != 0;
  c->prof_active = false;
  if (c->profile) {
    c->prof = hydra_comm_phases_t{};
    c->prof_peers.clear();
  }
  return rc ? rc : ok();  // (the collection error is still reported, with the switch applied)
}

int hydra_comm_phases(hydra_comm_t c, hydra_comm_phases_t* out) {
  if (!c || !out) return fail(HYDRA_ERR_INVALID, "null argument");
  hydra::DeviceScope ds(c->device);
  if (int rc = prof_collect(c)) return rc;
  *out = c->prof;
  return ok();
}

int hydra_comm_destroy(hydra_comm_t c) {
  if (!c) return ok();
  hydra::DeviceScope ds(c->device);  // the caller's current device is restored on return
  // Drain the DEVICE, not only cs/ks: the caller's stream may still hold waits on ev_cs/ev_ks
  // and on plan events (join_streams), and kernels of an earlier allreduce may still read the
  // scratch freed below.  Destroy is rare; a full drain is the safe order.
  // Every step is checked and the first failure returned (the rest still runs, so nothing
  // leaks): a late-reported device fault then names the teardown step it first
  // shows at, instead of surfacing in the caller's next HIP call.
  int rc = 0;
  auto step = [&rc](hipError_t e, const char* what) {
    if (e != hipSuccess && !rc) rc = hydra::hip_fail(e, what);
  };
  step(hydra::drain_device(c->device), "comm teardown: hipDeviceSynchronize");
  if (c->nccl) {
    ncclResult_t r = ncclCommDestroy(c->nccl);
    if (r != ncclSuccess && !rc)
      rc = fail(HYDRA_ERR_HIP, std::string("comm teardown: ncclCommDestroy: ") +
                                   ncclGetErrorString(r));
  }
  for (auto e : c->events) step(hydra::release_event(e), "comm teardown: release event");
  for (auto e : {c->ev_start, c->ev_cs, c->ev_ks, c->ev_mark})
    if (e) step(hydra::release_event(e), "comm teardown: release event");
  if (c->cs) step(hydra::release_stream(c->cs), "comm teardown: release stream");
  if (c->ks) step(hydra::release_stream(c->ks), "comm teardown: release stream");
  if (c->scratch) step(hydra::cached_free(c->scratch), "comm teardown: release scratch");
  for (auto& call : c->prof_calls) {
    c->prof_pool.push_back(call.t0);
    for (auto& r : call.ops) c->prof_pool.insert(c->prof_pool.end(), {r.s, r.e});
  }
  for (auto e : c->prof_pool) step(hipEventDestroy(e), "comm teardown: destroy timing event");
  step(hydra::drain_device(c->device), "comm teardown: hipDeviceSynchronize after the frees");
  delete c;
  return rc ? rc : ok();
}

}  // extern "C"

namespace {

// Argument checks + plan cache + scratch for one allreduce on `c`.  *skip: nothing to do
// (n == 0 or a single rank, allreduce.cc:129-133).
int prepare(hydra_comm* c, int* algo, int op, int dtype, int flags, void* buf, size_t n,
            size_t max_segment, size_t chunk_bytes, bool* skip, int root = -1) {
  if (!c) return fail(HYDRA_ERR_INVALID, "null comm");
  if (c->aborted) return fail(HYDRA_ERR_TIMEOUT, "communicator was aborted by an earlier timeout");
  size_t es;
  int rc = check_plan_args(*algo, op, dtype, flags, &es);
  if (rc) return rc;
  *skip = n == 0 || c->nranks == 1;
  if (*skip) return HYDRA_OK;
  if (!buf) return fail(HYDRA_ERR_INVALID, "null buffer");
  if (reinterpret_cast<uintptr_t>(buf) % es)
    return fail(HYDRA_ERR_INVALID, "buffer not aligned to the element size");
  *algo = root >= 0 ? *algo : resolve_algo(*algo, c->nranks, n, es, max_segment);
  if (*algo == HYDRA_ALGO_RCCL || *algo == HYDRA_ALGO_RCCL_RS_AG) {
    if (flags & HYDRA_ACC_F32) return fail(HYDRA_ERR_UNSUPPORTED, "ACC_F32 with RCCL");
    if (root >= 0) return fail(HYDRA_ERR_UNSUPPORTED, "RCCL algorithms for gloo::reduce");
    if (*algo == HYDRA_ALGO_RCCL_RS_AG && n % (size_t)c->nranks)
      return fail(HYDRA_ERR_UNSUPPORTED, "RCCL_RS_AG needs n to be a multiple of the rank count");
    return HYDRA_OK;
  }
  const size_t ms = max_segment ? max_segment : (1u << 20);
  if (root >= 0) {  // hydra_reduce_root: DIRECT's arguments, gloo::reduce's plan
    if (root >= c->nranks) return fail(HYDRA_ERR_INVALID, "root out of range");
    *algo = hydra::kAlgoReduce;
  }
  if (c->key_algo != *algo || c->key_n != n || c->key_es != es || c->key_ms != ms ||
      c->key_chunk != chunk_bytes || c->key_root != root) {
    if (root >= 0 && ms < es) return fail(HYDRA_ERR_INVALID, "max_segment below the element size");
    const hydra::PlanGeom g = root >= 0
                                  ? hydra::make_geom_reduce(c->nranks, n, es, ms, chunk_bytes, root)
                                  : hydra::make_geom(c->nranks, n, es, ms, chunk_bytes);
    rc = check_geometry(*algo, g);
    if (rc) return rc;
    std::vector<hydra::PlanOp> plan = hydra::make_plan(*algo, g, c->rank);
    const size_t need = hydra::plan_scratch_bytes(*algo, g);
    rc = validate_plan(plan, c->nranks, es, n * es, need);
    if (rc) return rc;
    c->key_algo = -1;  // invalid until the new plan, its scratch and events are all in place
    c->plan = std::move(plan);
    c->waited = waited_set(c->plan);
    if (need > c->scratch_bytes) {
      // (re)allocation happens outside any capture: first call with a new geometry
      if (c->scratch) HIP_TRY(hydra::cached_free(c->scratch));  // (drains the device first)
      c->scratch = nullptr;
      c->scratch_bytes = 0;
      HIP_TRY(hydra::cached_malloc(c->device, need, &c->scratch));
      c->scratch_bytes = need;
    }
    rc = ensure_events(c, c->plan.size());
    if (rc) return rc;
    c->key_algo = *algo;
    c->key_n = n;
    c->key_es = es;
    c->key_ms = ms;
    c->key_chunk = chunk_bytes;
    c->key_root = root;
  }
  return HYDRA_OK;
}

// Enqueue a prepared allreduce after `start`; ends recorded in c->ev_cs / c->ev_ks.
int enqueue(hydra_comm* c, int algo, int op, int dtype, int flags, void* buf, size_t n,
            hipEvent_t start, hipStream_t user_st) {
  if (algo == HYDRA_ALGO_RCCL_RS_AG) {  // RCCL's own reduce-scatter + all-gather, in place
    HIP_TRY(hipStreamWaitEvent(c->cs, start, 0));
    const size_t es = hydra::dtype_size(dtype), k = n / (size_t)c->nranks;
    char* mine = static_cast<char*>(buf) + (size_t)c->rank * k * es;
    const uint64_t link = (uint64_t)k * es * (c->nranks - 1);
    ProfOp rs(c, c->cs, true, link, link, 0);
    NCCL_TRY(ncclReduceScatter(buf, mine, k, nccl_type(dtype), nccl_op(op), c->nccl, c->cs));
    HIP_TRY(rs.end());
    ProfOp ag(c, c->cs, true, link, link, 0);
    NCCL_TRY(ncclAllGather(mine, buf, k, nccl_type(dtype), c->nccl, c->cs));
    HIP_TRY(ag.end());
    HIP_TRY(hipEventRecord(c->ev_cs, c->cs));
    HIP_TRY(hipEventRecord(c->ev_ks, c->ks));
    return HYDRA_OK;
  }
  if (algo == HYDRA_ALGO_RCCL) {
    HIP_TRY(hipStreamWaitEvent(c->cs, start, 0));
    // (RCCL's own ring: 2(P-1)/P of the bucket leaves this rank; its peers are RCCL's choice)
    const uint64_t link = (uint64_t)n * hydra::dtype_size(dtype) * 2 * (c->nranks - 1) / c->nranks;
    ProfOp pr(c, c->cs, true, link, link, 0);
    NCCL_TRY(ncclAllReduce(buf, buf, n, nccl_type(dtype), nccl_op(op), c->nccl, c->cs));
    HIP_TRY(pr.end());
    HIP_TRY(hipEventRecord(c->ev_cs, c->cs));
    HIP_TRY(hipEventRecord(c->ev_ks, c->ks));
    return HYDRA_OK;
  }
  return run_plan_rccl(c, op, dtype, (flags & HYDRA_ACC_F32) != 0, static_cast<char*>(buf), start,
                       user_st);
}

}  // namespace

extern "C" {

int hydra_allreduce(hydra_comm_t c, int algo, int op, int dtype, int flags, void* buf, size_t n,
                    size_t max_segment, size_t chunk_bytes, hydra_stream_t stream) {
  hydra::TraceRange trace_("hydra_allreduce");
  hydra::DeviceScope ds(c ? c->device : -1);  // the communicator's device, restored on return
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = HYDRA_OK;
  // before prepare: nothing (not even a first scratch allocation) happens under a refused capture
  if (c && n && (rc = capture_guard(c, flags, st))) return rc;
  bool skip = false;
  rc = prepare(c, &algo, op, dtype, flags, buf, n, max_segment, chunk_bytes, &skip);
  if (rc || skip) return rc ? rc : ok();
  if ((rc = prof_begin(c, st))) return rc;
  HIP_TRY(hipEventRecord(c->ev_start, st));
  rc = enqueue(c, algo, op, dtype, flags, buf, n, c->ev_start, st);
  if (rc) return rc;
  rc = join_streams(c, st);
  return rc ? rc : ok();
}

// gloo::reduce (reduce.cc:21-262) of a device bucket to `root`, in place: plan_reduce.
int hydra_reduce_root(hydra_comm_t c, int root, int op, int dtype, int flags, void* buf,
                      size_t n, size_t max_segment, size_t chunk_bytes, hydra_stream_t stream) {
  hydra::TraceRange trace_("hydra_reduce_root");
  // checked before the single-rank / empty short cuts, as the reference does (reduce.cc:31)
  if (root < 0 || (c && root >= c->nranks)) return fail(HYDRA_ERR_INVALID, "root out of range");
  hydra::DeviceScope ds(c ? c->device : -1);
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = HYDRA_OK;
  if (c && n && (rc = capture_guard(c, flags, st))) return rc;
  int algo = HYDRA_ALGO_DIRECT;
  bool skip = false;
  rc = prepare(c, &algo, op, dtype, flags, buf, n, max_segment, chunk_bytes, &skip, root);
  if (rc || skip) return rc ? rc : ok();
  if ((rc = prof_begin(c, st))) return rc;
  HIP_TRY(hipEventRecord(c->ev_start, st));
  rc = enqueue(c, algo, op, dtype, flags, buf, n, c->ev_start, st);
  if (rc) return rc;
  rc = join_streams(c, st);
  return rc ? rc : ok();
}

void hydra_split_elements(int table, int P, size_t n, size_t* e1, size_t* e2) {
  size_t a = 0, b = 0;
  hydra::split_elements(table, P, n, &a, &b);
  if (e1) *e1 = a;
  if (e2) *e2 = b;
}

int hydra_apipe_allreduce(hydra_comm_t rail1, hydra_comm_t rail2, int table, int algo, int op,
                          int dtype, int flags, void* buf, size_t n, size_t max_segment,
                          size_t chunk_bytes, hydra_stream_t stream) {
  hydra::TraceRange trace_("hydra_apipe_allreduce");
  if (!rail1 || !rail2 || rail1 == rail2)
    return fail(HYDRA_ERR_INVALID, "apipe needs two distinct communicators");
  if (rail1->rank != rail2->rank || rail1->nranks != rail2->nranks ||
      rail1->device != rail2->device)
    return fail(HYDRA_ERR_INVALID, "rails disagree on rank/nranks/device");
  if (table != HYDRA_SPLIT_AA && table != HYDRA_SPLIT_AG)
    return fail(HYDRA_ERR_INVALID, "invalid split table");
  const size_t es = hydra::dtype_size(dtype);
  if (!es) return fail(HYDRA_ERR_INVALID, "invalid dtype");
  size_t e1 = 0, e2 = 0;
  hydra::split_elements(table, rail1->nranks, n, &e1, &e2);
  char* p2 = static_cast<char*>(buf) + e1 * es;
  // one part empty: a single allreduce, as apipe_allreduce does (pipeallreduce-a.cc:51-57)
  if (e1 == 0 && e2 != 0)
    return hydra_allreduce(rail2, algo, op, dtype, flags, p2, e2, max_segment, chunk_bytes, stream);
  if (e2 == 0)
    return hydra_allreduce(rail1, algo, op, dtype, flags, buf, e1, max_segment, chunk_bytes,
                           stream);
  hydra::DeviceScope ds(rail1->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  int rc = capture_guard(rail1, flags, st);
  if (rc) return rc;
  int a1 = algo, a2 = algo;
  bool s1 = false, s2 = false;
  rc = prepare(rail1, &a1, op, dtype, flags, buf, e1, max_segment, chunk_bytes, &s1);
  if (!rc) rc = prepare(rail2, &a2, op, dtype, flags, p2, e2, max_segment, chunk_bytes, &s2);
  if (rc) return rc;
  if (s1 && s2) return ok();  // single rank
  if ((rc = prof_begin(rail1, st)) || (rc = prof_begin(rail2, st))) return rc;
  // both rails fork from one event on the caller's stream and run concurrently on their own
  // streams (the two std::threads of pipeallreduce-a.cc:32-50); the caller's stream joins both
  HIP_TRY(hipEventRecord(rail1->ev_start, st));
  rc = enqueue(rail1, a1, op, dtype, flags, buf, e1, rail1->ev_start, st);
  if (!rc) rc = enqueue(rail2, a2, op, dtype, flags, p2, e2, rail1->ev_start, st);
  if (!rc) rc = join_streams(rail1, st);
  if (!rc) rc = join_streams(rail2, st);
  return rc ? rc : ok();
}

namespace {
int plan_impl(int algo, int root, int P, int rank, size_t n, size_t esize, size_t max_segment,
              size_t chunk_bytes, hydra_plan_op_t* ops, size_t cap, size_t* count,
              size_t* scratch_bytes) {
  if (P < 1 || P > hydra::kMaxRanks || rank < 0 || rank >= P)
    return fail(HYDRA_ERR_INVALID, "bad rank/P");
  if (esize != 1 && esize != 2 && esize != 4 && esize != 8)
    return fail(HYDRA_ERR_INVALID, "bad element size");
  if (root >= P) return fail(HYDRA_ERR_INVALID, "root out of range");
  algo = root >= 0 ? hydra::kAlgoReduce : resolve_algo(algo, P, n, esize, max_segment);
  if (algo == HYDRA_ALGO_RCCL || algo == HYDRA_ALGO_RCCL_RS_AG)
    return fail(HYDRA_ERR_UNSUPPORTED, "RCCL has no plan");
  const size_t ms = max_segment ? max_segment : (1u << 20);
  if (root >= 0 && ms < esize) return fail(HYDRA_ERR_INVALID, "max_segment below the element size");
  const hydra::PlanGeom g = root >= 0 ? hydra::make_geom_reduce(P, n, esize, ms, chunk_bytes, root)
                                      : hydra::make_geom(P, n, esize, ms, chunk_bytes);
  if (int rc = check_geometry(algo, g)) return rc;
  const auto plan = hydra::make_plan(algo, g, rank);
  const size_t sbytes = hydra::plan_scratch_bytes(algo, g);
  // the library's own plans pass the executors' bounds check (CPU-testable, tests/test_plan.py)
  if (int rc = validate_plan(plan, P, esize, n * esize, sbytes)) return rc;
  if (count) *count = plan.size();
  if (scratch_bytes) *scratch_bytes = sbytes;
  if (ops) {
    static_assert(sizeof(hydra_plan_op_t) == sizeof(hydra::PlanOp), "layout");
    const size_t k = plan.size() < cap ? plan.size() : cap;
    std::memcpy(ops, plan.data(), k * sizeof(hydra::PlanOp));
  }
  return ok();
}
}  // namespace

int hydra_plan(int algo, int P, int rank, size_t n, size_t esize, size_t max_segment,
               size_t chunk_bytes, hydra_plan_op_t* ops, size_t cap, size_t* count,
               size_t* scratch_bytes) {
  return plan_impl(algo, -1, P, rank, n, esize, max_segment, chunk_bytes, ops, cap, count,
                   scratch_bytes);
}

int hydra_reduce_root_plan(int root, int P, int rank, size_t n, size_t esize, size_t max_segment,
                           size_t chunk_bytes, hydra_plan_op_t* ops, size_t cap, size_t* count,
                           size_t* scratch_bytes) {
  if (root < 0) return fail(HYDRA_ERR_INVALID, "root out of range");
  return plan_impl(HYDRA_ALGO_DIRECT, root, P, rank, n, esize, max_segment, chunk_bytes, ops, cap,
                   count, scratch_bytes);
}

// ---- one-GPU simulation of P ranks ---------------------------------------------------------
// Every rank's plan runs on ONE GPU with the real kernels: REDUCE/FOLD launch the gfx950 kernels,
// a matched SEND/RECV pair is a device copy, a collective is the copies it implies.  The ranks
// advance in lock-step (a rank stalls at a p2p group until every peer has posted its side) and
// everything is enqueued on ONE stream in that discovery order, which is a sequentially
// consistent execution of the schedule: a copy is enqueued only after both ranks enqueued every
// op before their group, and a rank's later ops only after its group's copies.  No events and
// no cross-stream waits: the simulator checks the kernels and the data movement; the plans'
// cross-stream edges are checked by the RCCL executor (hydra_comm_run_plan) and the CPU race
// checker (tests/test_plan.py).  (Round 1 ran 2P+1 streams with per-op events here; three
// intermittent device faults surfaced only after syncs that had returned success -- DESIGN.md
// 10.  One stream keeps the HIP runtime out of the picture.)
namespace {
int simulate_impl(int algo, int root, int op, int dtype, int flags, int P, void** bufs, size_t n,
                  size_t max_segment, size_t chunk_bytes) {
  size_t es;
  int rc = check_plan_args(algo, op, dtype, flags, &es);
  if (rc) return rc;
  if (P < 1 || P > hydra::kMaxRanks || !bufs) return fail(HYDRA_ERR_INVALID, "bad P/bufs");
  if (root >= P) return fail(HYDRA_ERR_INVALID, "root out of range");
  algo = root >= 0 ? hydra::kAlgoReduce : resolve_algo(algo, P, n, es, max_segment);
  if (algo == HYDRA_ALGO_RCCL || algo == HYDRA_ALGO_RCCL_RS_AG)
    return fail(HYDRA_ERR_UNSUPPORTED, "no RCCL in the simulator");
  if (n == 0 || P == 1) return ok();
  const bool acc32 = (flags & HYDRA_ACC_F32) != 0;
  const size_t ms = max_segment ? max_segment : (1u << 20);
  if (root >= 0 && ms < es) return fail(HYDRA_ERR_INVALID, "max_segment below the element size");
  const hydra::PlanGeom g = root >= 0 ? hydra::make_geom_reduce(P, n, es, ms, chunk_bytes, root)
                                      : hydra::make_geom(P, n, es, ms, chunk_bytes);
  rc = check_geometry(algo, g);
  if (rc) return rc;
  const size_t sbytes = hydra::plan_scratch_bytes(algo, g);
  for (int r = 0; r < P; r++)
    if (!bufs[r]) return fail(HYDRA_ERR_INVALID, "null bucket");

  struct Rank {
    std::vector<hydra::PlanOp> ops;
    char* scratch = nullptr;
    size_t pc = 0;
    bool posted = false;
    size_t group_end = 0;
    int outstanding = 0;
    int coll_posted = 0;  // collectives posted so far (sequence number)
  };
  std::vector<Rank> R(P);
  for (int r = 0; r < P; r++) {  // validated before anything is allocated or enqueued
    R[r].ops = hydra::make_plan(algo, g, r);
    rc = validate_plan(R[r].ops, P, es, n * es, sbytes);
    if (rc) return rc;
  }
  int coll_done = 0;  // collectives performed (every rank matched)
  hipStream_t st = nullptr;
  auto cleanup = [&]() {
    (void)hydra::drain_device(-1);
    for (auto& r : R)
      if (r.scratch) (void)hydra::cached_free(r.scratch);
    if (st) (void)hydra::release_stream(st);
  };
#define SIM_TRY(expr)                               \
  do {                                              \
    hipError_t e__ = (expr);                        \
    if (e__ != hipSuccess) {                        \
      int rc__ = hydra::hip_fail(e__, #expr);       \
      cleanup();                                    \
      return rc__;                                  \
    }                                               \
  } while (0)

  SIM_TRY(hydra::drain_device(-1));
  int dev = 0;
  SIM_TRY(hipGetDevice(&dev));
  SIM_TRY(hydra::cached_stream(dev, &st));
  for (int r = 0; r < P; r++)
    if (sbytes) SIM_TRY(hydra::cached_malloc(dev, sbytes, reinterpret_cast<void**>(&R[r].scratch)));
  struct Posted {
    int rank;
    size_t idx;
  };
  std::map<std::pair<int, int>, std::deque<Posted>> sends, recvs;  // key (src, dst)
  auto user = [&](int r) { return static_cast<char*>(bufs[r]); };
  for (;;) {
    bool progress = false, all_done = true;
    for (int r = 0; r < P; r++) {
      Rank& rk = R[r];
      while (rk.pc < rk.ops.size()) {
        const hydra::PlanOp& o = rk.ops[rk.pc];
        if (o.kind == hydra::kOpReduce || o.kind == hydra::kOpFold) {
          SIM_TRY(launch_compute(o, op, dtype, acc32, user(r), rk.scratch, es, st));
          rk.pc++;
          progress = true;
          continue;
        }
        if (o.kind == hydra::kOpAllToAll || o.kind == hydra::kOpAllGather) {
          if (!rk.posted) {  // this rank reached the collective
            rk.posted = true;
            rk.coll_posted++;
            progress = true;
          }
          bool all = true;
          for (int q = 0; q < P; q++) all = all && R[q].coll_posted == coll_done + 1;
          if (all) {  // every rank reached it: perform it
            const int64_t B = o.bytes;
            for (int sr = 0; sr < P; sr++)
              for (int dr = 0; dr < P; dr++) {
                if (o.kind == hydra::kOpAllToAll)
                  SIM_TRY(hipMemcpyAsync(R[dr].scratch + o.src_off + sr * B,
                                         user(sr) + o.off + dr * B, (size_t)B,
                                         hipMemcpyDeviceToDevice, st));
                else if (sr != dr)
                  SIM_TRY(hipMemcpyAsync(user(dr) + o.off + sr * B, user(sr) + o.off + sr * B,
                                         (size_t)B, hipMemcpyDeviceToDevice, st));
              }
            coll_done++;
            progress = true;
          }
          if (rk.posted && rk.coll_posted == coll_done) {  // this rank's collective is done
            rk.posted = false;
            rk.pc++;
            progress = true;
            continue;
          }
          break;  // waiting for the other ranks to reach the collective
        }
        if (!rk.posted) {  // post the whole group
          size_t gi = rk.pc;
          while (gi < rk.ops.size() && rk.ops[gi].kind != hydra::kOpGroup) gi++;
          rk.group_end = gi;  // validate_plan guarantees the group is closed
          rk.outstanding = 0;
          for (size_t j = rk.pc; j < gi; j++) {
            const hydra::PlanOp& p = rk.ops[j];
            if (p.kind == hydra::kOpSend) sends[{r, p.peer}].push_back({r, j});
            else recvs[{p.peer, r}].push_back({r, j});
            rk.outstanding++;
          }
          rk.posted = true;
          progress = true;
          for (auto& kv : sends) {  // match everything now matchable, FIFO per (src, dst)
            auto& sq = kv.second;
            auto& rq = recvs[kv.first];
            while (!sq.empty() && !rq.empty()) {
              Posted s = sq.front(), d = rq.front();
              sq.pop_front();
              rq.pop_front();
              Rank& S = R[s.rank];
              Rank& D = R[d.rank];
              const hydra::PlanOp& so = S.ops[s.idx];
              const hydra::PlanOp& ro = D.ops[d.idx];
              if (so.bytes != ro.bytes) {
                cleanup();
                return fail(HYDRA_ERR_INVALID, "plan: send/recv size mismatch");
              }
              const char* src = (so.buf == hydra::kBufUser ? user(s.rank) : S.scratch) + so.off;
              char* dst = (ro.buf == hydra::kBufUser ? user(d.rank) : D.scratch) + ro.off;
              if (so.bytes)
                SIM_TRY(hipMemcpyAsync(dst, src, (size_t)so.bytes, hipMemcpyDeviceToDevice, st));
              S.outstanding--;
              D.outstanding--;
            }
          }
        }
        if (rk.outstanding == 0) {  // group complete
          rk.pc = rk.group_end + 1;
          rk.posted = false;
          progress = true;
          continue;
        }
        break;  // stalled on peers
      }
      if (rk.pc < rk.ops.size()) all_done = false;
    }
    if (all_done) break;
    if (!progress) {
      cleanup();
      return fail(HYDRA_ERR_INVALID, "plan deadlock in simulation");
    }
  }
  SIM_TRY(hipStreamSynchronize(st));
  SIM_TRY(hipGetLastError());
#undef SIM_TRY
  // Teardown, every step checked: the intermittent late-reported fault has so
  // far surfaced at the first HIP call after a teardown like this one, so a fault reported here
  // names the step it first shows at instead of surfacing in the caller's next call.
  auto step = [](hipError_t e, const char* what) {
    return e == hipSuccess ? 0 : hydra::hip_fail(e, what);
  };
  rc = step(hydra::drain_device(-1), "simulate teardown: hipDeviceSynchronize before the frees");
  for (auto& r : R) {
    if (r.scratch && !rc) rc = step(hydra::cached_free(r.scratch), "simulate teardown: release scratch");
    else if (r.scratch) (void)hydra::cached_free(r.scratch);
    r.scratch = nullptr;
  }
  hipError_t ed = hydra::release_stream(st);
  if (!rc) rc = step(ed, "simulate teardown: release stream");
  if (!rc) rc = step(hydra::drain_device(-1), "simulate teardown: hipDeviceSynchronize after the frees");
  return rc ? rc : ok();
}
}  // namespace

int hydra_allreduce_simulate(int algo, int op, int dtype, int flags, int P, void** bufs, size_t n,
                             size_t max_segment, size_t chunk_bytes) {
  return simulate_impl(algo, -1, op, dtype, flags, P, bufs, n, max_segment, chunk_bytes);
}

int hydra_reduce_root_simulate(int root, int op, int dtype, int flags, int P, void** bufs,
                               size_t n, size_t max_segment, size_t chunk_bytes) {
  if (root < 0) return fail(HYDRA_ERR_INVALID, "root out of range");
  return simulate_impl(HYDRA_ALGO_DIRECT, root, op, dtype, flags, P, bufs, n, max_segment,
                       chunk_bytes);
}

// Executor test hook: run an arbitrary (validated) plan through the RCCL executor.  With a
// 1-rank communicator and every peer remapped to 0, RCCL's send/recv-to-self exercises the real
// executor -- groups, both streams, the event edges -- on one GPU.
int hydra_comm_run_plan(hydra_comm_t c, const hydra_plan_op_t* ops, size_t nops, int op, int dtype,
                        int flags, void* buf, size_t buf_bytes, size_t scratch_bytes,
                        hydra_stream_t stream) {
  if (!c || (!ops && nops)) return fail(HYDRA_ERR_INVALID, "null argument");
  if (c->aborted) return fail(HYDRA_ERR_TIMEOUT, "communicator was aborted by an earlier timeout");
  hydra::DeviceScope ds(c->device);
  size_t es;
  int rc = check_plan_args(HYDRA_ALGO_RING, op, dtype, flags, &es);
  if (rc) return rc;
  if ((rc = capture_guard(c, flags, static_cast<hipStream_t>(stream)))) return rc;
  std::vector<hydra::PlanOp> plan(nops);
  if (nops) std::memcpy(plan.data(), ops, nops * sizeof(hydra::PlanOp));
  // every access must stay inside buf / scratch: a bad plan must fail here, not fault the GPU
  rc = validate_plan(plan, c->nranks, es, buf_bytes, scratch_bytes);
  if (rc) return rc;
  if (scratch_bytes > c->scratch_bytes) {
    if (c->scratch) HIP_TRY(hydra::cached_free(c->scratch));  // (drains the device first)
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    HIP_TRY(hydra::cached_malloc(c->device, scratch_bytes, &c->scratch));
    c->scratch_bytes = scratch_bytes;
  }
  c->plan = std::move(plan);
  c->waited = waited_set(c->plan);
  c->key_algo = -1;  // the plan cache no longer holds a library plan
  rc = ensure_events(c, c->plan.size());
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // deterministic scratch for the hook (slots a 1-rank collective leaves untouched read as 0),
  // after the previous eager call's folds are done reading it (that call may be on another
  // stream)
  if (scratch_bytes) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(hipStreamIsCapturing(st, &cap));
    if (c->marked && cap == hipStreamCaptureStatusNone) HIP_TRY(hipStreamWaitEvent(st, c->ev_mark, 0));
    HIP_TRY(hipMemsetAsync(c->scratch, 0, scratch_bytes, st));
  }
  if ((rc = prof_begin(c, st))) return rc;
  HIP_TRY(hipEventRecord(c->ev_start, st));
  rc = run_plan_rccl(c, op, dtype, (flags & HYDRA_ACC_F32) != 0, static_cast<char*>(buf),
                     c->ev_start, st);
  if (!rc) rc = join_streams(c, st);
  return rc ? rc : ok();
}

// apipe on one GPU: the split, then each non-empty part through the P-rank simulator.
int hydra_apipe_allreduce_simulate(int table, int algo, int op, int dtype, int flags, int P,
                                   void** bufs, size_t n, size_t max_segment, size_t chunk_bytes) {
  if (table != HYDRA_SPLIT_AA && table != HYDRA_SPLIT_AG)
    return fail(HYDRA_ERR_INVALID, "invalid split table");
  const size_t es = hydra::dtype_size(dtype);
  if (!es) return fail(HYDRA_ERR_INVALID, "invalid dtype");
  if (P < 1 || P > hydra::kMaxRanks || !bufs) return fail(HYDRA_ERR_INVALID, "bad P/bufs");
  size_t e1 = 0, e2 = 0;
  hydra::split_elements(table, P, n, &e1, &e2);
  if (e1) {
    int rc = hydra_allreduce_simulate(algo, op, dtype, flags, P, bufs, e1, max_segment,
                                      chunk_bytes);
    if (rc) return rc;
  }
  if (e2) {
    std::vector<void*> b2(P);
    for (int r = 0; r < P; r++) b2[r] = static_cast<char*>(bufs[r]) + e1 * es;
    int rc = hydra_allreduce_simulate(algo, op, dtype, flags, P, b2.data(), e2, max_segment,
                                      chunk_bytes);
    if (rc) return rc;
  }
  return ok();
}

}  // extern "C"
