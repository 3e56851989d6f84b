// resident.h -- the resident reducer: a low-latency form of hydra_reduce_host's batched launch
// for the synchronous host Func (the reference ring calls it once per arriving segment,
// allreduce.cc:301-305, and waits for it).
//
// A fresh launch costs a dispatch (~4 us of host enqueue, ~2-3 us until the first wave runs)
// plus the completion wait: ~15 us per synchronous call however small.  The
// resident reducer instead keeps kResidentBlocks workgroups of one launch alive while calls
// keep coming.  ONE instance per device per process serves every host context:
//   * each context leases a slot of the device's host-mapped control block; a call writes its
//     descriptor (<= kResidentSegs segments, the same split as hydra_reduce_batch) into the
//     slot, then rings the slot's doorbell (the slot's sequence number);
//   * wave 0 of workgroup 0 polls every slot's doorbell at once (lane i loads slot i; system-
//     scope relaxed loads, s_sleep backoff) and serves pending slots round robin;
//   * a call of at most kSoloTiles tiles is summed by workgroup 0 alone; a larger one is copied
//     to device memory and published as a job (a device word tagged with the instance's
//     generation) to as many workgroups as it has pairs of tiles -- each workgroup's system-
//     scope fences cost, so a small job wakes few; each of them acquires at system scope, sums
//     its share, releases at system scope and arrives on a device counter; the last to arrive
//     writes the slot's completion word, on which the host spins;
//   * the instance runs on a non-blocking stream of the greatest priority, whose hardware queue
//     pool ordinary streams (torch's, RCCL's, hydra's own) do not use, so their work never
//     queues behind the persistent grid (tests/test_gpu_resident.py times it).
// Exit: workgroup 0 publishes an exit generation when every doorbell has been idle for the idle
// limit (default 2 ms) or the host sets `quit`; every spin is bounded, so the grid always
// drains.  The kernel clears `alive` (host-mapped) when it leaves; a host that rang while the
// kernel was deciding to leave sees alive == 0 with its call not done and launches a new
// instance on the same stream, which serves the pending doorbells (each slot's done word says
// what was served).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "reduce_kernels.h"

namespace hydra {

constexpr int kResidentSegs = 16;
constexpr int kResidentBlocks = 128;
constexpr int kResidentMaxBlocks = 1024;  // HYDRA_OPT_RESIDENT_BLOCKS's bound (the job word holds nwg)
constexpr int kResidentSlots = 32;  // contexts served at once per device (lanes of wave 0)

struct ResSeg {  // one c = op(a, b): vector body + ragged head / tail, split on c (as the batch)
  char* c;       // at the vector body (16-B aligned)
  const char* a;
  const char* b;
  uint64_t nvec;
  int32_t head, tail;
  uint32_t tile0;  // first tile of this segment in the call
  uint32_t c_old;  // float16 store quirk with c != a: load c's old bits
};

struct ResDesc {
  int32_t op, dtype, count;
  uint32_t tiles;  // total tiles of the call
  ResSeg s[kResidentSegs];
};

struct alignas(128) ResSlot {  // one context's channel (host-mapped)
  uint64_t doorbell;           // host: the slot's sequence number, written after desc
  uint32_t pad0[14];
  ResDesc desc;                // host
  alignas(64) uint64_t done;   // kernel: the slot's last finished sequence number
};

struct alignas(128) ResCtl {  // host-mapped (pinned), one per device
  uint32_t quit;             // host: leave now
  uint32_t pad0[15];
  alignas(64) uint32_t alive;  // host sets it before a launch, the kernel clears it on leaving
  uint32_t err;                // kernel: 1 = a wait inside the grid expired
  alignas(128) ResSlot slot[kResidentSlots];
};

struct ResJob {  // a call spread over workgroups 0 .. nwg-1 (device memory)
  uint64_t seq;
  uint32_t slot, nwg;
  ResDesc desc;
};

struct alignas(64) ResDev {  // device memory, zeroed before every launch (ensure_running)
  uint64_t pub;              // the last job published: tag | workgroups | job number (resident.hip)
  uint64_t exit_gen;
  alignas(64) uint64_t beat;  // workgroup 0's heartbeat: calls served by the running instance
  alignas(64) uint32_t arrive;
  alignas(64) uint64_t finished;  // the last job every workgroup finished (same tagging)
  alignas(64) ResJob job;
};

// The grid's shape (defaults; HYDRA_RESIDENT_SHAPE=blocks,batch,solo,tiles_per_block for A/B):
// `blocks` workgroups; each issues the loads of `batch` tiles (1, 2 or 4) together; a call of at
// most `solo` tiles is served by workgroup 0 alone; a larger job wakes ceil(tiles /
// tiles_per_block) workgroups (each workgroup's system-scope fences cost).
struct ResidentShape {  // defaults from the round-3 A/B (profiles/r03_resident_shape_ab.json)
  int blocks = kResidentBlocks;
  int batch = 4;
  uint32_t solo = 4;
  uint32_t tiles_per_block = 4;
};

// Launch one instance (generation `gen`) on `s`.  idle_ticks: leave after that long without a
// call; grace_ticks: the bound of every wait inside the grid (s_memrealtime ticks, 100 MHz).
hipError_t launch_resident(ResCtl* h, ResDev* d, uint64_t gen, uint64_t idle_ticks,
                           uint64_t grace_ticks, const ResidentShape& shape, hipStream_t s);

// ---- host side (resident_host.cpp) -------------------------------------------------------
// A context's slot on its device's resident reducer.  Calls through one lease are made by one
// thread at a time and are synchronous per round: submit, then wait, then the next submit.
struct ResidentLease;

// A slot of `device`'s reducer, or null when it is off or every slot is leased (the caller
// then launches).  Errors (device setup) are returned as HYDRA codes with the message set.
int resident_lease(int device, ResidentLease** out);
void resident_release(ResidentLease* l);
// Ring the slot with `count` (1..kResidentSegs) segments; makes sure an instance is running.
int resident_submit(ResidentLease* l, int op, int dtype, size_t es, const BatchSegDesc* segs,
                    size_t count);
// Wait until the last submitted call is done (bounded: 20 s, then HYDRA_ERR_TIMEOUT).  On any
// failure the instance is stopped and waited for before returning; *poisoned (if given) is set
// when it could not be confirmed gone -- the caller must then keep every buffer of the call
// mapped (the grid may still touch them), and the server is never used again.
int resident_wait(ResidentLease* l, bool* poisoned = nullptr);
// false once the lease's server was poisoned: the caller launches instead.
bool resident_usable(const ResidentLease* l);
uint64_t resident_calls(const ResidentLease* l);  // calls this lease submitted
uint64_t resident_launches(int device);            // instances launched on the device so far

// Device-wide drains while the reducer is serving.  A persistent grid keeps
// hipDeviceSynchronize -- and every call that synchronises the device implicitly (hipFree,
// hipHostFree, ...) -- waiting for as long as any thread keeps calling.  resident_pause stops the
// device's instance (-1: every device's), waiting a bounded time for it to leave, and holds
// relaunches until the matching resume; a call submitted meanwhile waits in ensure_running and
// is served by the instance launched after the resume.  drain_device = pause + synchronise +
// resume.  Every internal device-wide drain of the library goes through one of these.
void resident_pause(int device);
void resident_resume(int device);
struct ResidentPause {
  int device;
  explicit ResidentPause(int d) : device(d) { resident_pause(d); }
  ~ResidentPause() { resident_resume(device); }
  ResidentPause(const ResidentPause&) = delete;
  ResidentPause& operator=(const ResidentPause&) = delete;
};
hipError_t drain_device(int device);  // -1: the current device

}  // namespace hydra
