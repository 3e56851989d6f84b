// resident.h -- the resident reducer: a low-latency form of hydra_reduce_host's one batched
// launch for the synchronous host Func (the reference ring calls it once per arriving segment,
// allreduce.cc:301-305, and waits for it).
//
// A fresh launch costs a dispatch (~4 us of host enqueue, ~2-3 us until the first wave runs)
// plus the completion wait: ~13 us per synchronous call however small.  The
// resident reducer instead keeps kResidentBlocks workgroups of one launch alive on a private
// stream while calls keep coming:
//   * the host writes the call's descriptor (<= kResidentSegs segments, the same split as
//     hydra_reduce_batch) into a host-mapped control block, then rings a doorbell (a sequence
//     number);
//   * wave 0 of workgroup 0 polls the doorbell (system-scope relaxed loads, s_sleep backoff),
//     copies the descriptor into device memory and publishes the sequence number there; the
//     other workgroups poll that device word (agent scope);
//   * every workgroup does a system-scope acquire (the host wrote the operands / staging), sums
//     its share of the tiles, releases its stores at system scope and arrives on a device
//     counter; the last to arrive resets it and writes the sequence number into the host-mapped
//     completion word, on which the host spins.
// Exit: workgroup 0 publishes an exit generation when the doorbell has been idle for the idle
// limit (default 2 ms) or the host sets `quit`; every spin is bounded, so the grid always
// drains.  The kernel clears `alive` (host-mapped) when it leaves; a host that rang while the
// kernel was deciding to leave sees alive == 0 with its call not done and launches a new
// instance on the same stream, which serves the pending doorbell (served < doorbell).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace hydra {

constexpr int kResidentSegs = 16;
constexpr int kResidentBlocks = 32;

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

struct alignas(64) ResHost {  // host-mapped (pinned), written by the host unless noted
  uint64_t doorbell;  // the call's sequence number, written after desc
  uint32_t quit;
  uint32_t pad0[13];
  ResDesc desc;
  alignas(64) uint64_t done;  // written by the kernel: last finished sequence number
  alignas(64) uint32_t alive;  // cleared by the kernel when it leaves
  uint32_t err;                // set by the kernel: 1 = a worker's wait for workgroup 0 expired
};

struct alignas(64) ResDev {  // device memory, zeroed at creation
  uint64_t seq;  // the last multi-workgroup call published: (generation << 40) | sequence
  uint64_t exit_gen;
  uint32_t pad0[12];
  alignas(64) uint32_t arrive;
  alignas(64) ResDesc desc;
};

// Launch one instance (generation `gen`, last served sequence number `served`) on `s`.
hipError_t launch_resident(ResHost* h, ResDev* d, uint64_t served, uint64_t gen,
                           uint64_t idle_ticks, hipStream_t s);

}  // namespace hydra
