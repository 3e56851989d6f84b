// fault_report.h -- diagnostics for a GPU memory fault: WHERE the faulting address lies.
//
// HIP reports a device fault only as hipErrorIllegalAddress at some later API call, and its
// error-level log line carries no address.  hydra_fault_report_enable() installs
// an HSA system-event handler that, on HSA_AMD_GPU_MEMORY_FAULT_EVENT, prints the faulting
// virtual address and reason, the /proc/self/maps line that holds it (a GPU buffer object, an
// anonymous host mapping, or nothing: unmapped), and every range hydra's own ledger knows that
// contains its page: device and pinned blocks the caches allocated, host ranges registered by
// hydra_host_register, pageable operands pinned for one hydra_reduce_host call, peer
// allocations mapped by IPC and peer groups' own blocks -- live or already released (with
// when).  The last fault is kept for hydra_fault_last().
#pragma once

#include <cstddef>

namespace hydra {

enum LedgerKind : int {
  kLedgerDeviceBlock = 1,   // hipMalloc by the block cache
  kLedgerPinnedBlock = 2,   // hipHostMalloc by the block cache
  kLedgerHostRegister = 3,  // hydra_host_register
  kLedgerTempPin = 4,       // (round 2 only: a pageable operand pinned for one call; retired)
  kLedgerPeerMapping = 5,   // a peer's allocation mapped into this process by IPC (hydra_peer_*)
  kLedgerPeerLocal = 6,     // a peer group's own scratch / signal block (hydra_peer_*)
};

void ledger_add(LedgerKind kind, const void* p, size_t bytes);
void ledger_release(LedgerKind kind, const void* p);

}  // namespace hydra
