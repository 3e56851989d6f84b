// fault_report.cpp -- see fault_report.h.
#include "fault_report.h"

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <chrono>
#include <cinttypes>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "errors.h"
#include "hydra_hip.h"

namespace hydra {
namespace {

constexpr size_t kLedgerSize = 16384;  // ranges remembered, live and released (a ring)
constexpr uint64_t kPage = 4096;

struct Entry {
  uint64_t start = 0, end = 0;  // [start, end) as the caller passed it
  int kind = 0;
  uint64_t seq = 0;
  double t_add = 0, t_rel = -1;  // seconds since the ledger began; t_rel < 0: live
};

struct Ledger {
  std::timed_mutex m;
  std::vector<Entry> ring = std::vector<Entry>(kLedgerSize);
  uint64_t next = 0;
  std::map<std::pair<int, uint64_t>, uint64_t> live;  // (kind, start) -> seq of its entry
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  double now() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
};

Ledger& L() {  // never destroyed (the HSA event thread may still report during exit)
  static Ledger* l = new Ledger;
  return *l;
}

std::atomic<uint64_t> g_fault_va{0};
std::atomic<uint32_t> g_fault_reason{0};
std::atomic<uint64_t> g_fault_count{0};
std::atomic<bool> g_enabled{false};

const char* kind_name(int k) {
  switch (k) {
    case kLedgerDeviceBlock: return "device block (block cache hipMalloc)";
    case kLedgerPinnedBlock: return "pinned block (block cache hipHostMalloc)";
    case kLedgerHostRegister: return "host range registered by hydra_host_register";
    case kLedgerTempPin: return "pageable operand pinned for one hydra_reduce_host call";
    case kLedgerPeerMapping: return "peer allocation mapped by IPC (hydra_peer_*)";
    case kLedgerPeerLocal: return "peer group scratch / signal block (hydra_peer_*)";
  }
  return "?";
}

std::string reasons(uint32_t m) {
  static const std::pair<uint32_t, const char*> names[] = {
      {HSA_AMD_MEMORY_FAULT_PAGE_NOT_PRESENT, "page not present"},
      {HSA_AMD_MEMORY_FAULT_READ_ONLY, "write to read-only page"},
      {HSA_AMD_MEMORY_FAULT_NX, "execute of NX page"},
      {HSA_AMD_MEMORY_FAULT_HOST_ONLY, "host-only page"},
      {HSA_AMD_MEMORY_FAULT_DRAMECC, "DRAM ECC"},
      {HSA_AMD_MEMORY_FAULT_IMPRECISE, "imprecise address"},
      {HSA_AMD_MEMORY_FAULT_SRAMECC, "SRAM ECC"},
      {HSA_AMD_MEMORY_FAULT_HANG, "hang"}};
  std::string s;
  for (auto& n : names)
    if (m & n.first) s += (s.empty() ? "" : ", ") + std::string(n.second);
  return s.empty() ? "none given" : s;
}

// The /proc/self/maps line holding va, or its neighbours when no mapping holds it.
std::string maps_line(uint64_t va) {
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return "  /proc/self/maps: unreadable\n";
  char line[512], prev[512] = "";
  std::string out;
  while (std::fgets(line, sizeof line, f)) {
    uint64_t a = 0, b = 0;
    if (std::sscanf(line, "%" SCNx64 "-%" SCNx64, &a, &b) != 2) continue;
    if (va >= a && va < b) {
      out = "  mapped by: " + std::string(line);
      break;
    }
    if (a > va) {
      out = "  not mapped; between:\n    " + std::string(prev[0] ? prev : "(nothing)\n") +
            "    " + std::string(line);
      break;
    }
    std::strncpy(prev, line, sizeof prev - 1);
  }
  std::fclose(f);
  if (out.empty()) out = "  not mapped (above every mapping)\n";
  if (out.back() != '\n') out += '\n';
  return out;
}

// Every ledger range whose pages contain va.
std::string ledger_matches(uint64_t va) {
  Ledger& l = L();
  std::unique_lock<std::timed_mutex> g(l.m, std::defer_lock);
  // never block the reporter for long; the lock is only ever held for a few map operations
  if (!g.try_lock_for(std::chrono::milliseconds(200)))
    return "  hydra: ledger busy for 200 ms (held by another thread), not read\n";
  std::string out;
  char buf[320];
  int n = 0;
  const uint64_t first = l.next > kLedgerSize ? l.next - kLedgerSize : 0;
  for (uint64_t s = l.next; s-- > first;) {
    const Entry& e = l.ring[s % kLedgerSize];
    const uint64_t lo = e.start & ~(kPage - 1), hi = (e.end + kPage - 1) & ~(kPage - 1);
    if (va < lo || va >= hi) continue;
    if (++n > 16) break;
    if (e.t_rel < 0)
      std::snprintf(buf, sizeof buf, "  hydra: %s [0x%" PRIx64 ", 0x%" PRIx64 ") #%" PRIu64
                    ", since t=%.6f s, LIVE%s\n", kind_name(e.kind), e.start, e.end, e.seq,
                    e.t_add, (va >= e.start && va < e.end) ? "" : " (va in its pages, outside it)");
    else
      std::snprintf(buf, sizeof buf, "  hydra: %s [0x%" PRIx64 ", 0x%" PRIx64 ") #%" PRIu64
                    ", t=%.6f .. %.6f s, RELEASED %.6f s ago\n", kind_name(e.kind), e.start,
                    e.end, e.seq, e.t_add, e.t_rel, l.now() - e.t_rel);
    out += buf;
  }
  if (!n) out = "  hydra: no block, registration or per-call pin of hydra's holds this address "
                "(torch's own memory, or a host buffer the HIP runtime pinned for a copy)\n";
  return out;
}

std::string report(uint64_t va, uint32_t reason) {
  char head[200];
  std::snprintf(head, sizeof head, "hydra fault report: GPU memory fault at VA 0x%" PRIx64
                " (reason 0x%x: %s)\n", va, reason, reasons(reason).c_str());
  return head + maps_line(va) + ledger_matches(va);
}

hsa_status_t on_event(const hsa_amd_event_t* ev, void*) {
  if (!ev || ev->event_type != HSA_AMD_GPU_MEMORY_FAULT_EVENT) return HSA_STATUS_SUCCESS;
  const uint64_t va = ev->memory_fault.virtual_address;
  const uint32_t reason = ev->memory_fault.fault_reason_mask;
  g_fault_va.store(va);
  g_fault_reason.store(reason);
  g_fault_count.fetch_add(1);
  const std::string r = report(va, reason);
  std::fputs(r.c_str(), stderr);
  std::fflush(stderr);
  return HSA_STATUS_SUCCESS;
}

}  // namespace

void ledger_add(LedgerKind kind, const void* p, size_t bytes) {
  Ledger& l = L();
  std::lock_guard<std::timed_mutex> g(l.m);
  const uint64_t seq = l.next++;
  Entry& e = l.ring[seq % kLedgerSize];
  if (e.t_rel < 0 && e.end) {  // overwritten while live: drop its index, unless a newer entry owns it
    auto it = l.live.find({e.kind, e.start});
    if (it != l.live.end() && it->second == e.seq) l.live.erase(it);
  }
  e.start = reinterpret_cast<uint64_t>(p);
  e.end = e.start + bytes;
  e.kind = kind;
  e.seq = seq;
  e.t_add = l.now();
  e.t_rel = -1;
  l.live[{kind, e.start}] = seq;
}

void ledger_release(LedgerKind kind, const void* p) {
  Ledger& l = L();
  std::lock_guard<std::timed_mutex> g(l.m);
  auto it = l.live.find({kind, reinterpret_cast<uint64_t>(p)});
  if (it == l.live.end()) return;
  Entry& e = l.ring[it->second % kLedgerSize];
  if (e.seq == it->second) e.t_rel = l.now();
  l.live.erase(it);
}

}  // namespace hydra

extern "C" {

int hydra_fault_report_enable(void) {
  if (hydra::g_enabled.load()) return hydra::ok();
  int count = 0;
  HIP_TRY(hipGetDeviceCount(&count));  // initialises the runtime (and HSA under it)
  const hsa_status_t s = hsa_amd_register_system_event_handler(hydra::on_event, nullptr);
  if (s != HSA_STATUS_SUCCESS)
    return hydra::fail(HYDRA_ERR_HIP, "hsa_amd_register_system_event_handler failed (status " +
                                          std::to_string(static_cast<int>(s)) + ")");
  hydra::g_enabled.store(true);
  return hydra::ok();
}

int hydra_fault_last(uint64_t* va, uint32_t* reason, uint64_t* count) {
  if (va) *va = hydra::g_fault_va.load();
  if (reason) *reason = hydra::g_fault_reason.load();
  if (count) *count = hydra::g_fault_count.load();
  return hydra::ok();
}

int hydra_fault_lookup(uint64_t va, char* buf, size_t len) {
  if (!buf || !len) return hydra::fail(HYDRA_ERR_INVALID, "null/empty buffer");
  const std::string r = hydra::maps_line(va) + hydra::ledger_matches(va);
  std::snprintf(buf, len, "%s", r.c_str());
  return hydra::ok();
}

}  // extern "C"
