// options.h -- the library's tunables (hydra_set_option / hydra_ctx_set_option, hydra_hip.h).
//
// No environment variable is read anywhere in the library: every knob is an explicit option on
// the C-ABI with the tuned default below (the reference's benchmark takes its settings the same
// way, as flags: benchmark/options.cc:144-172).  Process-wide values apply to what starts after
// they are set (a resident reducer instance, the copy pool, a context created later); the
// per-context keys are copied into each context at hydra_ctx_create and can be overridden there.
#pragma once
#include <stdint.h>

#include <atomic>

#include "../../include/hydra_hip.h"

namespace hydra {

constexpr int kOptCount = HYDRA_OPT_RESIDENT_TILES + 1;

struct OptSpec {
  int64_t dflt, lo, hi;
  bool per_ctx;  // may be overridden per context
};

// key -> default and accepted range (hydra_hip.h documents each key)
inline const OptSpec& opt_spec(int key) {
  static const OptSpec kSpec[kOptCount] = {
      {0, 0, 0, false},                             // (unused)
      {1, 0, 1, true},                              // RESIDENT
      {4, 1, 64, true},                             // STAGE_SPLIT
      {512 << 10, 16 << 10, 4 << 20, true},         // ROUND_MIN
      {0, 0, int64_t(1) << 40, true},               // STAGE_RESULT_MAX
      {8 << 20, 0, int64_t(1) << 40, true},         // STAGE_RESULT_REG_MAX
      {0, 0, 1, true},                              // FORCE_STAGING
      {4, 0, 32, false},                            // COPY_THREADS
      {2000, 50, 1000000, false},                   // RESIDENT_IDLE_US
      {10000000, 1000, 600000000, false},           // RESIDENT_GRACE_US
      {0, 0, 2, false},                             // RESIDENT_QUEUE
      {128, 1, 1024, false},                        // RESIDENT_BLOCKS (kResidentMaxBlocks)
      {4, 1, 4, false},                             // RESIDENT_BATCH (1, 2 or 4)
      {4, 0, 64, false},                            // RESIDENT_SOLO
      {4, 1, 64, false},                            // RESIDENT_TILES
  };
  return kSpec[key];
}

// the process-wide value of `key` (its default until hydra_set_option changed it); options.cpp
int64_t opt(int key);
void opt_set(int key, int64_t value);  // (range-checked by hydra_set_option)

// one context's copy of the per-context keys
struct CtxOpts {
  int64_t v[kOptCount];
  void load() {
    for (int k = 1; k < kOptCount; k++) v[k] = opt(k);
  }
  int64_t operator[](int key) const { return v[key]; }
};

}  // namespace hydra
