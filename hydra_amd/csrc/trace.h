// trace.h -- named host ranges for rocprofv3 --marker-trace (roctx), the build's equivalent of
// the reference's ad-hoc per-call timing prints (pipeallreduce-a.cc:33-49).  Near-free when no
// profiler is attached.  Async entry points mark the enqueue; synchronous ones the whole call.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace hydra {
struct TraceRange {
  explicit TraceRange(const char* name) { roctxRangePushA(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};
}  // namespace hydra
