// roctx ranges around the serving path's stages, visible in
// `rocprofv3 --marker-trace` next to the kernel trace (tools/trace.sh).
//
// Reference counterpart: none beyond per-query wall time
// (src/services.rs:419,424; SURVEY.md §5 "Tracing / profiling"). Ranges here:
// engine ops (eager/profile mode; a replayed hipGraph is one range),
// executor stage/forward, member predict, leader query dispatch.
// A range costs a function-pointer call when no tool is attached.
// The ThreadSanitizer build defines DMLC_NO_ROCTX (it links no ROCm library).
#pragma once

#ifndef DMLC_NO_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

namespace dmlc {

class TraceRange {
 public:
  explicit TraceRange(const char* name) {
#ifndef DMLC_NO_ROCTX
    roctxRangePushA(name);
#else
    (void)name;
#endif
  }
  ~TraceRange() {
#ifndef DMLC_NO_ROCTX
    roctxRangePop();
#endif
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace dmlc

#define DMLC_TRACE_CAT2(a, b) a##b
#define DMLC_TRACE_CAT(a, b) DMLC_TRACE_CAT2(a, b)
#define DMLC_TRACE(name) ::dmlc::TraceRange DMLC_TRACE_CAT(dmlc_trace_, __LINE__)(name)
