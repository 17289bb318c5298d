// nm03/log.h — observability helpers.
//
//  * Log levels mirror FAST's Reporter configuration in the reference
//    (Reporter::setGlobalReportMethod(INFO, NONE); WARNING/ERROR → COUT, main_sequential.cpp:349-354):
//    NM03_LOG=info|warn|error|none (default warn). The reference message catalogue itself is
//    always printed; these levels gate the engine's own diagnostics.
//  * roctx ranges (NM03_ROCTX=1 or under rocprofv3 --marker-trace) around load / upload / kernels
//    / export so rocprofv3 timelines show the pipeline stages.
//  * Fault injection for the failure-isolation tests:
//    NM03_FAULT=corrupt_dicom:<i>[,fail_batch:<k>][,fail_write:<j>] makes work item i fail to
//    parse, batch k fail on the device path, or item j's export fail (indices within one run).
#pragma once

#include <atomic>
#include <cstdint>
#include <string>

namespace nm03 {

enum class LogLevel : int { kInfo = 0, kWarn = 1, kError = 2, kNone = 3 };

LogLevel log_level();
void log_msg(LogLevel lvl, const std::string& msg);  // → stdout (info/warn/error), like Reporter::COUT
inline void log_info(const std::string& m) { log_msg(LogLevel::kInfo, m); }
inline void log_warn(const std::string& m) { log_msg(LogLevel::kWarn, m); }

// RAII roctx range (no-op unless enabled; libroctx64 is loaded lazily with dlopen).
class TraceRange {
 public:
  explicit TraceRange(const char* name);
  ~TraceRange();
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool active_;
};

struct FaultPlan {
  int64_t corrupt_dicom = -1;  // work-item index whose DICOM is treated as corrupt
  int64_t fail_batch = -1;     // batch index whose device work fails
  int64_t fail_write = -1;     // work-item index whose JPEG export fails
  int64_t rank_exit = -1;      // rank (img_processing_parallel) that dies after the plan broadcast
};
const FaultPlan& fault_plan();  // parsed once from NM03_FAULT

// Fatal-signal reporter for the native executables: on SIGSEGV/SIGBUS/SIGFPE/SIGILL/SIGABRT it
// writes the signal, the faulting address and a symbolised backtrace (backtrace_symbols_fd, no
// allocation) to stderr, then re-raises with the default action so the exit status is unchanged.
// Runs on an alternate stack (a stack overflow still reports). Idempotent.
void install_crash_handler();

}  // namespace nm03
