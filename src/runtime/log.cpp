#include "nm03/log.h"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <mutex>
#include <sstream>

namespace nm03 {

LogLevel log_level() {
  static const LogLevel lvl = [] {
    const char* s = std::getenv("NM03_LOG");
    if (!s) return LogLevel::kWarn;
    if (!std::strcmp(s, "info")) return LogLevel::kInfo;
    if (!std::strcmp(s, "error")) return LogLevel::kError;
    if (!std::strcmp(s, "none")) return LogLevel::kNone;
    return LogLevel::kWarn;
  }();
  return lvl;
}

void log_msg(LogLevel lvl, const std::string& msg) {
  if ((int)lvl < (int)log_level() || lvl == LogLevel::kNone) return;
  static std::mutex m;
  static const char* tag[] = {"INFO", "WARNING", "ERROR"};
  std::lock_guard<std::mutex> g(m);
  std::cout << "[nm03 " << tag[(int)lvl] << "] " << msg << std::endl;
}

namespace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  bool on = false;
  Roctx() {
    const char* e = std::getenv("NM03_ROCTX");
    if (!e || !*e || *e == '0') return;
    // rocprofv3 --marker-trace intercepts the rocprofiler-sdk flavour; the legacy one is a fallback.
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    pop = (int (*)())dlsym(h, "roctxRangePop");
    on = push && pop;
  }
};

Roctx& roctx() {
  static Roctx r;
  return r;
}

}  // namespace

TraceRange::TraceRange(const char* name) : active_(roctx().on) {
  if (active_) roctx().push(name);
}
TraceRange::~TraceRange() {
  if (active_) roctx().pop();
}

const FaultPlan& fault_plan() {
  static const FaultPlan p = [] {
    FaultPlan f;
    const char* s = std::getenv("NM03_FAULT");
    if (!s) return f;
    std::stringstream ss(s);
    std::string item;
    while (std::getline(ss, item, ',')) {
      const size_t c = item.find(':');
      if (c == std::string::npos) continue;
      const std::string k = item.substr(0, c);
      const int64_t v = std::atoll(item.c_str() + c + 1);
      if (k == "corrupt_dicom") f.corrupt_dicom = v;
      else if (k == "fail_batch") f.fail_batch = v;
      else if (k == "fail_write") f.fail_write = v;
      else if (k == "rank_exit") f.rank_exit = v;
    }
    return f;
  }();
  return p;
}

}  // namespace nm03
