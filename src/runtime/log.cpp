#include "nm03/log.h"

#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

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

namespace {

void write_str(const char* s) {
  ssize_t r = ::write(2, s, std::strlen(s));
  (void)r;
}

void write_hex(uintptr_t v) {
  char buf[2 + 16 + 1];
  buf[0] = '0';
  buf[1] = 'x';
  for (int i = 0; i < 16; ++i) buf[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
  buf[18] = 0;
  write_str(buf);
}

void crash_handler(int sig, siginfo_t* si, void*) {
  // async-signal-safe only: write(2), backtrace (its libgcc is preloaded at install time)
  write_str("\n[nm03] fatal signal ");
  write_str(sig == SIGSEGV ? "SIGSEGV" : sig == SIGBUS ? "SIGBUS" : sig == SIGFPE ? "SIGFPE"
            : sig == SIGILL ? "SIGILL" : "SIGABRT");
  write_str(" at address ");
  write_hex((uintptr_t)(si ? si->si_addr : nullptr));
  write_str(", backtrace:\n");
  void* frames[64];
  const int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

void install_crash_handler() {
  static std::once_flag once;
  std::call_once(once, [] {
    void* warm[2];
    (void)backtrace(warm, 2);  // loads libgcc_s now, not inside the handler
    static char alt[64 * 1024];
    stack_t ss{};
    ss.ss_sp = alt;
    ss.ss_size = sizeof alt;
    sigaltstack(&ss, nullptr);
    struct sigaction sa{};
    sa.sa_sigaction = crash_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK | SA_RESETHAND;
    sigemptyset(&sa.sa_mask);
    for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT}) sigaction(sig, &sa, nullptr);
  });
}

}  // namespace nm03
