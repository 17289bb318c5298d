// In-process CPU sampling profiler (nm03/cpu_sampler.h).
//
// Output (text, one record per line):
//   # nm03 cpu samples v2
//   period_us <p>
//   samples <written> dropped <n>
//   map <start> <end> <file offset> <path>          executable mappings (hex), from /proc/self/maps
//   thread <tid> <name>
//   s <count> <tid> <rsi> <pc0> <pc1> ...           one distinct (thread, RSI, call chain), leaf first (hex);
//                                                   RSI at the interrupted pc: after a system call it
//                                                   still holds the call's second argument (an ioctl's
//                                                   request code, a futex's operation)
#include "nm03/cpu_sampler.h"

#include <dirent.h>
#include <errno.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace nm03::prof {

namespace {

constexpr int kMaxDepth = 64;

std::mutex g_m;                        // start/stop
std::atomic<bool> g_on{false};         // the handler records
std::atomic<int> g_inside{0};          // handlers currently running
std::atomic<size_t> g_next{0};         // next record
std::atomic<size_t> g_dropped{0};
std::unique_ptr<uint64_t[]> g_buf;     // records of g_stride words: tid, frames, rsi, pc...
size_t g_cap = 0, g_stride = 0;
int g_depth = 0, g_period_us = 0;
std::vector<timer_t> g_timers;  // one per thread alive at start()
bool g_have_timer = false;

void on_sigprof(int, siginfo_t*, void* ctx) {
  const int saved = errno;
  // seq_cst with sampler_stop's store of g_on and load of g_inside (a Dekker pair): either stop
  // sees this handler inside, or this handler sees the sampler off and records nothing.
  g_inside.fetch_add(1, std::memory_order_seq_cst);
  if (g_on.load(std::memory_order_seq_cst)) {
    const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
    if (i < g_cap) {
      uint64_t* r = g_buf.get() + i * g_stride;
      void* bt[kMaxDepth + 4];
      const int n = backtrace(bt, g_depth + 4);
      const uintptr_t pc = (uintptr_t)static_cast<ucontext_t*>(ctx)->uc_mcontext.gregs[REG_RIP];
      r[2] = (uint64_t)static_cast<ucontext_t*>(ctx)->uc_mcontext.gregs[REG_RSI];
      // Skip the handler's own frames and the signal trampoline: the chain starts at the
      // interrupted pc (the unwinder reports it exactly for the frame under a signal frame).
      int k = 0;
      while (k < n && (uintptr_t)bt[k] != pc) ++k;
      int m = 0;
      if (k == n) {
        r[3] = pc;  // unwinding did not reach it: the pc alone
        m = 1;
      } else {
        for (; k < n && m < g_depth; ++k) r[3 + m++] = (uint64_t)(uintptr_t)bt[k];
      }
      r[1] = (uint64_t)m;
      r[0] = (uint64_t)::syscall(SYS_gettid);
    } else {
      g_dropped.fetch_add(1, std::memory_order_relaxed);
    }
  }
  g_inside.fetch_sub(1, std::memory_order_release);
  errno = saved;
}

std::string thread_name(uint64_t tid) {
  std::ifstream f("/proc/self/task/" + std::to_string(tid) + "/comm");
  std::string s;
  if (!std::getline(f, s) || s.empty()) return "?";
  for (char& c : s)
    if (c == ' ') c = '_';
  return s;
}

}  // namespace

bool sampler_running() { return g_on.load(); }

bool sampler_start(int period_us, size_t max_samples, int depth) {
  std::lock_guard<std::mutex> g(g_m);
  if (g_on.load() || g_have_timer) return false;
  if (period_us < 10) period_us = 10;
  if (depth < 1) depth = 1;
  if (depth > kMaxDepth) depth = kMaxDepth;
  if (max_samples < 1) max_samples = 1;
  {
    void* warm[4];
    (void)backtrace(warm, 4);  // loads libgcc_s here, never inside the handler
  }
  g_depth = depth;
  g_stride = 3 + (size_t)depth;
  g_cap = max_samples;
  g_buf.reset(new uint64_t[g_cap * g_stride]);
  g_next = 0;
  g_dropped = 0;
  g_period_us = period_us;
  struct sigaction sa {};
  sa.sa_sigaction = on_sigprof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, nullptr) != 0) return false;
  // One timer per thread on that thread's CPU clock, signalling that thread: a timer on the
  // process clock fires at most once per scheduler tick for the whole process (≈ 1 sample per tick
  // however many threads run), per-thread timers once per tick per running thread. Threads started
  // later are not sampled (start after the engine and its pools exist).
  std::vector<long> tids;
  if (DIR* d = opendir("/proc/self/task")) {
    while (dirent* e = readdir(d))
      if (e->d_name[0] >= '0' && e->d_name[0] <= '9') tids.push_back(std::atol(e->d_name));
    closedir(d);
  }
  itimerspec its{};
  its.it_interval.tv_sec = period_us / 1000000;
  its.it_interval.tv_nsec = (long)(period_us % 1000000) * 1000;
  its.it_value = its.it_interval;
  g_on.store(true, std::memory_order_release);
  for (long tid : tids) {
    sigevent sev{};
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = (int)tid;
    // The CPU clock of thread `tid` (the kernel's MAKE_THREAD_CPUCLOCK(tid, CPUCLOCK_SCHED)).
    const clockid_t clk = (clockid_t)((~(unsigned)tid << 3) | 6);
    timer_t t{};
    if (timer_create(clk, &sev, &t) != 0) continue;  // the thread may have exited meanwhile
    if (timer_settime(t, 0, &its, nullptr) != 0) {
      timer_delete(t);
      continue;
    }
    g_timers.push_back(t);
  }
  g_have_timer = true;
  if (g_timers.empty()) {
    g_on = false;
    g_have_timer = false;
    return false;
  }
  return true;
}

size_t sampler_stop(const std::string& path) {
  std::lock_guard<std::mutex> g(g_m);
  if (!g_have_timer) return 0;
  for (timer_t t : g_timers) timer_delete(t);
  g_timers.clear();
  g_have_timer = false;
  g_on.store(false, std::memory_order_seq_cst);
  // A SIGPROF already pending is discarded once ignored; handlers already running finish first.
  struct sigaction ign {};
  ign.sa_handler = SIG_IGN;
  sigemptyset(&ign.sa_mask);
  sigaction(SIGPROF, &ign, nullptr);
  while (g_inside.load(std::memory_order_seq_cst) != 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
  const size_t n = std::min(g_next.load(), g_cap);
  // Distinct (thread, chain) with counts.
  std::map<std::vector<uint64_t>, uint64_t> stacks;
  std::set<uint64_t> tids;
  for (size_t i = 0; i < n; ++i) {
    const uint64_t* r = g_buf.get() + i * g_stride;
    const size_t m = std::min<uint64_t>(r[1], (uint64_t)g_depth);
    std::vector<uint64_t> key(r, r + 3 + m);
    key[1] = 0;
    ++stacks[key];
    tids.insert(r[0]);
  }
  FILE* f = std::fopen(path.c_str(), "w");
  if (!f) return 0;
  std::fprintf(f, "# nm03 cpu samples v2\nperiod_us %d\nsamples %zu dropped %zu\n", g_period_us, n, g_dropped.load());
  {
    std::ifstream maps("/proc/self/maps");
    std::string line;
    while (std::getline(maps, line)) {
      unsigned long long lo = 0, hi = 0, off = 0;
      char perms[8] = {0};
      int pos = 0;
      if (std::sscanf(line.c_str(), "%llx-%llx %7s %llx %*s %*s %n", &lo, &hi, perms, &off, &pos) < 4) continue;
      if (perms[2] != 'x' || pos <= 0 || pos >= (int)line.size()) continue;
      std::fprintf(f, "map %llx %llx %llx %s\n", lo, hi, off, line.c_str() + pos);
    }
  }
  for (uint64_t t : tids) std::fprintf(f, "thread %llu %s\n", (unsigned long long)t, thread_name(t).c_str());
  for (const auto& [key, count] : stacks) {
    std::fprintf(f, "s %llu %llu", (unsigned long long)count, (unsigned long long)key[0]);
    for (size_t k = 2; k < key.size(); ++k) std::fprintf(f, " %llx", (unsigned long long)key[k]);  // rsi, pcs
    std::fputc('\n', f);
  }
  std::fclose(f);
  g_buf.reset();
  return n;
}

}  // namespace nm03::prof
