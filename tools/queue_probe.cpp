// tools/queue_probe.cpp — what does a HIP stream cost at start-up? (round 5, cold CLI anatomy)
// Build: /opt/rocm/llvm/bin/clang++ -O2 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include tools/queue_probe.cpp \
//          -L/opt/rocm/lib -lamdhip64 -pthread -o build/bin/queue_probe
//
//   queue_probe <streams> <threads>
//
// hipInit + hipSetDevice, then `streams` non-blocking streams created by `threads` threads at once
// (each thread creates streams/threads), then one 25-slice-sized pinned and device allocation.
// Prints every phase in ms; run it under different GPU_MAX_HW_QUEUES values (HW queues are created
// lazily, one per stream up to that count, and then shared round-robin).
// PROBE_PREDLOPEN=1: a second thread dlopens libamd_comgr (the HIP runtime's code-object library,
// ≈ 8 ms to load) at start, while the main thread runs hipInit; the probe also prints after which
// phase the library is mapped.
// PROBE_SAMPLE=1: a 200 µs wall-clock timer on the main thread samples the interrupted PC during
// hipInit; the probe prints hipInit's time and the top library:symbol locations (slow vs fast mode).
#include <hip/hip_runtime_api.h>

#include <dlfcn.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <string>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool comgr_mapped() {
  FILE* f = std::fopen("/proc/self/maps", "r");
  if (!f) return false;
  char l[1024];
  bool m = false;
  while (!m && std::fgets(l, sizeof(l), f)) m = std::strstr(l, "libamd_comgr") != nullptr;
  std::fclose(f);
  return m;
}

static void* g_pcs[8192];
static volatile int g_npc = 0;
static void on_sample(int, siginfo_t*, void* uc) {
  const int i = g_npc;
  if (i < 8192) {
    g_pcs[i] = (void*)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
    g_npc = i + 1;
  }
}
struct Sampler {
  timer_t tm{};
  bool on = false;
  void start() {
    struct sigaction sa{};
    sa.sa_sigaction = on_sample;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGRTMIN, &sa, nullptr);
    sigevent ev{};
    ev.sigev_notify = SIGEV_THREAD_ID;
    ev.sigev_signo = SIGRTMIN;
    ev._sigev_un._tid = (pid_t)syscall(SYS_gettid);
    if (timer_create(CLOCK_MONOTONIC, &ev, &tm) != 0) return;
    itimerspec it{};
    it.it_interval.tv_nsec = it.it_value.tv_nsec = 200000;
    timer_settime(tm, 0, &it, nullptr);
    on = true;
  }
  void stop(double init_ms) {
    if (!on) return;
    timer_delete(tm);
    std::map<std::string, int> hist;
    for (int i = 0; i < g_npc; ++i) {
      Dl_info di{};
      std::string k = "?";
      if (dladdr(g_pcs[i], &di) && di.dli_fname) {
        const char* b = std::strrchr(di.dli_fname, '/');
        k = std::string(b ? b + 1 : di.dli_fname) + ":" + (di.dli_sname ? di.dli_sname : "?");
      }
      ++hist[k];
    }
    std::vector<std::pair<int, std::string>> v;
    for (auto& e : hist) v.push_back({e.second, e.first});
    std::sort(v.rbegin(), v.rend());
    std::printf("sample hipInit %.1f ms, %d samples:", init_ms, (int)g_npc);
    for (size_t i = 0; i < v.size() && i < 8; ++i) std::printf(" | %d %s", v[i].first, v[i].second.substr(0, 60).c_str());
    std::printf("\n");
  }
};

int main(int argc, char** argv) {
  const int ns = argc > 1 ? std::atoi(argv[1]) : 5;
  const int nt = argc > 2 ? std::atoi(argv[2]) : 1;
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  const bool pre = std::getenv("PROBE_PREDLOPEN") && std::atoi(std::getenv("PROBE_PREDLOPEN"));
  double t0 = now_ms(), t_pre = 0;
  std::thread pre_th;
  if (pre)
    pre_th = std::thread([&] {
      const double a = now_ms();
      (void)dlopen("libamd_comgr.so.3", RTLD_LAZY | RTLD_GLOBAL);
      t_pre = now_ms() - a;
    });
  const bool mapped0 = comgr_mapped();
  Sampler smp;
  const bool sample = std::getenv("PROBE_SAMPLE") && std::atoi(std::getenv("PROBE_SAMPLE"));
  const double ti = now_ms();
  if (sample) smp.start();
  if (hipInit(0) != hipSuccess || hipSetDevice(0) != hipSuccess) return 1;
  void* p = nullptr;
  (void)hipMalloc(&p, 4096);
  const double t1 = now_ms();
  if (sample) smp.stop(t1 - ti);
  const bool mapped1 = comgr_mapped();
  if (pre_th.joinable()) pre_th.join();
  std::vector<hipStream_t> st(ns, nullptr);
  std::vector<double> each(ns, 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int i = t; i < ns; i += nt) {
        const double a = now_ms();
        (void)hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
        each[i] = now_ms() - a;
      }
    });
  for (auto& x : th) x.join();
  const double t2 = now_ms();
  void* h = nullptr;
  void* d = nullptr;
  (void)hipHostMalloc(&h, 4u << 20, hipHostMallocDefault);
  const double t3 = now_ms();
  (void)hipMalloc(&d, 16u << 20);
  const double t4 = now_ms();
  // first kernel-free work on every stream: a 4 KiB memset
  for (int i = 0; i < ns; ++i) (void)hipMemsetAsync(d, 0, 4096, st[i]);
  for (int i = 0; i < ns; ++i) (void)hipStreamSynchronize(st[i]);
  const double t5 = now_ms();
  std::printf("GPU_MAX_HW_QUEUES=%s streams %d threads %d | init %.1f | streams %.1f (", q ? q : "(unset)", ns, nt, t1 - t0,
              t2 - t1);
  for (int i = 0; i < ns; ++i) std::printf("%s%.1f", i ? " " : "", each[i]);
  std::printf(") | pinned 4MiB %.2f | device 16MiB %.2f | first memsets %.2f ms", t3 - t2, t4 - t3, t5 - t4);
  std::printf(" | comgr mapped: start %d, after init %d, end %d%s", (int)mapped0, (int)mapped1, (int)comgr_mapped(),
              pre ? "" : "\n");
  if (pre) std::printf(" | predlopen %.1f ms\n", t_pre);
  return 0;
}
