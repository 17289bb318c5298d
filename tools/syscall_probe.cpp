// tools/syscall_probe.cpp — cost of a trivial system call (entry/exit incl. the kernel's speculative
// execution mitigations) and of fstat/close-like calls on this host, one thread.
// Build: g++ -O2 tools/syscall_probe.cpp -o build/bin/syscall_probe
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
int main() {
  const int n = 500000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) syscall(SYS_getppid);
  auto t1 = std::chrono::steady_clock::now();
  int fd = open("/proc/self/exe", O_RDONLY);
  struct stat st;
  for (int i = 0; i < n; ++i) fstat(fd, &st);
  auto t2 = std::chrono::steady_clock::now();
  close(fd);
  auto ns = [&](auto a, auto b) { return std::chrono::duration<double>(b - a).count() * 1e9 / n; };
  std::printf("getppid %.0f ns, fstat %.0f ns\n", ns(t0, t1), ns(t1, t2));
  FILE* f = std::fopen("/sys/devices/system/cpu/vulnerabilities/spec_rstack_overflow", "r");
  char buf[256] = {0};
  if (f && std::fgets(buf, sizeof buf, f)) std::printf("srso: %s", buf);
  if (f) std::fclose(f);
  f = std::fopen("/sys/devices/system/cpu/vulnerabilities/retbleed", "r");
  if (f && std::fgets(buf, sizeof buf, f)) std::printf("retbleed: %s", buf);
  if (f) std::fclose(f);
  return 0;
}
