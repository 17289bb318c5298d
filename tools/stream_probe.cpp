// Host memory-bandwidth probe (STREAM-style) for the host-path ceiling model (docs/ARCHITECTURE.md
// "Host ceiling"). Per thread count T and placement (spread: one thread per physical core, cores
// spread over the allowed CPUs; packed: consecutive cores; float: unpinned) it measures
//   read   — sum of a DRAM-resident source (page-cache read analogue)
//   copy   — memcpy DRAM source → L2-resident 128 KiB buffer (the loader's pread)
//   ntw    — streaming stores of 96 KiB per "slice" into a large destination (12-bit pack → pinned blob)
//   slice  — the loader's memory work per 256² slice: copy 128 KiB into L2, then stream 96 KiB out
// Buffers are first-touched by their own thread (local NUMA node). Output: one line per case with
// the aggregate GB/s and the per-slice µs of the "slice" kernel.
//   build: clang++ -O2 -mavx2 -std=c++17 tools/stream_probe.cpp -lpthread -o build/bin/stream_probe
//   run:   stream_probe [max_threads=16] [MiB_per_thread=512]
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::string read_line(const std::string& p) {
  std::ifstream f(p);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}

// Physical cores of the allowed CPUs, in CPU order: each entry = its logical CPUs.
static std::vector<std::vector<int>> allowed_cores() {
  cpu_set_t set;
  sched_getaffinity(0, sizeof(set), &set);
  std::map<long, size_t> at;
  std::vector<std::vector<int>> cores;
  for (int c = 0; c < CPU_SETSIZE; ++c) {
    if (!CPU_ISSET(c, &set)) continue;
    const std::string b = "/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/";
    const std::string core = read_line(b + "core_id"), pkg = read_line(b + "physical_package_id");
    const long key = core.empty() ? (1L << 40) + c : (std::atol(pkg.c_str()) << 20) | std::atol(core.c_str());
    auto it = at.find(key);
    if (it == at.end()) {
      at.emplace(key, cores.size());
      cores.push_back({c});
    } else {
      cores[it->second].push_back(c);
    }
  }
  return cores;
}

static void pin(const std::vector<int>& cpus) {
  cpu_set_t s;
  CPU_ZERO(&s);
  for (int c : cpus) CPU_SET(c, &s);
  pthread_setaffinity_np(pthread_self(), sizeof(s), &s);
}

static void nt_copy(uint8_t* d, const uint8_t* s, size_t n) {
  for (size_t i = 0; i + 64 <= n; i += 64) {
    const __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
    const __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
    _mm256_stream_si256((__m256i*)(d + i), a);
    _mm256_stream_si256((__m256i*)(d + i + 32), b);
  }
}

int main(int argc, char** argv) {
  const int max_t = argc > 1 ? std::atoi(argv[1]) : 16;
  const size_t per_thread = (size_t)(argc > 2 ? std::atoi(argv[2]) : 512) << 20;
  const auto cores = allowed_cores();
  std::printf("allowed physical cores: %zu (logical CPUs %zu)\n", cores.size(),
              [&] { size_t n = 0; for (auto& c : cores) n += c.size(); return n; }());
  const size_t kIn = 128 << 10, kOut = 96 << 10;
  std::vector<int> counts;
  for (int t = 1; t <= max_t; t *= 2) counts.push_back(t);
  if (counts.back() != max_t) counts.push_back(max_t);
  for (const char* mode : {"spread", "packed", "float"}) {
    for (int T : counts) {
      if (T > (int)cores.size() && std::string(mode) != "float") continue;
      std::vector<double> gb_read(T), gb_copy(T), gb_ntw(T), us_slice(T);
      std::atomic<int> ready{0};
      std::atomic<bool> go{false};
      std::vector<std::thread> th;
      for (int i = 0; i < T; ++i)
        th.emplace_back([&, i] {
          if (std::string(mode) == "spread") pin(cores[(size_t)i * cores.size() / T]);
          if (std::string(mode) == "packed") pin(cores[(size_t)i]);
          auto* src = (uint8_t*)mmap(nullptr, per_thread, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
          auto* dst = (uint8_t*)mmap(nullptr, per_thread, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
          std::memset(src, 1, per_thread);  // first touch on this thread's node
          std::memset(dst, 0, per_thread);
          std::vector<uint8_t> l2(kIn);
          ready++;
          while (!go) std::this_thread::yield();
          // read
          double t0 = now();
          __m256i acc = _mm256_setzero_si256();
          for (size_t o = 0; o < per_thread; o += 64)
            acc = _mm256_add_epi64(acc, _mm256_loadu_si256((const __m256i*)(src + o)));
          volatile long sink = _mm256_extract_epi64(acc, 0);
          (void)sink;
          gb_read[i] = per_thread / (now() - t0) / 1e9;
          // copy DRAM -> L2 buffer
          t0 = now();
          for (size_t o = 0; o + kIn <= per_thread; o += kIn) std::memcpy(l2.data(), src + o, kIn);
          gb_copy[i] = per_thread / (now() - t0) / 1e9;
          // streaming writes
          t0 = now();
          for (size_t o = 0; o + kOut <= per_thread; o += kOut) nt_copy(dst + o, l2.data(), kOut);
          _mm_sfence();
          gb_ntw[i] = per_thread / (now() - t0) / 1e9;
          // slice = copy 128 KiB in + stream 96 KiB out
          const size_t slices = per_thread / kIn;
          t0 = now();
          for (size_t k = 0; k < slices; ++k) {
            std::memcpy(l2.data(), src + k * kIn, kIn);
            nt_copy(dst + (k * kOut) % (per_thread - kOut), l2.data(), kOut);
          }
          _mm_sfence();
          us_slice[i] = (now() - t0) * 1e6 / slices;
          munmap(src, per_thread);
          munmap(dst, per_thread);
        });
      while (ready < T) std::this_thread::yield();
      go = true;
      for (auto& t : th) t.join();
      double r = 0, c = 0, w = 0, us = 0;
      for (int i = 0; i < T; ++i) {
        r += gb_read[i];
        c += gb_copy[i];
        w += gb_ntw[i];
        us += us_slice[i];
      }
      std::printf("%-6s T=%2d  read %7.1f GB/s  copy->L2 %7.1f GB/s  nt-write %7.1f GB/s  slice %6.2f us/thread"
                  "  (%7.0f slices/s aggregate)\n",
                  mode, T, r, c, w, us / T, T / (us / T) * 1e6);
    }
  }
  return 0;
}
