// tools/bar_probe.cpp — can the host CPU write MI355X device memory directly (large BAR), and how fast?
// (pack 12-bit pixels straight into VRAM instead of pinned host
// memory + SDMA, which would take 197 of the 426 KB/slice off the host DRAM.)
//
// Build: g++ -O2 -mavx2 -pthread -I/opt/rocm/include tools/bar_probe.cpp -o build/bin/bar_probe \
//            -L/opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
//
// 1. PCI BAR sizes of every AMD display/accelerator function (sysfs `resource`).
// 2. Every memory pool of the GPU agent: flags, size, ACCESSIBLE_BY_ALL, and the CPU agent's
//    access (never / allowed by default / disallowed by default).
// 3. If a VRAM pool admits the CPU: allocate 256 MiB there, grant the CPU access, time
//    write-combining streaming stores into it from 1/4/8/16 threads (the packer's store form),
//    then copy it back with the DMA engine and check every byte.
#include <dirent.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                            \
  do {                                                                      \
    hsa_status_t s_ = (x);                                                  \
    if (s_ != HSA_STATUS_SUCCESS) {                                         \
      const char* m_ = nullptr;                                             \
      hsa_status_string(s_, &m_);                                           \
      std::printf("%s failed: %s\n", #x, m_ ? m_ : "?");                    \
      return 1;                                                             \
    }                                                                       \
  } while (0)

static void print_bars() {
  DIR* d = opendir("/sys/bus/pci/devices");
  if (!d) return;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    std::string base = std::string("/sys/bus/pci/devices/") + e->d_name;
    auto rd = [&](const char* f) {
      char buf[64] = {0};
      FILE* fp = std::fopen((base + "/" + f).c_str(), "r");
      if (fp) {
        if (!std::fgets(buf, sizeof buf, fp)) buf[0] = 0;
        std::fclose(fp);
      }
      return std::string(buf);
    };
    const std::string vendor = rd("vendor"), cls = rd("class");
    if (vendor.rfind("0x1002", 0) != 0 || (cls.rfind("0x03", 0) != 0 && cls.rfind("0x12", 0) != 0)) continue;
    FILE* fp = std::fopen((base + "/resource").c_str(), "r");
    if (!fp) continue;
    std::printf("pci %s class %s", e->d_name, cls.c_str());
    unsigned long long a, b, fl;
    int bar = 0;
    while (std::fscanf(fp, "%llx %llx %llx", &a, &b, &fl) == 3) {
      if (b > a && bar < 6) std::printf("  BAR%d %.1f MiB%s\n", bar, (b - a + 1) / 1048576.0, (fl & 0x8) ? " (prefetchable)" : "");
      ++bar;
    }
    std::fclose(fp);
  }
  closedir(d);
}

struct Ctx {
  hsa_agent_t cpu{}, gpu{};
  bool have_cpu = false, have_gpu = false;
  std::vector<hsa_amd_memory_pool_t> gpu_pools, cpu_pools;
};

static hsa_status_t agent_cb(hsa_agent_t a, void* p) {
  auto* c = (Ctx*)p;
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !c->have_cpu) c->cpu = a, c->have_cpu = true;
  if (t == HSA_DEVICE_TYPE_GPU && !c->have_gpu) c->gpu = a, c->have_gpu = true;
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* v) {
  ((std::vector<hsa_amd_memory_pool_t>*)v)->push_back(p);
  return HSA_STATUS_SUCCESS;
}

int main() {
  print_bars();
  CHECK(hsa_init());
  Ctx c;
  CHECK(hsa_iterate_agents(agent_cb, &c));
  if (!c.have_cpu || !c.have_gpu) {
    std::printf("no CPU/GPU agent pair\n");
    return 1;
  }
  CHECK(hsa_amd_agent_iterate_memory_pools(c.gpu, pool_cb, &c.gpu_pools));
  CHECK(hsa_amd_agent_iterate_memory_pools(c.cpu, pool_cb, &c.cpu_pools));
  int pick = -1;
  for (size_t i = 0; i < c.gpu_pools.size(); ++i) {
    auto p = c.gpu_pools[i];
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    uint32_t flags = 0;
    size_t size = 0;
    bool all = false, alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_ACCESSIBLE_BY_ALL, &all);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    hsa_amd_memory_pool_access_t acc = HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED;
    hsa_amd_agent_memory_pool_get_info(c.cpu, p, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
    std::printf("gpu pool %zu: segment %d flags%s%s%s%s size %.1f GiB alloc %d accessible_by_all %d cpu_access %s\n", i,
                (int)seg, flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED ? " fine" : "",
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED ? " coarse" : "",
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_EXTENDED_SCOPE_FINE_GRAINED ? " ext-fine" : "",
                flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT ? " kernarg" : "", size / 1073741824.0, (int)alloc,
                (int)all,
                acc == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED       ? "never"
                : acc == HSA_AMD_MEMORY_POOL_ACCESS_ALLOWED_BY_DEFAULT ? "allowed-by-default"
                                                                        : "disallowed-by-default");
    if (seg == HSA_AMD_SEGMENT_GLOBAL && alloc && acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED && pick < 0) pick = (int)i;
  }
  if (pick < 0) {
    std::printf("RESULT: no VRAM pool the CPU may access (no large-BAR host mapping): rejected\n");
    hsa_shut_down();
    return 0;
  }
  const size_t N = 256ull << 20;
  void* vram = nullptr;
  CHECK(hsa_amd_memory_pool_allocate(c.gpu_pools[pick], N, 0, &vram));
  CHECK(hsa_amd_agents_allow_access(1, &c.cpu, nullptr, vram));
  std::printf("allocated %zu MiB in gpu pool %d at %p\n", N >> 20, pick, vram);
  // host source: what a packer would hold in its L2 (8 MiB, re-used)
  std::vector<uint8_t> src(8u << 20);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 2654435761u >> 13);
  for (int T : {1, 4, 8, 16}) {
    for (int rep = 0; rep < 3; ++rep) {
      std::atomic<int> ready{0};
      std::atomic<bool> go{false};
      std::vector<std::thread> th;
      const size_t per = N / T / 64 * 64;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          ready++;
          while (!go.load()) {
          }
          uint8_t* dst = (uint8_t*)vram + t * per;
          for (size_t off = 0; off < per; off += 64) {
            const __m256i* s = (const __m256i*)(src.data() + (t * per + off) % src.size());
            __m256i a = _mm256_loadu_si256(s), b = _mm256_loadu_si256(s + 1);
            _mm256_stream_si256((__m256i*)(dst + off), a);
            _mm256_stream_si256((__m256i*)(dst + off + 32), b);
          }
          _mm_sfence();
        });
      while (ready.load() < T) {
      }
      const double t0 = now();
      go = true;
      for (auto& x : th) x.join();
      const double dt = now() - t0;
      std::printf("CPU streaming stores into VRAM: %2d threads %.1f GB/s\n", T, per * T / dt / 1e9);
    }
  }
  // Read-back check through the DMA engine into a host buffer.
  hsa_amd_memory_pool_t host_pool{};
  bool got_host = false;
  for (auto p : c.cpu_pools) {
    uint32_t flags = 0;
    bool alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) host_pool = p, got_host = true;
  }
  if (got_host) {
    void* host = nullptr;
    CHECK(hsa_amd_memory_pool_allocate(host_pool, N, 0, &host));
    hsa_agent_t both[2] = {c.gpu, c.cpu};
    CHECK(hsa_amd_agents_allow_access(2, both, nullptr, host));
    hsa_signal_t sig;
    CHECK(hsa_signal_create(1, 0, nullptr, &sig));
    CHECK(hsa_amd_memory_async_copy(host, c.cpu, vram, c.gpu, N, 0, nullptr, sig));
    hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    const int T = 16;
    const size_t per = N / T / 64 * 64;
    size_t bad = 0;
    for (int t = 0; t < T; ++t)
      for (size_t off = 0; off < per; ++off)
        bad += ((uint8_t*)host)[t * per + off] != src[(t * per + off) % src.size()];
    std::printf("DMA read-back of the 16-thread pass: %zu mismatching bytes\n", bad);
    hsa_signal_destroy(sig);
    hsa_amd_memory_pool_free(host);
  }
  hsa_amd_memory_pool_free(vram);
  hsa_shut_down();
  return 0;
}
