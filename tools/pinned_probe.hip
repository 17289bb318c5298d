// Pinned-memory probe: CPU-side cost of the host buffers the engine uses, per allocation kind —
// memcpy into / out of the buffer, streaming (non-temporal) stores into it, and pread of a tmpfs
// file into it. The engine's loader writes the upload blob (hipHostMalloc default) and its writers
// read the GPU-written JPEG area (hipHostMallocMapped); whether the CPU maps these write-back or
// uncached/write-combined decides which copy strategy is cheap.
//   hipcc --offload-arch=gfx950 -O2 tools/pinned_probe.hip -o build/bin/pinned_probe
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void nt_copy(void* d, const void* s, size_t n) {
  auto* dd = (__m128i*)d;
  auto* ss = (const __m128i*)s;
  for (size_t i = 0; i < n / 16; ++i) _mm_stream_si128(dd + i, _mm_loadu_si128(ss + i));
  _mm_sfence();
}

int main(int argc, char** argv) {
  const size_t chunk = 128 * 1024, total = 64ull << 20;
  const char* file = argc > 1 ? argv[1] : "/dev/shm/pinned_probe.bin";
  {
    std::vector<char> z(chunk, 7);
    int fd = open(file, O_CREAT | O_WRONLY | O_TRUNC, 0644);
    if (fd < 0 || write(fd, z.data(), chunk) != (ssize_t)chunk) return 1;
    close(fd);
  }
  std::vector<char> src(chunk, 3), dst(chunk);
  struct Kind {
    const char* name;
    unsigned flags;
    int mode;  // 0 hipHostMalloc, 1 malloc + hipHostRegister, 2 plain malloc
  } kinds[] = {{"plain malloc (reference)", 0, 2},
               {"hipHostMalloc default", hipHostMallocDefault, 0},
               {"hipHostMalloc mapped", hipHostMallocMapped, 0},
               {"hipHostMalloc coherent", hipHostMallocCoherent, 0},
               {"hipHostMalloc noncoherent", hipHostMallocNonCoherent, 0},
               {"malloc + hipHostRegister", 0, 1}};
  (void)hipSetDevice(0);
  for (const Kind& k : kinds) {
    char* buf = nullptr;
    if (k.mode == 0) {
      if (hipHostMalloc((void**)&buf, total, k.flags) != hipSuccess) {
        std::printf("%-30s alloc failed\n", k.name);
        continue;
      }
    } else {
      buf = (char*)aligned_alloc(4096, total);
      memset(buf, 0, total);
      if (k.mode == 1 && hipHostRegister(buf, total, hipHostRegisterDefault) != hipSuccess) {
        std::printf("%-30s register failed\n", k.name);
        continue;
      }
    }
    memset(buf, 1, total);
    const int fd = open(file, O_RDONLY);
    double t[4] = {1e9, 1e9, 1e9, 1e9};
    for (int rep = 0; rep < 3; ++rep) {
      double t0 = now();
      for (size_t o = 0; o + chunk <= total; o += chunk) memcpy(buf + o, src.data(), chunk);
      t[0] = std::min(t[0], now() - t0);
      t0 = now();
      for (size_t o = 0; o + chunk <= total; o += chunk) nt_copy(buf + o, src.data(), chunk);
      t[1] = std::min(t[1], now() - t0);
      t0 = now();
      for (size_t o = 0; o + chunk <= total; o += chunk) memcpy(dst.data(), buf + o, chunk);
      t[2] = std::min(t[2], now() - t0);
      t0 = now();
      for (size_t o = 0; o + chunk <= total; o += chunk)
        if (pread(fd, buf + o, chunk, 0) != (ssize_t)chunk) return 2;
      t[3] = std::min(t[3], now() - t0);
    }
    close(fd);
    const double gb = total / 1e9;
    std::printf("%-30s memcpy in %6.1f GB/s | NT stores in %6.1f GB/s | memcpy out %6.1f GB/s | pread in %6.1f GB/s\n",
                k.name, gb / t[0], gb / t[1], gb / t[2], gb / t[3]);
    if (k.mode == 0)
      (void)hipHostFree(buf);
    else {
      if (k.mode == 1) (void)hipHostUnregister(buf);
      free(buf);
    }
  }
  unlink(file);
  return 0;
}
