// Cost of pinning page-cache pages for zero-copy uploads: mmap a 128 KiB tmpfs file (one DICOM
// slice's size), hipHostRegister it, copy it to the device with SDMA, unregister, unmap — per file,
// single-threaded and with 8 threads — versus the engine's pread + copy into a pre-pinned buffer.
//   hipcc --offload-arch=gfx950 -O3 tools/register_probe.hip -o build/register_probe && build/register_probe
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int nfiles = 256;
  const size_t bytes = 131072 + 4096;
  const std::string dir = "/dev/shm/nm03_regprobe";
  std::string cmd = "mkdir -p " + dir;
  if (std::system(cmd.c_str()) != 0) return 1;
  std::vector<char> data(bytes, 7);
  for (int i = 0; i < nfiles; ++i) {
    const std::string p = dir + "/" + std::to_string(i);
    int fd = open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0 || write(fd, data.data(), bytes) != (ssize_t)bytes) return 2;
    close(fd);
  }
  CK(hipSetDevice(0));
  void* dev;
  CK(hipMalloc(&dev, bytes * 8));
  void* pinned;
  CK(hipHostMalloc(&pinned, bytes * 8, hipHostMallocDefault));
  hipStream_t st;
  CK(hipStreamCreate(&st));

  for (int threads : {1, 8}) {
    // (a) register path
    std::atomic<int> next{0};
    double t0 = now();
    auto reg_work = [&](int tid) {
      for (int i; (i = next.fetch_add(1)) < nfiles;) {
        const std::string p = dir + "/" + std::to_string(i);
        int fd = open(p.c_str(), O_RDONLY);
        void* m = mmap(nullptr, bytes, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, 0);
        if (m == MAP_FAILED) std::exit(3);
        CK(hipHostRegister(m, bytes, hipHostRegisterReadOnly));
        void* dp;
        CK(hipHostGetDevicePointer(&dp, m, 0));
        CK(hipMemcpyAsync((char*)dev + tid * bytes, m, bytes, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));
        CK(hipHostUnregister(m));
        munmap(m, bytes);
        close(fd);
      }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(reg_work, t);
    for (auto& t : th) t.join();
    double t1 = now();
    // (b) pread into pinned + copy
    next = 0;
    auto pread_work = [&](int tid) {
      for (int i; (i = next.fetch_add(1)) < nfiles;) {
        const std::string p = dir + "/" + std::to_string(i);
        int fd = open(p.c_str(), O_RDONLY);
        if (pread(fd, (char*)pinned + tid * bytes, bytes, 0) != (ssize_t)bytes) std::exit(4);
        CK(hipMemcpyAsync((char*)dev + tid * bytes, (char*)pinned + tid * bytes, bytes, hipMemcpyHostToDevice, st));
        CK(hipStreamSynchronize(st));
        close(fd);
      }
    };
    th.clear();
    for (int t = 0; t < threads; ++t) th.emplace_back(pread_work, t);
    for (auto& t : th) t.join();
    double t2 = now();
    std::printf("{\"threads\": %d, \"register_us_per_file\": %.1f, \"pread_pinned_us_per_file\": %.1f}\n", threads,
                (t1 - t0) * 1e6 * threads / nfiles, (t2 - t1) * 1e6 * threads / nfiles);
  }
  cmd = "rm -rf " + dir;
  return std::system(cmd.c_str());
}
