// tools/hip_init_probe.hip — where the CLI's ≈170 ms of HIP start-up goes (config.cli_wall:
// hip_init_s). Times, in a fresh process: hipInit, hipGetDeviceCount, hipSetDevice + hipFree(0)
// (context), first hipMalloc, first stream, first pinned allocation, first kernel launch + sync.
// Run it under different environments (all GPUs visible vs ROCR_VISIBLE_DEVICES=<one>).
// Build: hipcc --offload-arch=gfx950 -O2 tools/hip_init_probe.hip -o build/bin/hip_init_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
__global__ void tiny(int* p) {
  if (threadIdx.x == 0 && p) p[0] = 1;
}
int main() {
  const char* env[] = {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"};
  for (const char* e : env) std::printf("%s=%s ", e, std::getenv(e) ? std::getenv(e) : "(unset)");
  std::printf("\n");
  const double t0 = now();
  hipInit(0);
  const double t1 = now();
  int n = 0;
  hipGetDeviceCount(&n);
  const double t2 = now();
  hipSetDevice(0);
  hipFree(nullptr);
  const double t3 = now();
  void* p = nullptr;
  hipMalloc(&p, 1 << 20);
  const double t4 = now();
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  const double t5 = now();
  void* h = nullptr;
  hipHostMalloc(&h, 1 << 20, hipHostMallocDefault);
  const double t6 = now();
  tiny<<<1, 64, 0, s>>>((int*)p);
  hipStreamSynchronize(s);
  const double t7 = now();
  std::printf("devices %d | hipInit %.1f ms, count %.1f, setDevice+ctx %.1f, hipMalloc %.1f, stream %.1f, "
              "hostMalloc %.1f, first launch %.1f | total %.1f ms\n",
              n, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3, (t6 - t5) * 1e3,
              (t7 - t6) * 1e3, (t7 - t0) * 1e3);
  std::fflush(stdout);
  std::_Exit(0);
}
