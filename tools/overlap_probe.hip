// Do kernels on different HIP streams (HW queues) run concurrently on gfx950, and does a rocprofv3
// kernel trace show it? Two "half-GPU" kernels (128 single-wave workgroups spinning a fixed number of
// cycles) are launched one stream after another, then on two streams at once: with concurrent
// execution the pair takes about as long as one kernel. Run it plain and under
// `rocprofv3 --kernel-trace` and compare the walls and the trace's intervals (tools/timeline.py).
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/overlap_probe tools/overlap_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                                     \
    }                                                                                   \
  } while (0)

// Each workgroup (one wave) spins `iters` dependent integer steps and writes one word (vector store).
__global__ __launch_bounds__(64) void spin_kernel(unsigned* out, int iters) {
  unsigned v = threadIdx.x + blockIdx.x;
  for (int i = 0; i < iters; ++i) v = v * 1664525u + 1013904223u;
  if (v == 0x12345678u) out[blockIdx.x * 64 + threadIdx.x] = v;  // keeps the loop; practically never stores
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? std::atoi(argv[1]) : 128;  // half of the 256 CUs, one wave each
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200000;
  const int reps = 5;
  unsigned* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)blocks * 64 * sizeof(unsigned) * 2));
  hipStream_t s[2];
  for (auto& x : s) CHECK(hipStreamCreate(&x));
  // warm-up
  hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[0], out, 1000);
  CHECK(hipDeviceSynchronize());
  for (int rep = 0; rep < reps; ++rep) {
    double t0 = now_ms();
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[0], out, iters);
    CHECK(hipDeviceSynchronize());
    const double one = now_ms() - t0;
    t0 = now_ms();
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[0], out, iters);
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[0], out + blocks * 64, iters);
    CHECK(hipDeviceSynchronize());
    const double same = now_ms() - t0;
    t0 = now_ms();
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[0], out, iters);
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(64), 0, s[1], out + blocks * 64, iters);
    CHECK(hipDeviceSynchronize());
    const double two = now_ms() - t0;
    std::printf("rep %d: one kernel %.3f ms, two on one stream %.3f ms, two on two streams %.3f ms (%.2fx of one)\n",
                rep, one, same, two, two / one);
  }
  for (auto& x : s) CHECK(hipStreamDestroy(x));
  CHECK(hipFree(out));
  return 0;
}
