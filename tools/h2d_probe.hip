// Host->device upload probe for the engine's batch blob (≈8.4 MB = 64 slices of 256² u16 + tables):
// SDMA hipMemcpyAsync on 1/2/4 streams vs. a copy kernel that reads the pinned (host-mapped) blob
// over PCIe with 16-byte loads, for several grid sizes. Answers whether a shader-side upload beats
// the copy engine on this box (ARCHITECTURE.md §6).
//   hipcc --offload-arch=gfx950 -O3 tools/h2d_probe.hip -o build/h2d_probe && build/h2d_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) pull_kernel(const v4u* __restrict__ src, v4u* __restrict__ dst, size_t n) {
  size_t stride = size_t(gridDim.x) * blockDim.x;
  size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
  // 4 independent 16-byte loads in flight per lane hide PCIe latency.
  for (; i + 3 * stride < n; i += 4 * stride) {
    v4u a = __builtin_nontemporal_load(src + i);
    v4u b = __builtin_nontemporal_load(src + i + stride);
    v4u c = __builtin_nontemporal_load(src + i + 2 * stride);
    v4u d = __builtin_nontemporal_load(src + i + 3 * stride);
    dst[i] = a; dst[i + stride] = b; dst[i + 2 * stride] = c; dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

int main() {
  const size_t bytes = size_t(64) * 256 * 256 * 2 + 64 * 1024;
  const int nbuf = 6, reps = 48;
  std::vector<void*> host(nbuf), dev(nbuf);
  std::vector<hipStream_t> st(nbuf);
  for (int i = 0; i < nbuf; ++i) {
    CK(hipHostMalloc(&host[i], bytes, hipHostMallocDefault));
    std::memset(host[i], i + 1, bytes);
    CK(hipMalloc(&dev[i], bytes));
    CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto gbps = [&](float ms) { return double(bytes) * reps / (ms * 1e-3) / 1e9; };

  for (int ns : {1, 2, 3, 6}) {
    for (int w = 0; w < 2; ++w) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dev[r % ns], host[r % ns], bytes, hipMemcpyHostToDevice, st[r % ns]));
      for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(st[i]));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (w) std::printf("{\"mode\":\"sdma\",\"streams\":%d,\"GBps\":%.2f,\"us_per_copy\":%.1f}\n", ns, gbps(ms), ms * 1e3 / reps);
    }
  }
  const size_t n16 = bytes / 16;
  for (int grid : {8, 16, 32, 64, 128, 256, 512}) {
    for (int ns : {1, 2}) {
      for (int w = 0; w < 2; ++w) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r)
          pull_kernel<<<grid, 256, 0, st[r % ns]>>>((const v4u*)host[r % ns], (v4u*)dev[r % ns], n16);
        CK(hipGetLastError());
        for (int i = 0; i < ns; ++i) CK(hipStreamSynchronize(st[i]));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (w) std::printf("{\"mode\":\"kernel\",\"grid\":%d,\"streams\":%d,\"GBps\":%.2f,\"us_per_copy\":%.1f}\n", grid, ns, gbps(ms), ms * 1e3 / reps);
      }
    }
  }
  // check the last kernel copy
  std::vector<unsigned char> chk(bytes);
  CK(hipMemcpy(chk.data(), dev[1], bytes, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < bytes; ++i) bad += chk[i] != 2;
  std::printf("{\"check_bad_bytes\":%zu}\n", bad);
  return bad != 0;
}
