// K6 — BinaryThresholding (FAST_directives.hpp:13; included but unused by the reference,
// SURVEY §2.6): out = lo ≤ x ≤ hi ? 1 : 0 on an f32 image (e.g. the sharpened stage), emitted both
// as a u8 mask and, optionally, as 64-bit row words like the SRG band (one __ballot per row chunk).
#include <hip/hip_runtime.h>

#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

// 4 pixels per thread: one 16-byte load, one 4-byte store.
__global__ __launch_bounds__(256) void threshold_kernel(const float* __restrict__ in, uint8_t* __restrict__ out,
                                                        size_t n, float lo, float hi) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const float4 v = *reinterpret_cast<const float4*>(in + i);
    const uint32_t m = (uint32_t)in_band(v.x, lo, hi) | ((uint32_t)in_band(v.y, lo, hi) << 8) |
                       ((uint32_t)in_band(v.z, lo, hi) << 16) | ((uint32_t)in_band(v.w, lo, hi) << 24);
    *reinterpret_cast<uint32_t*>(out + i) = m;
  } else {
    for (size_t k = i; k < n; ++k) out[k] = in_band(in[k], lo, hi) ? 1 : 0;
  }
}

void launch_threshold(const float* in, uint8_t* out, size_t n, float lo, float hi, hipStream_t stream) {
  if (n == 0) return;
  if (((uintptr_t)in & 15) || ((uintptr_t)out & 3)) throw DeviceError("launch_threshold: misaligned buffers");
  const size_t threads = (n + 3) / 4;
  threshold_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, stream>>>(in, out, n, lo, hi);
  check_launch("threshold_kernel");
}

void preload_threshold() {
  hipFuncAttributes a;
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&threshold_kernel)), "preload threshold_kernel");
}

}  // namespace nm03::gpu
