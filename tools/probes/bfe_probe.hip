// Checks on the GPU that the JPEG staging's bit-field-extract conversion equals
// rescaled_value(key_from_raw(r)) for every 16-bit sample, pixel type and stored-bit count.
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -Iinclude tools/probes/bfe_probe.hip -o build/bin/bfe_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#include "nm03/common.h"
#include "nm03/pixel_math.h"

using namespace nm03;

__global__ void probe(int type, int sb, float slope, float intercept, unsigned* bad, unsigned* first) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= 65536u) return;
  const float ref = rescaled_value(key_from_raw((uint16_t)r, (uint8_t)type, (uint8_t)sb), (uint8_t)type, slope, intercept);
  const bool sgn = type == kI16, affine = slope != 1.0f || intercept != 0.0f;
  const uint32_t sbits = (uint32_t)sb;
  // The first form of the JPEG staging conversion (miscompiled for signed data: the select of the
  // two conversions became one unsigned conversion)...
  float x = sgn ? (float)__builtin_amdgcn_sbfe((int)r, 0u, sbits) : (float)__builtin_amdgcn_ubfe(r, 0u, sbits);
  // ... and the shipped one.
  const uint32_t vsh = 32u - sbits, up = r << vsh;
  float y = (float)(sgn ? (int32_t)up >> vsh : (int32_t)(up >> vsh));
  if (affine) {
    const float t = y * slope;
    y = t + intercept;
  }
  if (__float_as_uint(y) != __float_as_uint(ref)) atomicAdd(bad + 1, 1u);
  if (affine) {
    const float t = x * slope;
    x = t + intercept;
  }
  if (__float_as_uint(x) != __float_as_uint(ref)) {
    atomicAdd(bad, 1u);
    atomicMin(first, r);
  }
}

int main() {
  unsigned *bad, *first;
  if (hipMallocManaged(&bad, 8) != hipSuccess || hipMallocManaged(&first, 4) != hipSuccess) return 2;
  const int types[3] = {kU16, kI16, kU8};
  const int bits[4] = {8, 12, 15, 16};
  int total = 0;
  for (int t : types)
    for (int b : bits)
      for (int a = 0; a < 2; ++a) {
        bad[0] = bad[1] = 0;
        *first = 0xFFFFFFFFu;
        probe<<<256, 256>>>(t, b, a ? 1.5f : 1.0f, a ? 100.0f : 0.0f, bad, first);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        std::printf("type %d bits %2d affine %d: bfe-intrinsic form mismatches %u (first r = %u), shipped form %u\n", t, b,
                    a, bad[0], *first, bad[1]);
        total += bad[1] != 0;
      }
  std::printf("%s\n", total ? "MISMATCH in the shipped form" : "shipped form equal everywhere");
  return 0;
}
