// Device-side helpers shared by the gfx950 kernels (wave64 reductions/scans, ordered floats).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "nm03/common.h"

namespace nm03::gpu {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 vmin(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 vmax(u16x2 a, u16x2 b) { return __builtin_elementwise_max(a, b); }

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }

// f32 ↔ order-preserving u32 (for atomicMin/atomicMax on floats).
__host__ __device__ __forceinline__ uint32_t float_to_ordered(float f) {
  uint32_t u = __builtin_bit_cast(uint32_t, f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ __forceinline__ float ordered_to_float(uint32_t u) {
  u = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
  return __builtin_bit_cast(float, u);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Inclusive wave scan (sum) of uint32.
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Block-wide exclusive scan for blockDim.x ≤ 1024 (multiple of 64). `sh` needs 17 uint32.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t inc = wave_inclusive_scan(v, lane);
  if (lane == 63) sh[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    uint32_t w = lane < nw ? sh[lane] : 0u;
    uint32_t wi = wave_inclusive_scan(w, lane);
    if (lane < nw) sh[lane] = wi - w;
    if (lane == nw - 1) sh[16] = wi;
  }
  __syncthreads();
  uint32_t res = inc - v + sh[wave];
  *total = sh[16];
  __syncthreads();
  return res;
}

// 64×64 bit-matrix transpose across a wave: lane l holds row l (bit c = column c) and receives
// column l. Six butterfly stages of off-diagonal block swaps.
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, int lane) {
  const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                             0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int j = 32 >> s;
    const uint64_t m = masks[s];
    const uint64_t other = __shfl_xor(x, j, 64);
    if ((lane & j) == 0) {
      const uint64_t t = ((x >> j) ^ other) & m;
      x ^= t << j;
    } else {
      const uint64_t t = ((other >> j) ^ x) & m;
      x ^= t;
    }
  }
  return x;
}

}  // namespace nm03::gpu
