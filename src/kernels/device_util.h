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

// x of lane (lane ^ J), without the LDS crossbar: v_permlane32_swap / v_permlane16_swap (gfx950)
// for J = 32 / 16, DPP row rotates for J = 8 / 4 (row_ror:N = from lane − N within a 16-lane
// row) and DPP quad permutes for J = 2 / 1. Each is 1–3 VALU ops; a ds_bpermute_b32 round trip
// costs ~100 cycles, and the bit transposes below chain six of them.
template <int J>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, int lane) {
  if constexpr (J == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // {dst', src'}
    return (lane & 32) ? r[0] : r[1];
  } else if constexpr (J == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else if constexpr (J == 8) {
    return __builtin_amdgcn_update_dpp(0u, x, 0x128, 0xF, 0xF, true);  // row_ror:8
  } else if constexpr (J == 4) {
    const uint32_t from_lo = __builtin_amdgcn_update_dpp(0u, x, 0x124, 0xF, 0xF, true);  // row_ror:4  (lane − 4)
    const uint32_t from_hi = __builtin_amdgcn_update_dpp(0u, x, 0x12C, 0xF, 0xF, true);  // row_ror:12 (lane + 4)
    return (lane & 4) ? from_lo : from_hi;
  } else if constexpr (J == 2) {
    return __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  } else {
    static_assert(J == 1, "lane_xor: J in {1,2,4,8,16,32}");
    return __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  }
}

template <int J>
__device__ __forceinline__ void transpose_stage(uint64_t& x, int lane, uint64_t m) {
  const uint64_t other = ((uint64_t)lane_xor<J>((uint32_t)(x >> 32), lane) << 32) | lane_xor<J>((uint32_t)x, lane);
  if ((lane & J) == 0) {
    const uint64_t t = ((x >> J) ^ other) & m;
    x ^= t << J;
  } else {
    const uint64_t t = ((other >> J) ^ x) & m;
    x ^= t;
  }
}

// 64×64 bit-matrix transpose across a wave: lane l holds row l (bit c = column c) and receives
// column l. Six butterfly stages of off-diagonal block swaps; the 32-block stage (lanes < 32 take
// the partner's low half into their high half and vice versa) is exactly one v_permlane32_swap of
// (lo, hi). All stages stay in VALU (the r2 form was 12 dependent ds_bpermute_b32).
__device__ __forceinline__ uint64_t wave_transpose64(uint64_t x, int lane) {
  {
    const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)x, (uint32_t)(x >> 32), false, false);
    x = ((uint64_t)r[1] << 32) | r[0];
  }
  transpose_stage<16>(x, lane, 0x0000FFFF0000FFFFull);
  transpose_stage<8>(x, lane, 0x00FF00FF00FF00FFull);
  transpose_stage<4>(x, lane, 0x0F0F0F0F0F0F0F0Full);
  transpose_stage<2>(x, lane, 0x3333333333333333ull);
  transpose_stage<1>(x, lane, 0x5555555555555555ull);
  return x;
}

}  // namespace nm03::gpu
