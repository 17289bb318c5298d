// K1b — IntensityNormalization + IntensityClipping (applied to the median keys; exact because
// both are monotone), ImageSharpening (9×9 Gaussian unsharp mask, main_sequential.cpp:208-210)
// and the SeededRegionGrowing band test [0.74, 0.91] (main_sequential.cpp:232-233).
//
// One workgroup = 256 threads = a 64×64 output tile; the mask radius R is a template parameter
// (compile-time tile geometry: no runtime divisions in the index math).
//  1. the clamp-to-edge (64+2R)² input tile is loaded in 8-byte groups of 4 median keys
//     (per-key clamped loads only where a group leaves the image), normalised+clipped once per
//     key and kept in LDS as f32;
//  2. vertical pass: a thread owns a column × 16 rows and slides a (16+2R)-value window held in
//     registers (each LDS value read once instead of 2R+1 times);
//  3. horizontal pass + combine + band: a thread owns 16 columns of a row (register window
//     again); the band bits of the four 16-column segments form the row's 64-bit mask word.
// The Gaussian is applied separably in the contract order of golden::sharpen (vertical, then
// horizontal, taps ascending, no FMA contraction), so the result is bit-identical to the CPU
// golden model.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

constexpr int kMaxR = 7;
static_assert(kShpTileW == 64 && kShpTileH == 64, "sharpen tile is 64x64");

template <int R>
__global__ __launch_bounds__(256) void sharpen_band_kernel(const uint16_t* __restrict__ med, uint64_t* __restrict__ band,
                                                           float* __restrict__ sharpened,
                                                           const SliceDesc* __restrict__ descs,
                                                           const TileDesc* __restrict__ tiles, PipeConsts pc,
                                                           SliceStats* stats, const uint32_t* __restrict__ tile_mm) {
  constexpr int TW = kShpTileW, TH = kShpTileH;
  constexpr int CW = TW + 2 * R, CH = TH + 2 * R;
  constexpr int CS = CW | 1;          // odd LDS row stride
  constexpr int RA = (R + 3) / 4;     // 4-key groups of halo on each side
  constexpr int G = TW / 4 + 2 * RA;  // groups per input row
  constexpr int RB = 16;              // rows per vertical-pass task
  __shared__ float C[CH * CS];
  __shared__ float T[TH * CS];
  const TileDesc t = tiles[blockIdx.x];
  const SliceDesc d = descs[t.slice];
  const int x0 = t.tx * TW, y0 = t.ty * TH;
  const int W = d.w, H = d.h;
  const uint16_t* src = med + d.raw_off;
  NormClip nc;
  nc.slope = d.slope;
  nc.intercept = d.intercept;
  nc.nmin = pc.nmin;
  nc.nmax = pc.nmax;
  nc.nlow = pc.nlow;
  nc.nhigh = pc.nhigh;
  nc.cmin = pc.cmin;
  nc.cmax = pc.cmax;

  // The slice's first tile folds the median tiles' key ranges into stats (render window).
  if (tile_mm && stats && t.tx == 0 && t.ty == 0 && threadIdx.x < 64) {
    const int ntl = ((W + kMedTileW - 1) / kMedTileW) * ((H + kMedTileH - 1) / kMedTileH);
    uint32_t a = 0xFFFFFFFFu, b = 0u;
    for (int i = threadIdx.x; i < ntl; i += 64) {
      a = min(a, tile_mm[2 * (d.med_tile0 + i)]);
      b = max(b, tile_mm[2 * (d.med_tile0 + i) + 1]);
    }
    a = wave_min_u32(a);
    b = wave_max_u32(b);
    if (threadIdx.x == 0) {
      stats[t.slice].key_min = a;
      stats[t.slice].key_max = b;
    }
  }

  // ---- 1. input tile → normalised+clipped f32 in LDS ------------------------------------------
  if ((W & 3) == 0 && (d.raw_off & 3) == 0) {
    // Window columns x0 - 4·RA + 4g + q; tile column c = 4g + q - (4·RA - R).
    for (int i = threadIdx.x; i < CH * G; i += 256) {
      const int r = i / G, g = i - r * G;
      const int y = clampi(y0 - R + r, 0, H - 1);
      const uint16_t* row = src + (size_t)y * W;
      const int xs = x0 - 4 * RA + 4 * g;
      uint16_t px[4];
      if (xs >= 0 && xs + 4 <= W) {
        const uint2 v = *reinterpret_cast<const uint2*>(row + xs);
        px[0] = (uint16_t)v.x;
        px[1] = (uint16_t)(v.x >> 16);
        px[2] = (uint16_t)v.y;
        px[3] = (uint16_t)(v.y >> 16);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) px[q] = row[clampi(xs + q, 0, W - 1)];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * g + q - (4 * RA - R);
        if (c >= 0 && c < CW) C[r * CS + c] = norm_clip_key(px[q], d.type, nc);
      }
    }
  } else {
    for (int i = threadIdx.x; i < CH * CW; i += 256) {
      const int r = i / CW, c = i - r * CW;
      const int y = clampi(y0 - R + r, 0, H - 1), x = clampi(x0 - R + c, 0, W - 1);
      C[r * CS + c] = norm_clip_key(src[(size_t)y * W + x], d.type, nc);
    }
  }
  __syncthreads();

  // ---- 2. vertical pass: column c, rows [RB·rb, RB·rb + RB) from a register window -----------
  for (int task = threadIdx.x; task < CW * (TH / RB); task += 256) {
    const int rb = task / CW, c = task - rb * CW;
    float win[RB + 2 * R];
#pragma unroll
    for (int k = 0; k < RB + 2 * R; ++k) win[k] = C[(rb * RB + k) * CS + c];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k <= 2 * R; ++k) {
        const float p = pc.taps[k] * win[rr + k];
        acc = acc + p;
      }
      T[(rb * RB + rr) * CS + c] = acc;
    }
  }
  __syncthreads();

  // ---- 3. horizontal pass + combine + band: a thread owns row r, columns [16·seg, 16·seg + 16)
  //         and slides a (16+2R)-value register window; band bits go through LDS to form the
  //         64-bit row words. Wave = segment, lane = row: a half-wave reads 32 rows at the odd
  //         stride CS, i.e. 32 distinct banks (row-major lanes put segments 0/2 and 1/3 of a row
  //         on one bank: 2-way conflicts on every read).
  __shared__ uint16_t bm[4 * TH];
  const int r = threadIdx.x & (TH - 1), seg = threadIdx.x / TH;
  const int y = y0 + r;
  float smin = INFINITY, smax = -INFINITY;
  {
    float win[16 + 2 * R];
#pragma unroll
    for (int k = 0; k < 16 + 2 * R; ++k) win[k] = T[r * CS + 16 * seg + k];
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k <= 2 * R; ++k) {
        const float p = pc.taps[k] * win[j + k];
        acc = acc + p;
      }
      const int xj = x0 + 16 * seg + j;
      const float cv = C[(r + R) * CS + 16 * seg + j + R];
      const float sv = sharpen_combine(cv, acc, pc.gain);
      const bool inside = xj < W && y < H;
      bits |= (inside && in_band(sv, pc.band_lo, pc.band_hi)) ? (1u << j) : 0u;
      if (sharpened && inside) {
        sharpened[d.f32_off + (size_t)y * W + xj] = sv;
        smin = fminf(smin, sv);
        smax = fmaxf(smax, sv);
      }
    }
    bm[seg * TH + r] = (uint16_t)bits;
  }
  __syncthreads();
  if (threadIdx.x < TH && y0 + (int)threadIdx.x < H) {
    const uint16_t* q = bm + threadIdx.x;
    const uint64_t word = (uint64_t)q[0] | ((uint64_t)q[TH] << 16) | ((uint64_t)q[2 * TH] << 32) |
                          ((uint64_t)q[3 * TH] << 48);
    band[d.mask_off + (size_t)(y0 + threadIdx.x) * d.wpr + t.tx] = word;
  }
  if (sharpened && stats) {
    uint32_t a = float_to_ordered(smin), b = float_to_ordered(smax);
    a = wave_min_u32(a);
    b = wave_max_u32(b);
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&stats[t.slice].s_min, a);
      atomicMax(&stats[t.slice].s_max, b);
    }
  }
}

void launch_sharpen_band(const uint16_t* med, uint64_t* band, float* sharpened, const SliceDesc* descs,
                         const TileDesc* tiles, int ntiles, const PipeConsts& pc, SliceStats* stats,
                         hipStream_t stream, const uint32_t* tile_mm) {
  if (ntiles <= 0) return;
#define NM03_SHARPEN_CASE(RR)                                                                              \
  case RR:                                                                                               \
    sharpen_band_kernel<RR><<<ntiles, 256, 0, stream>>>(med, band, sharpened, descs, tiles, pc, stats, tile_mm); \
    break;
  switch (pc.mask_radius) {
    NM03_SHARPEN_CASE(0)
    NM03_SHARPEN_CASE(1)
    NM03_SHARPEN_CASE(2)
    NM03_SHARPEN_CASE(3)
    NM03_SHARPEN_CASE(4)
    NM03_SHARPEN_CASE(5)
    NM03_SHARPEN_CASE(6)
    NM03_SHARPEN_CASE(7)
    default: throw DeviceError("sharpen mask must be ≤ 15");
  }
#undef NM03_SHARPEN_CASE
  check_launch("sharpen_band_kernel");
}

}  // namespace nm03::gpu
