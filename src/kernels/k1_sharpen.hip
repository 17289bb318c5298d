// K1b — IntensityNormalization + IntensityClipping (applied to the median keys; exact because
// both are monotone), ImageSharpening (9×9 Gaussian unsharp mask, main_sequential.cpp:208-210)
// and the SeededRegionGrowing band test [0.74, 0.91] (main_sequential.cpp:232-233).
//
// One workgroup = 256 threads = a 64×16 output tile. Lane = column, so the band test of a row
// is one __ballot → one 64-bit mask word (no bit packing pass). The clamp-to-edge input tile
// (16+2R)×(64+2R) f32 and the vertical-pass tile live in LDS; the Gaussian is applied
// separably in the contract order of golden::sharpen (vertical, then horizontal, taps ascending,
// no FMA contraction), so the result is bit-identical to the CPU golden model.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

constexpr int kMaxR = 7;
constexpr int kCW = kShpTileW + 2 * kMaxR;  // 78
constexpr int kCS = kCW + 1;                // LDS row stride (odd)

__global__ __launch_bounds__(256) void sharpen_band_kernel(const uint16_t* __restrict__ med, uint64_t* __restrict__ band,
                                                           float* __restrict__ sharpened,
                                                           const SliceDesc* __restrict__ descs,
                                                           const TileDesc* __restrict__ tiles, PipeConsts pc,
                                                           SliceStats* stats, const uint32_t* __restrict__ tile_mm) {
  __shared__ float C[(kShpTileH + 2 * kMaxR) * kCS];
  __shared__ float T[kShpTileH * kCS];
  const TileDesc t = tiles[blockIdx.x];
  const SliceDesc d = descs[t.slice];
  const int R = pc.mask_radius;
  const int cw = kShpTileW + 2 * R, ch = kShpTileH + 2 * R;
  const int x0 = t.tx * kShpTileW, y0 = t.ty * kShpTileH;
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
  for (int i = threadIdx.x; i < ch * cw; i += 256) {
    const int r = i / cw, c = i - r * cw;
    const int y = clampi(y0 - R + r, 0, H - 1), x = clampi(x0 - R + c, 0, W - 1);
    C[r * kCS + c] = norm_clip_key(src[(size_t)y * W + x], d.type, nc);
  }
  __syncthreads();
  // Vertical pass for the 16 output rows over all cw columns.
  for (int i = threadIdx.x; i < kShpTileH * cw; i += 256) {
    const int r = i / cw, c = i - r * cw;
    float acc = 0.0f;
    for (int k = 0; k <= 2 * R; ++k) {
      const float p = pc.taps[k] * C[(r + k) * kCS + c];
      acc = acc + p;
    }
    T[r * kCS + c] = acc;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float smin = INFINITY, smax = -INFINITY;
  for (int rr = wave * 4; rr < wave * 4 + 4; ++rr) {
    float acc = 0.0f;
    for (int k = 0; k <= 2 * R; ++k) {
      const float p = pc.taps[k] * T[rr * kCS + lane + k];
      acc = acc + p;
    }
    const float c = C[(rr + R) * kCS + lane + R];
    const float s = sharpen_combine(c, acc, pc.gain);
    const int x = x0 + lane, y = y0 + rr;
    const bool inside = x < W && y < H;
    const unsigned long long word = __ballot(inside && in_band(s, pc.band_lo, pc.band_hi));
    if (y < H && lane == 0) band[d.mask_off + (size_t)y * d.wpr + t.tx] = word;
    if (sharpened && inside) {
      sharpened[d.f32_off + (size_t)y * W + x] = s;
      smin = fminf(smin, s);
      smax = fmaxf(smax, s);
    }
  }
  if (sharpened && stats) {
    uint32_t a = float_to_ordered(smin), b = float_to_ordered(smax);
    a = wave_min_u32(a);
    b = wave_max_u32(b);
    if (lane == 0) {
      atomicMin(&stats[t.slice].s_min, a);
      atomicMax(&stats[t.slice].s_max, b);
    }
  }
}

void launch_sharpen_band(const uint16_t* med, uint64_t* band, float* sharpened, const SliceDesc* descs,
                         const TileDesc* tiles, int ntiles, const PipeConsts& pc, SliceStats* stats,
                         hipStream_t stream, const uint32_t* tile_mm) {
  if (ntiles <= 0) return;
  if (pc.mask_radius < 0 || pc.mask_radius > kMaxR) throw DeviceError("sharpen mask must be ≤ 15");
  sharpen_band_kernel<<<ntiles, 256, 0, stream>>>(med, band, sharpened, descs, tiles, pc, stats, tile_mm);
  check_launch("sharpen_band_kernel");
}

}  // namespace nm03::gpu
