// Render pixel math shared by K3 (canvas render) and K4 (fused 2× render inside the JPEG block
// kernel). Both paths evaluate exactly the same f32 expressions (pixel_math.h), so a fused JPEG
// is byte-identical to render-then-encode.
#pragma once

#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

struct RWindow {
  float lo, inv;  // window start and 1/(hi-lo) (pixel_math.h window_inv)
};

__device__ __forceinline__ RWindow render_window(const RenderDesc& d, const SliceStats* stats) {
  const SliceStats st = stats[d.slice];
  if (d.kind == kRenderRawGray) {
    const float a = rescaled_value((uint16_t)st.key_min, d.type, d.slope, d.intercept);
    const float b = rescaled_value((uint16_t)st.key_max, d.type, d.slope, d.intercept);
    const float lo = fminf(a, b), hi = fmaxf(a, b);
    return {lo, window_inv(lo, hi)};
  }
  const float lo = ordered_to_float(st.s_min), hi = ordered_to_float(st.s_max);
  return {lo, window_inv(lo, hi)};
}

// Source value for gray renders at clamped (x, y).
__device__ __forceinline__ float render_src_value(const RenderDesc& d, const uint16_t* raw, const float* f32, int x,
                                                  int y) {
  if (d.kind == kRenderRawGray) {
    const uint16_t r = raw[d.src_off + (size_t)y * d.src_w + x];
    return rescaled_value(key_from_raw(r, d.type, d.stored_bits), d.type, d.slope, d.intercept);
  }
  return f32[d.src_off + (size_t)y * d.src_w + x];
}

__device__ __forceinline__ uint32_t render_label_pixel(const RenderDesc& d, const uint64_t* bits, int x, int y) {
  const uint64_t bit = 1ull << (x & 63);
  const size_t wi = (size_t)y * d.wpr + (x >> 6);
  if (bits[d.border_off + wi] & bit) return d.border_value;
  return (bits[d.src_off + wi] & bit) ? d.fill : 0u;
}

// Generic per-pixel render (any geometry): canvas pixel (u, v).
__device__ __forceinline__ uint32_t render_pixel(const RenderDesc& d, const uint16_t* raw, const float* f32,
                                                 const uint64_t* bits, RWindow win, int u, int v) {
  const int W = d.src_w, H = d.src_h;
  const float sy = render_src_coord(v, d.oy, d.invy);
  const float sx = render_src_coord(u, d.ox, d.invx);
  if (!(sy >= 0.0f && sy < (float)H) || !(sx >= 0.0f && sx < (float)W)) return 0u;
  if (d.kind == kRenderLabels) {
    const int y = clampi((int)floorf(sy), 0, H - 1), x = clampi((int)floorf(sx), 0, W - 1);
    return render_label_pixel(d, bits, x, y);
  }
  if (d.filter == 1) {  // --render-filter nearest: the source pixel under the canvas pixel's centre
    const int y = clampi((int)floorf(sy), 0, H - 1), x = clampi((int)floorf(sx), 0, W - 1);
    return gray_u8(render_src_value(d, raw, f32, x, y), win.lo, win.inv);
  }
  const float fy = sy - 0.5f, fx = sx - 0.5f;
  const float y0f = floorf(fy), x0f = floorf(fx);
  const float wy = fy - y0f, wx = fx - x0f;
  const int y0 = clampi((int)y0f, 0, H - 1), y1 = clampi((int)y0f + 1, 0, H - 1);
  const int x0 = clampi((int)x0f, 0, W - 1), x1 = clampi((int)x0f + 1, 0, W - 1);
  const float a = render_src_value(d, raw, f32, x0, y0), b = render_src_value(d, raw, f32, x1, y0);
  const float c = render_src_value(d, raw, f32, x0, y1), e = render_src_value(d, raw, f32, x1, y1);
  return gray_u8(bilerp(a, b, c, e, wx, wy), win.lo, win.inv);
}

#ifndef NM03_VEC_PATCH
#define NM03_VEC_PATCH 0
#endif
constexpr bool kVecPatch = NM03_VEC_PATCH;  // 8-byte row loads measured slower (97 vs 93 us / batch)

// Exact-2× bilinear interpolation + window of one 8×8 canvas block from its 6×6 source patch
// (source rows 4by-1..4by+4, columns 4bx-1..4bx+4, edge-clamped; fetch(j, i) → f32 value) into
// px[64]. The patch is a local array filled here so it stays in registers.
template <class Fetch>
__device__ __forceinline__ void render_patch_2x(Fetch&& fetch, RWindow win, int32_t* px) {
  // Exact 2× fit: the source coordinate of canvas pixel k is 2b + k/2 - 0.25 (exact in f32), so
  // the interpolation weight is 0.75 for even and 0.25 for odd k — the very values render_pixel
  // computes — and floor(f) - (4b-1) == (k+1)/2 is a compile-time patch index.
  // Columns are processed in pairs (2m, 2m+1) as float2 so the f32 multiplies and adds map to
  // v_pk_mul_f32 / v_pk_add_f32; every element goes through exactly bilerp()'s and gray_u8()'s
  // operation sequence (no contraction), so results are bit-identical to the scalar contract.
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 wx2 = {0.75f, 0.25f}, ix2 = {1.0f - 0.75f, 1.0f - 0.25f};
  // Horizontal lerps of patch row j at canvas columns (2m, 2m+1). Output row r blends rows
  // j0 = (r+1)/2 and j0+1, so a sliding window of two lerp rows suffices (low register pressure;
  // the rows are produced in the same order and with the same operations as a full table).
  auto hrow = [&](int j, f2 (&h)[4]) {
    float row[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) row[i] = fetch(j, i);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f2 a = {row[m], row[m + 1]}, bb = {row[m + 1], row[m + 2]};
      const f2 t0 = ix2 * a;
      const f2 t1 = wx2 * bb;
      h[m] = t0 + t1;
    }
  };
  f2 h0[4], h1[4];
  hrow(0, h0);
  hrow(1, h1);
  const f2 lo2 = {win.lo, win.lo}, inv2 = {win.inv, win.inv};
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    if (r & 1) {  // j0 = (r+1)/2 advances on odd rows
#pragma unroll
      for (int m = 0; m < 4; ++m) h0[m] = h1[m];
      hrow(((r + 1) >> 1) + 1, h1);
    }
    const float wy = (r & 1) ? 0.25f : 0.75f, iy = 1.0f - wy;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const f2 u0 = iy * h0[m];
      const f2 u1 = wy * h1[m];
      const f2 val = u0 + u1;
      f2 g = val - lo2;
      g = g * inv2;
      // gray_u8's clamp to [0, 1] as one clamped v_max_f32 (g is never NaN: finite samples and
      // window). The u8 cast below is a no-op on [0.5, 255.5] but keeps the allocation at 127
      // VGPRs (without it the encoder spills to scratch).
      g.x = __builtin_amdgcn_fmed3f(g.x, 0.0f, 1.0f);
      g.y = __builtin_amdgcn_fmed3f(g.y, 0.0f, 1.0f);
      f2 t = g * 255.0f;
      t = t + 0.5f;
      px[r * 8 + 2 * m] = (int32_t)(uint8_t)(int)t.x;
      px[r * 8 + 2 * m + 1] = (int32_t)(uint8_t)(int)t.y;
    }
  }
}

// --render-filter nearest on an exact 2× fit: canvas pixel (8bx + c, 8by + r) samples source
// (4bx + c/2, 4by + r/2) — floor of its centre's source coordinate, render_pixel's nearest path —
// which is patch element (r/2 + 1, c/2 + 1): 16 distinct values, each covering a 2×2 canvas cell.
template <class Fetch>
__device__ __forceinline__ void render_patch_2x_nearest(Fetch&& fetch, RWindow win, int32_t* px) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int32_t g = (int32_t)gray_u8(fetch(j + 1, i + 1), win.lo, win.inv);
      px[(2 * j) * 8 + 2 * i] = g;
      px[(2 * j) * 8 + 2 * i + 1] = g;
      px[(2 * j + 1) * 8 + 2 * i] = g;
      px[(2 * j + 1) * 8 + 2 * i + 1] = g;
    }
}

// Exact-2× label render of the 8×8 canvas block (bx, by): canvas columns 8bx..8bx+7 map to source
// columns 4bx..4bx+3, always inside one 64-bit word k = 4bx/64 of the label and border rows;
// words(y, k, lab, brd) returns word k of source row y (edge-clamped row index).
template <class Words>
__device__ __forceinline__ void render_labels_2x(const RenderDesc& d, Words&& words, int bx, int by, int32_t* px) {
  const int W = d.src_w, H = d.src_h;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const float sy = render_src_coord(by * 8 + r, d.oy, d.invy);
    const int y = clampi((int)floorf(sy), 0, H - 1);
    uint64_t lab, brd;
    words(y, (4 * bx) >> 6, lab, brd);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float sx = render_src_coord(bx * 8 + c, d.ox, d.invx);
      const int x = clampi((int)floorf(sx), 0, W - 1);
      const uint64_t bit = 1ull << (x & 63);
      px[r * 8 + c] = (brd & bit) ? (int32_t)d.border_value : ((lab & bit) ? (int32_t)d.fill : 0);
    }
  }
}

// render_labels_2x for a fit known to be exactly 2× (render_is_exact_2x: origin 0, scale 1/2):
// canvas (8bx + c, 8by + r) samples source (4bx + c/2, 4by + r/2), so the block is 4 × 4 cells of
// 2 × 2 equal pixels, one nibble of one word per source row — 16 bit tests instead of 64 (the
// generic form evaluates every pixel's source coordinate). Same values as render_labels_2x.
template <class Words>
__device__ __forceinline__ void render_labels_exact2x(const RenderDesc& d, Words&& words, int bx, int by, int32_t* px) {
  const int sh = (4 * bx) & 63;
#pragma unroll
  for (int r2 = 0; r2 < 4; ++r2) {
    uint64_t lab, brd;
    words(4 * by + r2, (4 * bx) >> 6, lab, brd);
    const uint32_t nl = (uint32_t)(lab >> sh), nb = (uint32_t)(brd >> sh);
#pragma unroll
    for (int c2 = 0; c2 < 4; ++c2) {
      const int32_t v = ((nb >> c2) & 1u) ? (int32_t)d.border_value : (((nl >> c2) & 1u) ? (int32_t)d.fill : 0);
      px[(2 * r2) * 8 + 2 * c2] = v;
      px[(2 * r2) * 8 + 2 * c2 + 1] = v;
      px[(2 * r2 + 1) * 8 + 2 * c2] = v;
      px[(2 * r2 + 1) * 8 + 2 * c2 + 1] = v;
    }
  }
}

// Fused 2× render of the 8×8 canvas block (bx, by) into px[64] (row-major), for a RenderDesc
// with render_is_exact_2x(): the block's source footprint is a 6×6 patch (gray) or 4×4 (labels).
// kNearest: gray renders with --render-filter nearest (a compile-time choice: the bilinear encoder's
// code stays as it was).
template <bool kNearest = false>
__device__ __forceinline__ void render_block_2x(const RenderDesc& d, const uint16_t* raw, const float* f32,
                                                const uint64_t* bits, RWindow win, int bx, int by, int32_t* px,
                                                bool synth_src = false) {
  const int W = d.src_w, H = d.src_h;
  if (d.kind == kRenderLabels) {
    render_labels_2x(d, [&](int y, int k, uint64_t& lab, uint64_t& brd) {
      const size_t wi = (size_t)y * d.wpr + k;
      lab = bits[d.src_off + wi];
      brd = bits[d.border_off + wi];
    }, bx, by, px);
    return;
  }
  const int sx0 = 4 * bx - 1, sy0 = 4 * by - 1;
  float patch[6][6];
  if (kVecPatch && d.kind == kRenderRawGray && sx0 >= 1 && sx0 + 6 <= W && !(W & 1)) {
    // Interior columns: the patch row plus one sample either side is 8 contiguous 4-byte-aligned
    // u16 (source column 4bx-2 is even, rows are even-sized) → two 8-byte loads per row.
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int y = clampi(sy0 + j, 0, H - 1);
      const uint2* p = reinterpret_cast<const uint2*>(raw + d.src_off + (size_t)y * W + (sx0 - 1));
      const uint2 lo = p[0], hi = p[1];
      const uint32_t wv[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const uint32_t word = wv[(i + 1) >> 1];
        const uint16_t r = (uint16_t)((i + 1) & 1 ? (word >> 16) : (word & 0xFFFFu));
        patch[j][i] = rescaled_value(key_from_raw(r, d.type, d.stored_bits), d.type, d.slope, d.intercept);
      }
    }
  } else if (synth_src) {  // synthetic source (no loads): same math; kept for kernel experiments
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int i = 0; i < 6; ++i) patch[j][i] = (float)((sx0 + i) * 3 + (sy0 + j) * 5) * win.inv;
  } else {
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int y = clampi(sy0 + j, 0, H - 1);
#pragma unroll
      for (int i = 0; i < 6; ++i) patch[j][i] = render_src_value(d, raw, f32, clampi(sx0 + i, 0, W - 1), y);
    }
  }
  if (kNearest)
    render_patch_2x_nearest([&](int j, int i) { return patch[j][i]; }, win, px);
  else
    render_patch_2x([&](int j, int i) { return patch[j][i]; }, win, px);
}

}  // namespace nm03::gpu
