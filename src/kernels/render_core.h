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
  const float fy = sy - 0.5f, fx = sx - 0.5f;
  const float y0f = floorf(fy), x0f = floorf(fx);
  const float wy = fy - y0f, wx = fx - x0f;
  const int y0 = clampi((int)y0f, 0, H - 1), y1 = clampi((int)y0f + 1, 0, H - 1);
  const int x0 = clampi((int)x0f, 0, W - 1), x1 = clampi((int)x0f + 1, 0, W - 1);
  const float a = render_src_value(d, raw, f32, x0, y0), b = render_src_value(d, raw, f32, x1, y0);
  const float c = render_src_value(d, raw, f32, x0, y1), e = render_src_value(d, raw, f32, x1, y1);
  return gray_u8(bilerp(a, b, c, e, wx, wy), win.lo, win.inv);
}

// Fused 2× render of the 8×8 canvas block (bx, by) into px[64] (row-major), for a RenderDesc
// with render_is_exact_2x(): the block's source footprint is a 6×6 patch (gray) or 4×4 (labels).
__device__ __forceinline__ void render_block_2x(const RenderDesc& d, const uint16_t* raw, const float* f32,
                                                const uint64_t* bits, RWindow win, int bx, int by, int32_t* px) {
  const int W = d.src_w, H = d.src_h;
  if (d.kind == kRenderLabels) {
    // Canvas columns 8bx..8bx+7 map to source columns 4bx..4bx+3: always inside one 64-bit word.
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float sy = render_src_coord(by * 8 + r, d.oy, d.invy);
      const int y = clampi((int)floorf(sy), 0, H - 1);
      const size_t wi = (size_t)y * d.wpr + ((4 * bx) >> 6);
      const uint64_t lab = bits[d.src_off + wi], brd = bits[d.border_off + wi];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float sx = render_src_coord(bx * 8 + c, d.ox, d.invx);
        const int x = clampi((int)floorf(sx), 0, W - 1);
        const uint64_t bit = 1ull << (x & 63);
        px[r * 8 + c] = (brd & bit) ? (int32_t)d.border_value : ((lab & bit) ? (int32_t)d.fill : 0);
      }
    }
    return;
  }
  const int sx0 = 4 * bx - 1, sy0 = 4 * by - 1;
  float patch[6][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int y = clampi(sy0 + j, 0, H - 1);
#pragma unroll
    for (int i = 0; i < 6; ++i) patch[j][i] = render_src_value(d, raw, f32, clampi(sx0 + i, 0, W - 1), y);
  }
  // Per-column and per-row interpolation weights (same expressions as render_pixel, hoisted).
  float wxs[8], wys[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float fx = render_src_coord(bx * 8 + c, d.ox, d.invx) - 0.5f;
    wxs[c] = fx - floorf(fx);
    const float fy = render_src_coord(by * 8 + c, d.oy, d.invy) - 0.5f;
    wys[c] = fy - floorf(fy);
  }
  // For an exact 2× fit floor(f) - (4b-1) == (k+1)/2; the compile-time index keeps the patch in
  // registers (a float-derived index would force it to scratch). The weights stay float-derived.
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int j0 = (r + 1) >> 1;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int i0 = (c + 1) >> 1;
      const float val =
          bilerp(patch[j0][i0], patch[j0][i0 + 1], patch[j0 + 1][i0], patch[j0 + 1][i0 + 1], wxs[c], wys[r]);
      px[r * 8 + c] = (int32_t)gray_u8(val, win.lo, win.inv);
    }
  }
}

}  // namespace nm03::gpu
