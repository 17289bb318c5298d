// K3 — RenderToImage(Black, 512, 512) of ImageRenderer / SegmentationRenderer
// (main_sequential.cpp:255-262, main_parallel.cpp:183-210), as a kernel.
//   kRenderRawGray : bilinear sample of the modality-rescaled original, window = slice min/max
//                    (from the per-slice key range reduced by K1a).
//   kRenderF32Gray : same on the f32 sharpened image (test_pipeline "preprocessed_image").
//   kRenderLabels  : nearest label sample; label → 0.6·255, border (radius 2, from K2) → 255.
// Each thread produces 4 horizontally adjacent canvas pixels (one 32-bit store).
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

__global__ __launch_bounds__(256) void render_kernel(const uint16_t* __restrict__ raw, const float* __restrict__ f32,
                                                     const uint64_t* __restrict__ bits,
                                                     const SliceStats* __restrict__ stats,
                                                     const RenderDesc* __restrict__ rds, int out_w, int out_h,
                                                     uint8_t* __restrict__ canvas) {
  const RenderDesc d = rds[blockIdx.y];
  const int qpr = out_w >> 2;
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int v = q / qpr;
  if (v >= out_h) return;
  const int u0 = (q - v * qpr) * 4;
  const int W = d.src_w, H = d.src_h;
  uint32_t packed = 0;
  const float sy = render_src_coord(v, d.oy, d.invy);
  const bool row_in = sy >= 0.0f && sy < (float)H;
  if (row_in) {
    if (d.kind == kRenderLabels) {
      const int y = clampi((int)floorf(sy), 0, H - 1);
      const uint64_t* lab = bits + d.src_off + (size_t)y * d.wpr;
      const uint64_t* brd = bits + d.border_off + (size_t)y * d.wpr;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float sx = render_src_coord(u0 + k, d.ox, d.invx);
        if (!(sx >= 0.0f && sx < (float)W)) continue;
        const int x = clampi((int)floorf(sx), 0, W - 1);
        const uint64_t bit = 1ull << (x & 63);
        const uint32_t val = (brd[x >> 6] & bit) ? d.border_value : ((lab[x >> 6] & bit) ? d.fill : 0u);
        packed |= val << (8 * k);
      }
    } else {
      float lo, hi;
      const SliceStats st = stats[d.slice];
      if (d.kind == kRenderRawGray) {
        const float a = rescaled_value((uint16_t)st.key_min, d.type, d.slope, d.intercept);
        const float b = rescaled_value((uint16_t)st.key_max, d.type, d.slope, d.intercept);
        lo = fminf(a, b);
        hi = fmaxf(a, b);
      } else {
        lo = ordered_to_float(st.s_min);
        hi = ordered_to_float(st.s_max);
      }
      const float fy = sy - 0.5f;
      const float y0f = floorf(fy);
      const float wy = fy - y0f;
      const int y0 = clampi((int)y0f, 0, H - 1), y1 = clampi((int)y0f + 1, 0, H - 1);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float sx = render_src_coord(u0 + k, d.ox, d.invx);
        if (!(sx >= 0.0f && sx < (float)W)) continue;
        const float fx = sx - 0.5f;
        const float x0f = floorf(fx);
        const float wx = fx - x0f;
        const int x0 = clampi((int)x0f, 0, W - 1), x1 = clampi((int)x0f + 1, 0, W - 1);
        float a, b, c, e;
        if (d.kind == kRenderRawGray) {
          const uint16_t* s = raw + d.src_off;
          a = rescaled_value(key_from_raw(s[(size_t)y0 * W + x0], d.type, d.stored_bits), d.type, d.slope, d.intercept);
          b = rescaled_value(key_from_raw(s[(size_t)y0 * W + x1], d.type, d.stored_bits), d.type, d.slope, d.intercept);
          c = rescaled_value(key_from_raw(s[(size_t)y1 * W + x0], d.type, d.stored_bits), d.type, d.slope, d.intercept);
          e = rescaled_value(key_from_raw(s[(size_t)y1 * W + x1], d.type, d.stored_bits), d.type, d.slope, d.intercept);
        } else {
          const float* s = f32 + d.src_off;
          a = s[(size_t)y0 * W + x0];
          b = s[(size_t)y0 * W + x1];
          c = s[(size_t)y1 * W + x0];
          e = s[(size_t)y1 * W + x1];
        }
        const float val = bilerp(a, b, c, e, wx, wy);
        packed |= (uint32_t)gray_u8(val, lo, hi) << (8 * k);
      }
    }
  }
  *reinterpret_cast<uint32_t*>(canvas + d.canvas_off + (size_t)v * out_w + u0) = packed;
}

void launch_render(const uint16_t* raw, const float* f32, const uint64_t* bits, const SliceStats* stats,
                   const RenderDesc* rd, int ncanvas, int out_w, int out_h, uint8_t* canvas, hipStream_t stream) {
  if (ncanvas <= 0) return;
  if (out_w % 4) throw DeviceError("canvas width must be a multiple of 4");
  const int quads = out_w / 4 * out_h;
  dim3 grid((quads + 255) / 256, ncanvas);
  render_kernel<<<grid, 256, 0, stream>>>(raw, f32, bits, stats, rd, out_w, out_h, canvas);
  check_launch("render_kernel");
}

}  // namespace nm03::gpu
