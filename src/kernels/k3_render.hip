// K3 — RenderToImage(Black, 512, 512) of ImageRenderer / SegmentationRenderer
// (main_sequential.cpp:255-262, main_parallel.cpp:183-210), as a kernel.
//   kRenderRawGray : bilinear sample of the modality-rescaled original, window = slice min/max
//                    (from the per-slice key range reduced by K1a).
//   kRenderF32Gray : same on the f32 sharpened image (test_pipeline "preprocessed_image").
//   kRenderLabels  : nearest label sample; label → 0.6·255, border (radius 2, from K2) → 255.
// Each thread produces 4 horizontally adjacent canvas pixels (one 32-bit store).
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "render_core.h"
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
  const RWindow win = d.kind == kRenderLabels ? RWindow{0.f, 0.f} : render_window(d, stats);
  uint32_t packed = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) packed |= render_pixel(d, raw, f32, bits, win, u0 + k, v) << (8 * k);
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

void preload_render() {
  hipFuncAttributes a;
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&render_kernel)), "preload render_kernel");
}

}  // namespace nm03::gpu
