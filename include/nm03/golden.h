// nm03/golden.h — single-threaded CPU golden model of every pipeline stage (SURVEY §1.2 L1',
// App. A). It is the test oracle for the HIP kernels and the `--cpu` plumbing path of
// test_pipeline (BASELINE config 1). It is NOT a backend: the engine never falls back to it.
//
// Stage ↔ reference call site:
//   norm_clip        IntensityNormalization + IntensityClipping  main_sequential.cpp:195-202
//   median           VectorMedianFilter(7)                       main_sequential.cpp:204-206
//   sharpen          ImageSharpening(2.0, 0.5, 9)                main_sequential.cpp:208-210
//   region_grow      SeededRegionGrowing(0.74, 0.91, seeds)      main_sequential.cpp:232-243
//   dilate / erode   ImageCaster(UINT8) + Dilation(3) / Erosion(3) main_sequential.cpp:246-252
//   render_*         ImageRenderer / SegmentationRenderer / RenderToImage(512²)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "nm03/common.h"
#include "nm03/params.h"
#include "nm03/pixel_math.h"

namespace nm03::golden {

struct SliceInput {
  int w = 0, h = 0;
  PixelType type = kU16;
  int stored_bits = 16;
  float slope = 1.f, intercept = 0.f;
  float spacing_x = 1.f, spacing_y = 1.f;
  std::vector<uint16_t> raw;  // raw 16-bit samples, row-major
};

// DICOM import (setLoadSeries(false)); applies the <100 guard when `min_dim` > 0.
// `frame`: dicom::select_frame policy (-1 rejects multi-frame files, k ≥ 0 imports frame k).
SliceInput load_slice(const std::string& path, int min_dim, int frame = -1);

NormClip make_normclip(const SliceInput& s, const PipelineParams& p);

std::vector<uint16_t> keys(const SliceInput& s);
std::vector<float> norm_clip(const SliceInput& s, const PipelineParams& p);
// Rescaled (modality) values used by the original-image renderer.
std::vector<float> rescaled(const SliceInput& s, const PipelineParams& p);

// Exact k×k median with clamp-to-edge (A.4).
std::vector<float> median(const std::vector<float>& img, int w, int h, int k);
std::vector<uint16_t> median_u16(const std::vector<uint16_t>& img, int w, int h, int k);
// FAST's vector-median definition (argmin_k Σ_j |w_k − w_j|, first in scan order on ties).
std::vector<float> vector_median(const std::vector<float>& img, int w, int h, int k);

// Unsharp mask with the separable contract (vertical then horizontal, taps ascending).
std::vector<float> sharpen(const std::vector<float>& img, int w, int h, float gain, float sigma, int mask);
// FAST's direct 2D mask form (for tolerance tests only).
std::vector<float> sharpen_direct(const std::vector<float>& img, int w, int h, float gain, float sigma, int mask);

std::vector<uint8_t> band(const std::vector<float>& s, float lo, float hi);
// BinaryThresholding (lo ≤ x ≤ hi → 1): the band test as a standalone op (k6_threshold.hip).
inline std::vector<uint8_t> binary_threshold(const std::vector<float>& s, float lo, float hi) { return band(s, lo, hi); }

// Seeded region growing: pixels connected (4 or 8) to an in-band seed through in-band pixels.
std::vector<uint8_t> region_grow(const std::vector<uint8_t>& band, int w, int h, const std::vector<Seed>& seeds,
                                 int connectivity);
// Square structuring element of odd `size`, out-of-image samples ignored (A.7).
// `disc`: the digital disc of radius size/2 (PipelineParams::se_shape) instead of the square.
std::vector<uint8_t> dilate(const std::vector<uint8_t>& m, int w, int h, int size, bool disc = false);
std::vector<uint8_t> erode(const std::vector<uint8_t>& m, int w, int h, int size, bool disc = false);
// SegmentationRenderer border: label pixels with a 0 within Chebyshev radius r (image space).
std::vector<uint8_t> border(const std::vector<uint8_t>& m, int w, int h, int radius);

// 3D variants (BASELINE config 5): 6/26-connected region growing, cube dilation.
std::vector<uint8_t> region_grow3d(const std::vector<uint8_t>& band, int w, int h, int d,
                                   const std::vector<Seed>& seeds, int connectivity);
// `ball`: the digital ball of radius size/2 instead of the size³ cube.
std::vector<uint8_t> dilate3d(const std::vector<uint8_t>& m, int w, int h, int d, int size, bool ball = false);

// Renderers (A.9) onto an out_w×out_h black canvas.
// `nearest`: RenderParams::filter == kFilterNearest (the source pixel under each canvas pixel's centre).
std::vector<uint8_t> render_gray(const std::vector<float>& values, const RenderGeom& g, float lo, float hi,
                                 bool nearest = false);
std::vector<uint8_t> render_labels(const std::vector<uint8_t>& label, const std::vector<uint8_t>& border_mask,
                                   const RenderGeom& g, uint8_t fill, uint8_t border_value);

struct SliceResult {
  std::vector<float> clipped, median, sharpened;
  std::vector<uint8_t> band, region, eroded, dilated;
  float window_lo = 0, window_hi = 0;  // original render window (rescaled min/max)
};

SliceResult run(const SliceInput& s, const PipelineParams& p, bool with_erosion);

// Render + JPEG of the two exported images of seq/par (original, processed).
struct SliceJpegs {
  std::vector<uint8_t> original, processed;
};
SliceJpegs export_jpegs(const SliceInput& s, const SliceResult& r, const PipelineParams& p, const RenderParams& rp);

// test_pipeline's five stage images (test_pipeline.cpp:164-179): original, preprocessed,
// segmentation, erosion, dilation — canvases and their JPEG files.
struct StageImages {
  std::vector<std::vector<uint8_t>> canvases, jpegs;
};
// `stages` (optional) receives the intermediate arrays (for --dump-mhd).
StageImages test_pipeline_images(const SliceInput& s, const PipelineParams& p, const RenderParams& rp,
                                 SliceResult* stages = nullptr);

}  // namespace nm03::golden
