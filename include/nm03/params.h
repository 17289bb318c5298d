// nm03/params.h — pipeline parameters. Defaults are the literals hard-coded in the reference
// (SURVEY.md §2.7): main_sequential.cpp:196-262, test_pipeline.cpp:55-125, main_parallel.cpp:33,401.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "nm03/common.h"

namespace nm03 {

struct PipelineParams {
  // IntensityNormalization::create(0.5f, 2.5f, 0.0f, 10000.0f)   main_sequential.cpp:195-198
  float norm_low = 0.5f;
  float norm_high = 2.5f;
  float norm_min = 0.0f;
  float norm_max = 10000.0f;
  // IntensityClipping::create(0.68f, 4000.0f)                      main_sequential.cpp:200-202
  float clip_min = 0.68f;
  float clip_max = 4000.0f;
  // VectorMedianFilter::create(7)                                  main_sequential.cpp:204-206
  int median_window = 7;
  // ImageSharpening::create(2.0f, 0.5f, 9)                         main_sequential.cpp:208-210
  float sharpen_gain = 2.0f;
  float sharpen_sigma = 0.5f;
  int sharpen_mask = 9;
  // SeededRegionGrowing::create(0.74f, 0.91f, seeds)              main_sequential.cpp:232-243
  float srg_min = 0.74f;
  float srg_max = 0.91f;
  int srg_connectivity = 4;  // 4 | 8 in 2D (6 | 26 in 3D)
  // Dilation::create(3) / Erosion::create(3)                      main_sequential.cpp:250, test_pipeline.cpp:119
  int dilation_size = 3;
  int erosion_size = 3;
  // Structuring element of Dilation/Erosion (2D) and of the 3D dilation: FAST's shape is not pinned
  // by the reference (SURVEY App. A.7 / §7.6 risk 1), so it is a flag. kSeSquare (default): the
  // size×size square / size³ cube; kSeDisc: the digital disc / ball of radius r = size/2, i.e. the
  // offsets with dx² + dy² (+ dz²) ≤ r² (size 3: the 4-neighbour cross). Out-of-image samples are
  // ignored either way.
  int se_shape = 0;
  // Reject slices with width<100 || height<100                    main_sequential.cpp:189-192
  int min_dim = 100;
  // Apply DICOM modality rescale (slope/intercept) if present.
  bool apply_rescale = true;
  // Multi-frame files (dicom::select_frame): -1 rejects them (default), k ≥ 0 imports frame k.
  int frame = -1;
};

enum SeShape : int { kSeSquare = 0, kSeDisc = 1 };

struct RenderParams {
  // RenderToImage::create(Color::Black(), 512, 512)               main_sequential.cpp:258
  int out_width = 512;
  int out_height = 512;
  // SegmentationRenderer::create(labelColors{1:White}, 0.6f, 1.0f, 2)  main_sequential.cpp:255-262
  float label_opacity = 0.6f;
  float border_opacity = 1.0f;
  int border_radius = 2;
  // ImageFileExporter .jpg → Qt/libjpeg default quality 75.
  int jpeg_quality = 75;
  // Interpolation of the gray renders (original / preprocessed image; labels are always nearest):
  // FAST's ImageRenderer filtering is not pinned by the reference (main_sequential.cpp:259), so it is
  // a flag (--render-filter). kFilterBilinear (default) or kFilterNearest.
  int filter = 0;
  // Component layout of the JPEG files (jpeg::Sampling, --jpeg-sampling): YCbCr 4:2:0 (default),
  // 4:4:4, or a one-component gray file — which one Qt writes for FAST's image is not pinned.
  int jpeg_sampling = 0;
};

enum RenderFilter : int { kFilterBilinear = 0, kFilterNearest = 1 };

// Adaptive seed points of the reference (main_sequential.cpp:214-241): centre, centre ± (W/8, H/8)
// and a grid x∈[W/4, 3W/4) step W/10 (same for y). Integer division as in the reference.
// The step is clamped to ≥1 (width<10 would loop forever in the reference).
struct Seed {
  int32_t x, y, z;
};

inline std::vector<Seed> reference_seeds(int width, int height) {
  std::vector<Seed> s;
  const int cx = width / 2, cy = height / 2;
  const int ox = width / 8, oy = height / 8;
  s.push_back({cx, cy, 0});
  s.push_back({cx + ox, cy, 0});
  s.push_back({cx - ox, cy, 0});
  s.push_back({cx, cy + oy, 0});
  s.push_back({cx, cy - oy, 0});
  const int sx = width / 10 > 0 ? width / 10 : 1;
  const int sy = height / 10 > 0 ? height / 10 : 1;
  for (int x = width / 4; x < width * 3 / 4; x += sx)
    for (int y = height / 4; y < height * 3 / 4; y += sy) s.push_back({x, y, 0});
  return s;
}

}  // namespace nm03
