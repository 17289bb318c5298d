// nm03/gpu_types.h — plain-old-data descriptors shared by the host runtime and the gfx950
// kernels. A batch is uploaded as ONE pinned blob (descriptors, tile lists, seeds, raw pixels)
// with a single hipMemcpyAsync; every kernel then walks descriptor tables, so slices of different
// sizes/pixel types can share one launch (SURVEY §7.1 "batched launches").
#pragma once

#include <cstdint>

namespace nm03::gpu {

// Median kernel output tile (64 columns × 64 rows) and sharpen/band tile (64 × 16: one mask word
// per row, produced by a wave ballot).
inline constexpr int kMedTileW = 64, kMedTileH = 64;
inline constexpr int kShpTileW = 64, kShpTileH = 64;
// Largest slice the LDS-resident region-growing kernel handles (bit-planes in LDS).
inline constexpr int kSrgMaxDim = 512;
// Largest 2D slice side the engine accepts. Slices above kSrgMaxDim keep K1/K3/K4 unchanged and
// run K2 with its bit planes in a global-memory scratch instead of LDS (launch_srg_morph).
inline constexpr int kMaxSliceDim = 4096;

// XCD-aware tile order: the dispatcher deals workgroups round-robin over the 8 XCDs (workgroup b runs on
// XCD b mod 8), so mapping b to logical tile (b mod 8)·⌈n/8⌉ + b/8 (remainder-adjusted) gives each XCD a
// contiguous run of tiles, whose shared halo rows then hit that XCD's L2. A bijection on [0, n)
// (constexpr: host and device). Used by K1b (sharpen: 20.4 → 19.0 µs per 96-slice batch); K1a's median
// got slower with it (28.4 → 29.8 µs), so it keeps the plain order (profiles/r5/xcd/).
constexpr uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, k = b >> 3, q = n >> 3, r = n & 7u;
  return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + k;
}

struct SliceDesc {
  uint32_t raw_off;    // u16 element offset of the slice in the raw/median buffers
  uint32_t mask_off;   // u64 word offset of the slice in every bitmap buffer (h * wpr words)
  uint16_t w, h;
  uint16_t wpr;        // mask words per row = ceil(w/64)
  uint8_t type;        // PixelType
  uint8_t stored_bits;
  float slope, intercept;
  uint32_t seed_off;   // index into the seed table (int16 x,y pairs)
  uint16_t seed_count;
  uint16_t flags;
  uint32_t f32_off;    // f32 element offset for optional sharpened output
  uint32_t med_tile0;  // index of the slice's first median tile in the batch tile list
  uint32_t blob_off;   // u16 element offset of the slice as uploaded (engine batches: K0 expands it to raw_off)
  // normalise+clip lookup table of the slice's (type, stored bits, rescale) — K1b reads
  // lut[lut_off + key − lut_base] instead of evaluating norm_clip_key per staged key;
  // lut_off == kNoLut: no table (the kernel evaluates the function).
  uint32_t lut_off;
  uint32_t lut_base;
};
static_assert(sizeof(SliceDesc) == 52, "SliceDesc layout");
inline constexpr uint32_t kNoLut = 0xFFFFFFFFu;
// SliceDesc::flags
inline constexpr uint16_t kSliceFlagPacked12 = 1;  // uploaded as 12-bit pairs (nm03/pack12.h)

struct TileDesc {
  uint32_t slice;
  uint16_t tx, ty;  // tile column / row
};

struct SeedXY {
  int16_t x, y;
};

// Per-slice statistics produced on device (ordered-u32 encodings so atomicMin/Max work).
struct SliceStats {
  uint32_t key_min, key_max;  // raw keys (render window of the original image)
  uint32_t s_min, s_max;      // sharpened f32 as ordered u32 (preprocessed_image window)
};

struct PipeConsts {
  // normalise + clip (slope/intercept are per slice)
  float nmin, nmax, nlow, nhigh, cmin, cmax;
  float gain;
  float band_lo, band_hi;
  float taps[16];
  int mask_radius;  // sharpen radius R (taps 2R+1)
  int median_k;
  int connectivity;  // 4 | 8
  int dilation_size, erosion_size, border_radius;
  uint32_t outputs;  // bit set of kOut* below
  int se_disc;       // PipelineParams::se_shape == kSeDisc: disc structuring element (else square)
};

enum : uint32_t {
  kOutRegion = 1u << 0,        // SRG result bitmap
  kOutDilated = 1u << 1,       // dilation(region)
  kOutEroded = 1u << 2,        // erosion(region) (test_pipeline only)
  kOutBorderRegion = 1u << 3,  // renderer border of region / eroded / dilated
  kOutBorderEroded = 1u << 4,
  kOutBorderDilated = 1u << 5,
  kOutSharpened = 1u << 6,     // f32 sharpened image (test_pipeline preprocessed_image)
};

// Render job: one canvas.
enum RenderKind : uint8_t { kRenderRawGray = 0, kRenderF32Gray = 1, kRenderLabels = 2 };

struct RenderDesc {
  uint8_t kind;
  uint8_t type, stored_bits;
  uint8_t fill, border_value;
  uint8_t filter;       // gray kinds: RenderFilter (0 bilinear, 1 nearest); labels: always nearest
  uint8_t pad0[2];
  uint32_t slice;       // stats index
  uint32_t src_off;     // u16 elements (raw) / f32 elements / u64 words (labels)
  uint32_t border_off;  // u64 words (labels)
  uint16_t src_w, src_h, wpr, pad1;
  float ox, oy, invx, invy;
  float slope, intercept;
  uint32_t canvas_off;  // byte offset into the canvas buffer
};

// JPEG job: one canvas (out_w×out_h, both multiples of 16) → one entropy-coded segment.
struct JpegDesc {
  uint32_t canvas_off;  // bytes (generic path: rendered canvas)
  uint32_t stage_off;   // u32 word offset of the bit staging area
  uint32_t stage_words;
  uint64_t out_off;     // byte offset in the output buffer (host-mapped)
  uint32_t out_cap;     // capacity in bytes
  int32_t render;       // -1: read canvas; else the fused 2× render from RenderDesc[render], where
                        // render is this descriptor's own index (the encoder loads both at once)
};

// Byte-stuffing chunk (bytes of entropy-coded data per workgroup in the stuffing kernels).
inline constexpr int kStuffChunk = 4096;

}  // namespace nm03::gpu
