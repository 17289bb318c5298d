// nm03/kernels.h — host-callable launchers of the gfx950 kernels (src/kernels/*.hip).
// All launchers are asynchronous on `stream` and allocation-free (graph-capturable).
#pragma once

#include <hip/hip_runtime_api.h>

#include <string>

#include "nm03/common.h"
#include "nm03/gpu_types.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

void check_hip(hipError_t e, const char* what);
void check_launch(const char* what);
// NM03_SYNC_LAUNCHES=1: synchronise after every launch (debugging; disables graph capture).
bool sync_launches();
// Profiling variant of `kernel` ("jpeg", "median") from NM03_PROFILE_VARIANT="jpeg=12,median=1"; 0 = the
// real kernel. Variants truncate the kernel for time splits; their output is invalid.
int profile_variant(const char* kernel);

// Loads the code object of every kernel translation unit (k1 median and sharpen, k2 SRG, k3 render,
// k4 JPEG, k5 volume, k6 threshold; every template instance) on the current device. HIP loads a
// translation unit's code object at the first launch of one of its kernels; preloading makes that
// happen on one thread before any launch (Engine and VolumeEngine constructors), never from a slot
// thread in the middle of a run. Fails loudly (DeviceError) when a code object does not load.
// with_volume = false leaves out k5 volume and k6 threshold, which the 2D engine never launches.
void preload_kernels(bool with_volume = true);
void preload_median();
void preload_sharpen();
void preload_srg();
void preload_render();
void preload_volume();
void preload_threshold();

// The engine's per-format normalise+clip table (n = 2^stored_bits keys from `base`), built on the
// device on `stream` with the shared pixel_math.h function.
void launch_build_norm_lut(float* out, uint32_t n, uint32_t base, uint8_t type, const NormClip& nc, hipStream_t stream);
// The first host→device copy of a process initialises the runtime's copy path (≈ 10 ms on a cold
// MI355X process, profiles/r5/cold/): one 4 MiB pinned H2D on `stream` (the SDMA path), synchronised.
void warm_copy_path(hipStream_t stream);

// K1a: k×k median of raw keys → `med` (u16 keys, same layout as raw). k ∈ {3,5,7,9}.
// Per-slice key range: with `tile_mm` (2 u32 per tile) each tile stores its (min, max) and
// launch_sharpen_band reduces them into stats (no atomics); without it, atomics on stats.
// With `blob` (engine batches) the samples are read from the uploaded blob at SliceDesc::blob_off
// (12-bit packed slices decoded on the fly) instead of `raw`, and the expanded 16-bit samples are
// written to `raw_out` at raw_off (the samples the render stage reads).
void launch_median(const uint16_t* raw, uint16_t* med, const SliceDesc* descs, const TileDesc* tiles, int ntiles,
                   int k, SliceStats* stats, hipStream_t stream, uint32_t* tile_mm = nullptr,
                   const uint16_t* blob = nullptr, uint16_t* raw_out = nullptr);

// K1b: normalise+clip of the median keys, separable Gaussian unsharp mask, SRG band test →
// `band` bitmaps (u64 words, LSB = left-most pixel). Optionally the f32 sharpened image.
// `lut` (optional): the engine's normalise+clip tables (SliceDesc::lut_off / lut_base).
void launch_sharpen_band(const uint16_t* med, uint64_t* band, float* sharpened, const SliceDesc* descs,
                         const TileDesc* tiles, int ntiles, const PipeConsts& pc, SliceStats* stats,
                         hipStream_t stream, const uint32_t* tile_mm = nullptr, const float* lut = nullptr);

// Bitmap planes produced by K2 (each null when not requested).
struct SrgOutputs {
  uint64_t* region = nullptr;
  uint64_t* dilated = nullptr;
  uint64_t* eroded = nullptr;
  uint64_t* border_region = nullptr;
  uint64_t* border_eroded = nullptr;
  uint64_t* border_dilated = nullptr;
  int32_t* iterations = nullptr;  // per-slice fixpoint iteration count (diagnostics)
  // Slices larger than kSrgMaxDim: 4 × srg_scratch_words(max_w, max_h) words per slice of device
  // scratch for the bit planes (the LDS-resident form cannot hold them).
  uint64_t* scratch = nullptr;
};
// Words per bit plane of the K2 kernel for slices up to max_w × max_h (odd row strides).
size_t srg_plane_words(int max_w, int max_h);

// K2: LDS-resident seeded region growing (bit-parallel run fills on rows and on the transposed
// bitmap until fixpoint) + dilation/erosion + renderer borders. One workgroup per slice; the four
// bit planes live in LDS for slices ≤ kSrgMaxDim, else in `out.scratch` (same code, global memory).
void launch_srg_morph(const uint64_t* band, const SliceDesc* descs, int nslices, const SeedXY* seeds,
                      const PipeConsts& pc, const SrgOutputs& out, int max_w, int max_h, hipStream_t stream);

// 3D region growing on a w×h×d bit volume (planes of h rows × ceil(w/64) words) by plane sweeps in
// ONE cooperative launch that decides convergence on the device (k5_volume.hip): no host
// synchronisation. seeds_xyz: device int32 triples. d_ctl: kSrg3dCtlWords device words; h_ctl
// (optional): pinned host words receiving them at the end of the launch — srg_volume_result(h_ctl)
// after the stream is synchronised gives the sweep count (or throws). Planes too large for LDS
// (a side > 512) need `scratch` of srg3d_scratch_words(w, h, d) words. reset = false continues from
// the region already in `region` (⊆ band): the z-slab decomposition (volume_slabs.h) re-grows a slab
// after neighbouring slabs contributed boundary voxels.
constexpr int kSrg3dCtlWords = 8;
size_t srg3d_scratch_words(int w, int h, int d);
void srg_volume(const uint64_t* band, uint64_t* region, int w, int h, int d, const int32_t* seeds_xyz, int nseeds,
                int connectivity, uint32_t* d_ctl, uint32_t* h_ctl, uint64_t* scratch, hipStream_t stream,
                bool reset = true);
int srg_volume_result(const uint32_t* h_ctl);
// Scratch for border_volume / dilate_volume when a plane does not fit LDS (else 0).
size_t morph3d_scratch_words(int w, int h, int d);
// Per-plane renderer border of a bit volume: label ∧ ¬erode_{(2r+1)²}(label) (2D, every plane).
void border_volume(const uint64_t* src, uint64_t* dst, int w, int h, int d, int radius, hipStream_t stream,
                   uint64_t* scratch = nullptr);
// Cube dilation of a bit volume (size odd), separable; `tmp` same size as the volume.
// `ball`: the digital ball of radius size/2 (one pass, dilate_ball_kernel) instead of the size³ cube.
void dilate_volume(const uint64_t* src, uint64_t* dst, uint64_t* tmp, int w, int h, int d, int size,
                   hipStream_t stream, uint64_t* scratch = nullptr, bool ball = false);
// z-slab boundary step (volume_slabs.h), one plane: add = band ∧ touch(nb) ∧ ¬region, region |= add,
// *added += popcount(add); touch = nb (6-connectivity) or its 3×3 in-plane dilation (26).
void launch_slab_seed(const uint64_t* band, uint64_t* region, const uint64_t* nb, int w, int h, bool conn26,
                      unsigned long long* added, hipStream_t stream);

// K3: render canvases (out_w×out_h u8 each).
void launch_render(const uint16_t* raw, const float* f32, const uint64_t* bits, const SliceStats* stats,
                   const RenderDesc* rd, int ncanvas, int out_w, int out_h, uint8_t* canvas, hipStream_t stream);

// K4: JPEG in one pass, workgroup per 256 luma blocks of an image: [fused 2× render or canvas
// read] → islow FDCT → reciprocal quantisation → Huffman coding → workgroup scan → bit range in
// LDS → decoupled look-back across the image (bit offset and 0xFF-stuffing count) → the stuffed
// bytes straight into `out` (host-mapped pinned memory, JpegDesc.out_off).
// out_sizes[i] = bytes, or -1 when the image exceeded its staging/out capacity (caller
// re-encodes on the CPU).
struct JpegWork {
  uint64_t* look = nullptr;      // 2 × 3 × look_cap record words, zeroed once at allocation: two
                                 // halves, each launch uses one and clears the other (launch_jpeg)
  size_t look_cap = 0;           // ≥ ncanvas × ceil(blocks / 256) workgroups
  size_t look_used = 0;          // set by launch_jpeg
  size_t look_base = 0, clear_base = 0, clear_words = 0, prev_words = 0;  // launch_jpeg's bookkeeping
  uint32_t* ticket = nullptr;    // per-image part ticket counters (≥ ncanvas; zeroed once; self-resetting)
  uint32_t* spill = nullptr;     // look_cap × 256 × 56 words: Huffman bits of very detailed blocks
};
// Fused-render inputs (needed when any JpegDesc.render ≥ 0).
struct JpegRenderSrc {
  const uint16_t* raw = nullptr;
  const float* f32 = nullptr;
  const uint64_t* bits = nullptr;
  const SliceStats* stats = nullptr;
  // Render descriptors, one per canvas: JpegDesc k's `render` is either -1 (encode canvas k from
  // `canvas`) or k itself (render descriptor k fused into the encoder). launch_jpeg checks that
  // `nrd` covers every canvas when rd is set.
  const RenderDesc* rd = nullptr;
  int nrd = 0;
};
void launch_jpeg(const uint8_t* canvas, const JpegDesc* jd, int ncanvas, int out_w, int out_h, const int32_t* div_luma,
                 JpegWork& w, uint8_t* out, int32_t* out_sizes, hipStream_t stream,
                 const JpegRenderSrc* fused = nullptr, int sampling = 0,  // jpeg::Sampling
                 bool nearest = false);  // fused gray renders use --render-filter nearest (4:2:0 only)
// Whether the fused encoder renders --render-filter nearest gray images for this layout (else callers
// render them into canvases first).
inline bool jpeg_fuses_nearest(int sampling) { return sampling == 0; }
// K6: binary threshold lo ≤ x ≤ hi → u8 0/1 (in 16-byte aligned, out 4-byte aligned).
void launch_threshold(const float* in, uint8_t* out, size_t n, float lo, float hi, hipStream_t stream);

// True when RenderDesc r is an exact 2× fit onto the canvas (the fused fast path applies).
bool render_is_exact_2x(const RenderDesc& r, int out_w, int out_h);

// Upload the 64 islow divisors (8·Q, natural order) for `quality` into a device buffer.
void jpeg_divisors(int quality, int32_t* host_out64);

}  // namespace nm03::gpu
