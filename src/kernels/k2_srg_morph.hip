// K2 — SeededRegionGrowing (main_sequential.cpp:232-243) + ImageCaster(UINT8) + Dilation(3) /
// Erosion(3) (main_sequential.cpp:246-252, test_pipeline.cpp:119-125) + the SegmentationRenderer
// border mask (radius 2), fused in one launch with ONE WORKGROUP PER SLICE and every bit-plane
// resident in LDS (256² slice: 8 KiB per plane).
//
// FAST grows the region with an iterative OpenCL kernel plus host polling of a stop flag
// (a host↔device round trip per poll, hundreds of iterations). Here the fixpoint
// runs entirely on-chip:
//   * horizontal step: every row's runs of in-band pixels that contain a region pixel are filled
//     at once with the carry trick  F = (((M + S) ^ M) & M) | S  (S = R & M ⊆ M), upward, and
//     downward on bit-reversed words; carries chain across the row's words;
//   * vertical step: the same run fill on the TRANSPOSED planes (64×64 bit-block transposes done
//     in registers with wave64 butterflies, device_util.h);
//   * 8-connectivity adds a diagonal seeding step R |= M & (dil1(R↑) | dil1(R↓)).
// The loop stops when a full iteration changes nothing (workgroup barrier + LDS flag; no host).
// Morphology uses shifted-word ORs/ANDs; out-of-image samples are ignored (App. A.7). The
// Dilation/Erosion structuring element is the square (default) or the digital disc
// (PipeConsts::se_disc, --se-shape disc); the renderer border always erodes with a square.
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "srg_core.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

// Threads per slice workgroup. Row/column fills use one thread per row (≤ 512), the 64×64 bit
// transposes and morphology passes spread over every wave. A batch has only one workgroup per
// slice, so per-workgroup latency is the cost: 256 → 512 → 1024 threads measured 32.4 → 24.9 →
// 23.1 µs per 64-slice batch (isolated rocprofv3 kernel timings, round 1).
#ifndef NM03_SRG_THREADS
#define NM03_SRG_THREADS 1024
#endif
constexpr int kSrgThreads = NM03_SRG_THREADS;


// One slice's region growing + morphology, on four bit planes at `smem` (LDS or global scratch).
// NW > 0: every row has NW words and every column HB words (compile time: unrolled register fills).
template <int NW, int HB>
__device__ __forceinline__ void srg_slice(uint64_t* const smem, int* flag, const uint64_t* __restrict__ band,
                                          const SliceDesc& d, const SeedXY* __restrict__ seeds, const PipeConsts& pc,
                                          const SrgOutputs& out, int plane_words) {
  const int W = d.w, H = d.h, n = NW > 0 ? NW : d.wpr, hb = HB > 0 ? HB : (H + 63) >> 6;
  const int words = H * n;
  // LDS row strides: odd word counts, so the thread-per-row sweeps and the 64-row transposes (lane
  // = row) hit 32 distinct 8-byte bank pairs per half-wave instead of 4-way conflicts at stride 4.
  const int sn = n | 1, st = hb | 1;
  auto at = [&](int q) { const int y = q / n; return y * sn + (q - y * n); };  // dense → LDS index
  uint64_t* M = smem;
  uint64_t* Rg = M + plane_words;
  uint64_t* Mt = Rg + plane_words;
  uint64_t* Rt = Mt + plane_words;

  for (int i = threadIdx.x; i < words; i += blockDim.x) {
    const int j = at(i);
    M[j] = band[d.mask_off + i];
    Rg[j] = 0ull;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < d.seed_count; s += blockDim.x) {
    const SeedXY sd = seeds[d.seed_off + s];
    if (sd.x < 0 || sd.y < 0 || sd.x >= W || sd.y >= H) continue;
    const int wi = sd.y * sn + (sd.x >> 6);
    const uint64_t bit = 1ull << (sd.x & 63);
    if (M[wi] & bit) atomicOr((unsigned long long*)&Rg[wi], (unsigned long long)bit);
  }
  transpose_plane(M, H, n, Mt, W, false, nullptr, sn, st);
  __syncthreads();

  const int iters = srg_fixpoint<NW, HB>(M, Rg, Mt, Rt, W, H, n, pc.connectivity, flag, sn, st);
  // An iteration in which no step changed anything ⇒ Rg is the fixpoint region.
  if (out.iterations && threadIdx.x == 0) out.iterations[blockIdx.x] = iters;
  const size_t off = d.mask_off;
  if (out.region) store_plane(Rg, out.region + off, H, n, sn);
  // Scratch planes now: M, Mt, Rt (all used in row layout, stride sn, from here on).
  if (out.dilated || out.border_dilated) {
    morph_se<NW>(Rg, Mt, M, W, H, n, pc.dilation_size, true, pc.se_disc, sn);  // Mt = D
    if (out.dilated) store_plane(Mt, out.dilated + off, H, n, sn);
    if (out.border_dilated) {
      morph<NW>(Mt, Rt, M, W, H, n, 2 * pc.border_radius + 1, false, sn);  // Rt = erode(D)
      for (int i = threadIdx.x; i < words; i += blockDim.x) out.border_dilated[off + i] = Mt[at(i)] & ~Rt[at(i)];
    }
    __syncthreads();
  }
  if (out.border_region) {
    morph<NW>(Rg, Rt, M, W, H, n, 2 * pc.border_radius + 1, false, sn);
    for (int i = threadIdx.x; i < words; i += blockDim.x) out.border_region[off + i] = Rg[at(i)] & ~Rt[at(i)];
    __syncthreads();
  }
  if (out.eroded || out.border_eroded) {
    morph_se<NW>(Rg, Mt, M, W, H, n, pc.erosion_size, false, pc.se_disc, sn);  // Mt = E
    if (out.eroded) store_plane(Mt, out.eroded + off, H, n, sn);
    if (out.border_eroded) {
      morph<NW>(Mt, Rt, M, W, H, n, 2 * pc.border_radius + 1, false, sn);
      for (int i = threadIdx.x; i < words; i += blockDim.x) out.border_eroded[off + i] = Mt[at(i)] & ~Rt[at(i)];
    }
  }
}

// kGlobal: slices above kSrgMaxDim — the same algorithm on bit planes in a per-slice global scratch
// (L2-resident for a 1024² slice: 4 × 128 KiB), for capability rather than speed. 256×256 slices
// (the cohort shape) take the 4-word specialisation.
template <bool kGlobal>
__global__ __launch_bounds__(kSrgThreads) void srg_morph_kernel(const uint64_t* __restrict__ band,
                                                        const SliceDesc* __restrict__ descs,
                                                        const SeedXY* __restrict__ seeds, PipeConsts pc,
                                                        SrgOutputs out, int plane_words) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_planes[];
  __shared__ int flag[2];  // srg_fixpoint's two alternating change words
  uint64_t* const smem = kGlobal ? out.scratch + (size_t)blockIdx.x * 4 * plane_words : lds_planes;
  const SliceDesc d = descs[blockIdx.x];
  if (!kGlobal && d.wpr == 4 && d.h > 192 && d.h <= 256)
    srg_slice<4, 4>(smem, flag, band, d, seeds, pc, out, plane_words);
  else
    srg_slice<0, 0>(smem, flag, band, d, seeds, pc, out, plane_words);
}

size_t srg_plane_words(int max_w, int max_h) {
  // Planes hold rows at the kernel's odd strides (n | 1 and hb | 1 words); a slice's n ≤ this n.
  const int n = (max_w + 63) / 64, hb = (max_h + 63) / 64;
  size_t plane_words = (size_t)max_h * (n | 1);
  if ((size_t)max_w * (hb | 1) > plane_words) plane_words = (size_t)max_w * (hb | 1);
  return (plane_words + 1) & ~(size_t)1;
}

void launch_srg_morph(const uint64_t* band, const SliceDesc* descs, int nslices, const SeedXY* seeds,
                      const PipeConsts& pc, const SrgOutputs& out, int max_w, int max_h, hipStream_t stream) {
  if (nslices <= 0) return;
  if (max_w > kMaxSliceDim || max_h > kMaxSliceDim)
    throw DeviceError("launch_srg_morph: slice larger than " + std::to_string(kMaxSliceDim));
  const int plane_words = (int)srg_plane_words(max_w, max_h);
  if (max_w > kSrgMaxDim || max_h > kSrgMaxDim) {
    if (!out.scratch) throw DeviceError("launch_srg_morph: slices above 512 need SrgOutputs.scratch");
    srg_morph_kernel<true><<<nslices, kSrgThreads, 0, stream>>>(band, descs, seeds, pc, out, plane_words);
  } else {
    const size_t lds = (size_t)plane_words * 4 * sizeof(uint64_t);
    srg_morph_kernel<false><<<nslices, kSrgThreads, lds, stream>>>(band, descs, seeds, pc, out, plane_words);
  }
  check_launch("srg_morph_kernel");
}

void preload_srg() {
  hipFuncAttributes a;
  for (const void* f : {reinterpret_cast<const void*>(&srg_morph_kernel<false>), reinterpret_cast<const void*>(&srg_morph_kernel<true>)})
    check_hip(hipFuncGetAttributes(&a, f), "preload srg_morph_kernel");
}

}  // namespace nm03::gpu
