// K5 — 3D mode (BASELINE config 5: 256³ volume, SeededRegionGrowing + 7×7×7 Dilation).
//
// Region growing on a bit volume [z][y][ceil(w/64)] by PLANE SWEEPS that alternate orientation:
// xy planes (workgroup per z) and xz planes (workgroup per y; a plane row is the strided row
// (z, y) of the volume, so no transposed copy of the volume is needed). Each workgroup loads its
// band and region plane into LDS, seeds from the two neighbouring planes (26-connectivity dilates
// them in-plane first), and runs the same on-chip 2D fixpoint as K2 (srg_core.h: row run fills +
// transposed column run fills). Because xz sweeps fill whole z-runs at once, the sweep count is
// ≈ the number of direction turns of the region, not its z extent. Planes read neighbours while
// those are being rewritten — harmless: the iteration is monotone (bits are only added, 64-bit
// words are written atomically); a sweep that changes nothing proves the fixpoint.
// Cube dilation is separable: in-plane square dilation in LDS (row shifts + row ORs), then an OR
// over z. Out-of-volume samples are ignored (App. A.7).
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "srg_core.h"

namespace nm03::gpu {

__global__ void srg3d_seed_kernel(const uint64_t* __restrict__ band, uint64_t* __restrict__ region, int w, int h,
                                  int d, const int32_t* __restrict__ seeds, int nseeds) {
  const int n = (w + 63) >> 6;
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseeds) return;
  const int x = seeds[3 * s], y = seeds[3 * s + 1], z = seeds[3 * s + 2];
  if (x < 0 || y < 0 || z < 0 || x >= w || y >= h || z >= d) return;
  const size_t wi = ((size_t)z * h + y) * n + (x >> 6);
  const uint64_t bit = 1ull << (x & 63);
  if (band[wi] & bit) atomicOr((unsigned long long*)&region[wi], (unsigned long long)bit);
}

// One sweep over all planes of one orientation. axis 0: plane p = z, rows = y (xy planes);
// axis 1: plane p = y, rows = z (xz planes). Row r of plane p starts at word row_base(p, r).
__device__ __forceinline__ size_t row_base(int axis, int p, int r, int h, int n) {
  return axis == 0 ? ((size_t)p * h + r) * n : ((size_t)r * h + p) * n;
}

__global__ __launch_bounds__(256) void srg3d_sweep_kernel(const uint64_t* __restrict__ band, uint64_t* region, int w,
                                                          int h, int d, int axis, int connectivity, int plane_words,
                                                          uint32_t* changed) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  __shared__ int flag;
  const int p = blockIdx.x;
  const int nplanes = axis == 0 ? d : h;
  const int rows = axis == 0 ? h : d;
  const int n = (w + 63) >> 6;
  const int words = rows * n;
  uint64_t* M = smem;
  uint64_t* Rg = M + plane_words;
  uint64_t* Mt = Rg + plane_words;
  uint64_t* Rt = Mt + plane_words;
  for (int i = threadIdx.x; i < words; i += blockDim.x) {
    const int r = i / n, c = i - r * n;
    const size_t g = row_base(axis, p, r, h, n) + c;
    M[i] = band[g];
    Rg[i] = region[g];
    uint64_t nb = 0;  // seeds from the neighbouring planes
    if (p > 0) nb |= region[row_base(axis, p - 1, r, h, n) + c];
    if (p + 1 < nplanes) nb |= region[row_base(axis, p + 1, r, h, n) + c];
    Mt[i] = nb;
  }
  __syncthreads();
  // 26-connectivity: neighbour planes dilated in-plane by one (3×3) before seeding.
  if (connectivity == 26) morph(Mt, Mt, Rt, w, rows, n, 3, true);
  for (int i = threadIdx.x; i < words; i += blockDim.x) Rg[i] |= M[i] & Mt[i];
  __syncthreads();
  transpose_plane(M, rows, n, Mt, w, false, nullptr);
  __syncthreads();
  srg_fixpoint(M, Rg, Mt, Rt, w, rows, n, connectivity == 26 ? 8 : 4, &flag);
  int local_change = 0;
  for (int i = threadIdx.x; i < words; i += blockDim.x) {
    const int r = i / n, c = i - r * n;
    const size_t g = row_base(axis, p, r, h, n) + c;
    const uint64_t old = region[g];
    const uint64_t nv = Rg[i] | old;
    if (nv != old) {
      region[g] = nv;
      local_change = 1;
    }
  }
  if (local_change) atomicOr(changed, 1u);
}

__global__ __launch_bounds__(256) void dilate_plane_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                           int w, int h, int size, int plane_words) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int n = (w + 63) >> 6, words = h * n;
  const size_t off = (size_t)blockIdx.x * words;
  uint64_t* A = smem;
  uint64_t* B = A + plane_words;
  uint64_t* T = B + plane_words;
  for (int i = threadIdx.x; i < words; i += blockDim.x) A[i] = src[off + i];
  __syncthreads();
  morph(A, B, T, w, h, n, size, true);
  for (int i = threadIdx.x; i < words; i += blockDim.x) dst[off + i] = B[i];
}

// Renderer border of every plane: label ∧ ¬erode_{size×size}(label) in 2D per plane (the
// SegmentationRenderer outlines each displayed slice; size = 2·radius + 1).
__global__ __launch_bounds__(256) void border_plane_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                           int w, int h, int size, int plane_words) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int n = (w + 63) >> 6, words = h * n;
  const size_t off = (size_t)blockIdx.x * words;
  uint64_t* A = smem;
  uint64_t* B = A + plane_words;
  uint64_t* T = B + plane_words;
  for (int i = threadIdx.x; i < words; i += blockDim.x) A[i] = src[off + i];
  __syncthreads();
  morph(A, B, T, w, h, n, size, false);
  for (int i = threadIdx.x; i < words; i += blockDim.x) dst[off + i] = A[i] & ~B[i];
}

__global__ void dilate_z_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int words, int d, int r) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)words * d) return;
  const int z = (int)(i / words);
  uint64_t acc = src[i];
  for (int k = 1; k <= r; ++k) {
    if (z - k >= 0) acc |= src[i - (size_t)k * words];
    if (z + k < d) acc |= src[i + (size_t)k * words];
  }
  dst[i] = acc;
}

int srg_volume(const uint64_t* band, uint64_t* region, int w, int h, int d, const int32_t* seeds_xyz, int nseeds,
               int connectivity, uint32_t* d_flag, uint32_t* h_flag, hipStream_t stream, bool reset) {
  if (w > kSrgMaxDim || h > kSrgMaxDim || d > kSrgMaxDim) throw DeviceError("srg_volume: dimension larger than 512");
  const int n = (w + 63) / 64, wb = (w + 63) / 64;
  const size_t words = (size_t)h * n;
  // LDS plane sized for both orientations: rows ≤ max(h, d), transposed rows = w.
  const int maxrows = h > d ? h : d;
  int plane_words = maxrows * n;
  if (w * ((maxrows + 63) / 64) > plane_words) plane_words = w * ((maxrows + 63) / 64);
  plane_words = (plane_words + 1) & ~1;
  (void)wb;
  if (reset) check_hip(hipMemsetAsync(region, 0, words * d * sizeof(uint64_t), stream), "memset region");
  if (nseeds > 0) {
    srg3d_seed_kernel<<<(nseeds + 63) / 64, 64, 0, stream>>>(band, region, w, h, d, seeds_xyz, nseeds);
    check_launch("srg3d_seed_kernel");
  }
  const size_t lds = (size_t)plane_words * 4 * sizeof(uint64_t);
  // Alternate xy-plane and xz-plane sweeps; each pair is checked with one D2H of two flags. A sweep
  // that changes nothing proves the 3D fixpoint (closed in-plane and under neighbour seeding).
  int sweeps = 0;
  for (;;) {
    check_hip(hipMemsetAsync(d_flag, 0, 2 * sizeof(uint32_t), stream), "memset flags");
    for (int axis = 0; axis < 2; ++axis) {
      srg3d_sweep_kernel<<<axis == 0 ? d : h, 256, lds, stream>>>(band, region, w, h, d, axis, connectivity,
                                                                  plane_words, d_flag + axis);
      check_launch("srg3d_sweep_kernel");
    }
    sweeps += 2;
    check_hip(hipMemcpyAsync(h_flag, d_flag, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream), "flag d2h");
    check_hip(hipStreamSynchronize(stream), "sweep sync");
    if (h_flag[0] == 0 || h_flag[1] == 0 || sweeps > 4 * (w + h + d)) break;
  }
  return sweeps;
}

void border_volume(const uint64_t* src, uint64_t* dst, int w, int h, int d, int radius, hipStream_t stream) {
  const int n = (w + 63) / 64;
  const int plane_words = (h * n + 1) & ~1;
  border_plane_kernel<<<d, 256, (size_t)plane_words * 3 * sizeof(uint64_t), stream>>>(src, dst, w, h, 2 * radius + 1,
                                                                                    plane_words);
  check_launch("border_plane_kernel");
}

void dilate_volume(const uint64_t* src, uint64_t* dst, uint64_t* tmp, int w, int h, int d, int size, hipStream_t stream) {
  const int n = (w + 63) / 64;
  const int words = h * n;
  const int plane_words = (words + 1) & ~1;
  dilate_plane_kernel<<<d, 256, (size_t)plane_words * 3 * sizeof(uint64_t), stream>>>(src, tmp, w, h, size, plane_words);
  check_launch("dilate_plane_kernel");
  const size_t total = (size_t)words * d;
  dilate_z_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(tmp, dst, words, d, size / 2);
  check_launch("dilate_z_kernel");
}

}  // namespace nm03::gpu
