// K5 — 3D mode (BASELINE config 5: 256³ volume, SeededRegionGrowing + 7×7×7 Dilation).
//
// Region growing on a bit volume [z][y][ceil(w/64)] by PLANE SWEEPS that alternate orientation:
// xy planes (plane per z) and xz planes (plane per y; a plane row is the strided row (z, y) of the
// volume, so no transposed copy of the volume is needed). A workgroup loads a plane's band and
// region bits, seeds from the two neighbouring planes (26-connectivity dilates them in-plane
// first), and runs the same on-chip 2D fixpoint as K2 (srg_core.h: row run fills + transposed
// column run fills). Because xz sweeps fill whole z-runs at once, the sweep count is ≈ the number
// of direction turns of the region, not its z extent. Planes read neighbours while those are being
// rewritten — harmless: the iteration is monotone (bits are only added, 64-bit words are written
// atomically); a sweep that changes nothing proves the fixpoint.
//
// Convergence is decided ON THE DEVICE (FAST polls a stop flag from the host): ONE
// cooperative launch of a persistent kernel runs every sweep; workgroups stride over the planes of
// the sweep, meet at a grid barrier (co-residency guaranteed by hipLaunchCooperativeKernel), and
// read the sweep's change flag — a ring of three words, so clearing the next one never races a
// reader. The barrier's spin is bounded (error word set, every workgroup leaves), so a broken
// launch can never hang the GPU. No host synchronisation inside srg_volume.
//
// Planes larger than LDS holds (any side > 512) run the same code on per-workgroup global scratch
// (as K2 does for large 2D slices). Cube dilation is separable: in-plane square dilation (row
// shifts + row ORs), then an OR over z. Out-of-volume samples are ignored (App. A.7).
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "srg_core.h"

namespace nm03::gpu {

constexpr int kSrg3dThreads = 512;
constexpr size_t kLdsBudget = 160 * 1024;  // LDS per workgroup on gfx950
// Control words (kSrg3dCtlWords, zeroed before every launch).
enum : int { kCtlBarCount = 0, kCtlBarGen = 1, kCtlChanged = 2 /* 3 words */, kCtlSweeps = 5, kCtlError = 6 };

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

// Row r of plane p. axis 0: plane p = z, rows = y (xy planes); axis 1: plane p = y, rows = z.
__device__ __forceinline__ size_t row_base(int axis, int p, int r, int h, int n) {
  return axis == 0 ? ((size_t)p * h + r) * n : ((size_t)r * h + p) * n;
}

// Grows plane p of one orientation to its in-plane fixpoint under neighbour seeding and writes the
// additions back. `planes`: 4 × plane_words scratch (LDS or global). Returns whether the volume's
// plane changed (workgroup-uniform after the caller's barrier; here per thread).
__device__ bool sweep_plane(const uint64_t* __restrict__ band, uint64_t* region, int w, int h, int d, int axis, int p,
                            int connectivity, int plane_words, uint64_t* planes, int* flag) {
  const int nplanes = axis == 0 ? d : h;
  const int rows = axis == 0 ? h : d;
  const int n = (w + 63) >> 6;
  const int words = rows * n;
  uint64_t* M = planes;
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
  srg_fixpoint(M, Rg, Mt, Rt, w, rows, n, connectivity == 26 ? 8 : 4, flag);
  bool local_change = false;
  for (int i = threadIdx.x; i < words; i += blockDim.x) {
    const int r = i / n, c = i - r * n;
    const size_t g = row_base(axis, p, r, h, n) + c;
    const uint64_t old = region[g];
    const uint64_t nv = Rg[i] | old;
    if (nv != old) {
      region[g] = nv;
      local_change = true;
    }
  }
  __syncthreads();  // the scratch planes are reused by the workgroup's next plane
  return local_change;
}

// Grid barrier for a cooperative launch: arrival counter + generation word, agent-scope fences
// around it (the region planes written before it are read by other XCDs after it). The wait is
// bounded (~seconds): on expiry the error word is set and false returned — the caller leaves.
__device__ bool grid_barrier(uint32_t* ctl, uint32_t nblocks) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __threadfence();  // release this workgroup's region writes
    const uint32_t g = __hip_atomic_load(&ctl[kCtlBarGen], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (atomicAdd(&ctl[kCtlBarCount], 1u) == nblocks - 1) {
      __hip_atomic_store(&ctl[kCtlBarCount], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
      atomicAdd(&ctl[kCtlBarGen], 1u);
    } else {
      uint32_t spins = 0;
      while (__hip_atomic_load(&ctl[kCtlBarGen], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
        if (++spins > (1u << 25) ||
            __hip_atomic_load(&ctl[kCtlError], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
          atomicOr(&ctl[kCtlError], 1u);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(4);
      }
    }
    __threadfence();  // acquire the other workgroups' writes
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Every sweep of the region growing in one launch (see the file comment). kGlobal: the four bit
// planes per workgroup live in `scratch` (plane sides > 512) instead of LDS.
template <bool kGlobal>
__global__ __launch_bounds__(kSrg3dThreads) void srg3d_kernel(const uint64_t* __restrict__ band, uint64_t* region,
                                                              int w, int h, int d, int connectivity, int plane_words,
                                                              uint32_t* ctl, int max_sweeps, uint64_t* scratch) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_planes[];
  __shared__ int flag[2];  // srg_fixpoint's two alternating change words
  uint64_t* const planes = kGlobal ? scratch + (size_t)blockIdx.x * 4 * plane_words : lds_planes;
  int sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    const int axis = sweep & 1;
    const int nplanes = axis == 0 ? d : h;
    // The change word of the next sweep was last read after the barrier that ended sweep − 2,
    // which every workgroup has passed by now.
    if (blockIdx.x == 0 && threadIdx.x == 0)
      __hip_atomic_store(&ctl[kCtlChanged + (sweep + 1) % 3], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool changed = false;
    for (int p = blockIdx.x; p < nplanes; p += gridDim.x)
      changed |= sweep_plane(band, region, w, h, d, axis, p, connectivity, plane_words, planes, flag);
    if (__syncthreads_or(changed) && threadIdx.x == 0) atomicOr(&ctl[kCtlChanged + sweep % 3], 1u);
    if (!grid_barrier(ctl, gridDim.x)) return;
    const uint32_t c = __hip_atomic_load(&ctl[kCtlChanged + sweep % 3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (c == 0u) {  // nothing changed anywhere: the fixpoint
      ++sweep;
      break;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) ctl[kCtlSweeps] = (uint32_t)sweep;
}

namespace {

struct Srg3dShape {
  int plane_words;
  size_t lds;
  bool global;
};

Srg3dShape srg3d_shape(int w, int h, int d) {
  const int n = (w + 63) / 64;
  // One plane buffer sized for both orientations: rows ≤ max(h, d), transposed rows = w.
  const int maxrows = h > d ? h : d;
  int plane_words = maxrows * n;
  if (w * ((maxrows + 63) / 64) > plane_words) plane_words = w * ((maxrows + 63) / 64);
  plane_words = (plane_words + 1) & ~1;
  const size_t lds = (size_t)plane_words * 4 * sizeof(uint64_t);
  return {plane_words, lds, lds + 1024 > kLdsBudget};
}

int cu_count() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 64;
  return cus;
}

// Workgroups of the persistent launch: every one must be resident at once (grid barrier).
int srg3d_grid(const Srg3dShape& s, int w, int h, int d) {
  (void)w;
  const int nplanes = d > h ? d : h;
  int per_cu = 0;
  const void* f = s.global ? (const void*)srg3d_kernel<true> : (const void*)srg3d_kernel<false>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, kSrg3dThreads, s.global ? 0 : s.lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  int grid = per_cu * cu_count();
  if (s.global) grid = grid < 2 * cu_count() ? grid : 2 * cu_count();  // bounds the scratch
  return grid < nplanes ? grid : nplanes;
}

}  // namespace

size_t srg3d_scratch_words(int w, int h, int d) {
  const Srg3dShape s = srg3d_shape(w, h, d);
  if (!s.global) return 0;
  return (size_t)srg3d_grid(s, w, h, d) * 4 * (size_t)s.plane_words;
}

void srg_volume(const uint64_t* band, uint64_t* region, int w, int h, int d, const int32_t* seeds_xyz, int nseeds,
                int connectivity, uint32_t* d_ctl, uint32_t* h_ctl, uint64_t* scratch, hipStream_t stream,
                bool reset) {
  if (w > kMaxSliceDim || h > kMaxSliceDim || d > kMaxSliceDim)
    throw DeviceError("srg_volume: volume side larger than " + std::to_string(kMaxSliceDim));
  const int n = (w + 63) / 64;
  const size_t words = (size_t)h * n;
  const Srg3dShape s = srg3d_shape(w, h, d);
  if (s.global && !scratch) throw DeviceError("srg_volume: planes above the LDS size need scratch (srg3d_scratch_words)");
  if (reset) check_hip(hipMemsetAsync(region, 0, words * d * sizeof(uint64_t), stream), "memset region");
  check_hip(hipMemsetAsync(d_ctl, 0, kSrg3dCtlWords * sizeof(uint32_t), stream), "memset srg3d control");
  if (nseeds > 0) {
    srg3d_seed_kernel<<<(nseeds + 63) / 64, 64, 0, stream>>>(band, region, w, h, d, seeds_xyz, nseeds);
    check_launch("srg3d_seed_kernel");
  }
  const int grid = srg3d_grid(s, w, h, d);
  int max_sweeps = 4 * (w + h + d);
  int plane_words = s.plane_words;
  void* args[] = {(void*)&band, (void*)&region, (void*)&w, (void*)&h, (void*)&d, (void*)&connectivity,
                  (void*)&plane_words, (void*)&d_ctl, (void*)&max_sweeps, (void*)&scratch};
  const void* f = s.global ? (const void*)srg3d_kernel<true> : (const void*)srg3d_kernel<false>;
  check_hip(hipLaunchCooperativeKernel(f, dim3(grid), dim3(kSrg3dThreads), args, s.global ? 0 : s.lds, stream),
            "srg3d_kernel (cooperative launch)");
  check_launch("srg3d_kernel");
  if (h_ctl)
    check_hip(hipMemcpyAsync(h_ctl, d_ctl, kSrg3dCtlWords * sizeof(uint32_t), hipMemcpyDeviceToHost, stream),
              "srg3d control D2H");
}

int srg_volume_result(const uint32_t* h_ctl) {
  if (h_ctl[kCtlError]) throw DeviceError("3D region growing: grid barrier timed out (workgroups not co-resident)");
  return (int)h_ctl[kCtlSweeps];
}

// ---- morphology on planes --------------------------------------------------------------------
// kGlobal: the three plane buffers of a workgroup in `scratch` (planes too large for LDS).
template <bool kGlobal>
__global__ __launch_bounds__(256) void dilate_plane_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                           int w, int h, int size, int plane_words, uint64_t* scratch) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int n = (w + 63) >> 6, words = h * n;
  const size_t off = (size_t)blockIdx.x * words;
  uint64_t* A = kGlobal ? scratch + (size_t)blockIdx.x * 3 * plane_words : smem;
  uint64_t* B = A + plane_words;
  uint64_t* T = B + plane_words;
  for (int i = threadIdx.x; i < words; i += blockDim.x) A[i] = src[off + i];
  __syncthreads();
  morph(A, B, T, w, h, n, size, true);
  for (int i = threadIdx.x; i < words; i += blockDim.x) dst[off + i] = B[i];
}

// Renderer border of every plane: label ∧ ¬erode_{size×size}(label) in 2D per plane (the
// SegmentationRenderer outlines each displayed slice; size = 2·radius + 1).
template <bool kGlobal>
__global__ __launch_bounds__(256) void border_plane_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                           int w, int h, int size, int plane_words, uint64_t* scratch) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int n = (w + 63) >> 6, words = h * n;
  const size_t off = (size_t)blockIdx.x * words;
  uint64_t* A = kGlobal ? scratch + (size_t)blockIdx.x * 3 * plane_words : smem;
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

// Ball dilation (se_shape = disc in 3D): one thread per output word; the ball of radius r is the
// union over (dz, dy) of the row segments |dx| ≤ floor(sqrt(r² − dy² − dz²)), so each word is the
// OR of ≤ (2r+1)² horizontally dilated words of the planes around it (reads hit L2: a 256² plane is
// 8 KiB). Out-of-volume rows are ignored.
__global__ __launch_bounds__(256) void dilate_ball_kernel(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst,
                                                          int w, int h, int d, int r) {
  const int n = (w + 63) >> 6;
  const size_t words = (size_t)h * n;
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= words * d) return;
  const int z = (int)(q / words);
  const int rem = (int)(q - (size_t)z * words);
  const int y = rem / n, i = rem - y * n;
  const uint64_t lm = last_mask(w);
  uint64_t acc = 0;
  for (int dz = -r; dz <= r; ++dz) {
    const int zz = z + dz;
    if (zz < 0 || zz >= d) continue;
    for (int dy = -r; dy <= r; ++dy) {
      const int yy = y + dy;
      const int k = disc_halfwidth(r * r - dy * dy - dz * dz);
      if (yy < 0 || yy >= h || k < 0) continue;
      acc |= hmorph_word(src + (size_t)zz * words + (size_t)yy * n, i, n, lm, k, true);
    }
  }
  dst[q] = i == n - 1 ? (acc & lm) : acc;
}

namespace {
int morph_plane_words(int w, int h) { return (h * ((w + 63) / 64) + 1) & ~1; }
bool morph_global(int w, int h) { return (size_t)morph_plane_words(w, h) * 3 * sizeof(uint64_t) + 1024 > kLdsBudget; }
}  // namespace

size_t morph3d_scratch_words(int w, int h, int d) {
  return morph_global(w, h) ? (size_t)d * 3 * (size_t)morph_plane_words(w, h) : 0;
}

void border_volume(const uint64_t* src, uint64_t* dst, int w, int h, int d, int radius, hipStream_t stream,
                   uint64_t* scratch) {
  const int plane_words = morph_plane_words(w, h);
  if (morph_global(w, h)) {
    if (!scratch) throw DeviceError("border_volume: planes above the LDS size need scratch (morph3d_scratch_words)");
    border_plane_kernel<true><<<d, 256, 0, stream>>>(src, dst, w, h, 2 * radius + 1, plane_words, scratch);
  } else {
    border_plane_kernel<false><<<d, 256, (size_t)plane_words * 3 * sizeof(uint64_t), stream>>>(
        src, dst, w, h, 2 * radius + 1, plane_words, nullptr);
  }
  check_launch("border_plane_kernel");
}

void dilate_volume(const uint64_t* src, uint64_t* dst, uint64_t* tmp, int w, int h, int d, int size, hipStream_t stream,
                   uint64_t* scratch, bool ball) {
  const int n = (w + 63) / 64;
  const int words = h * n;
  if (ball) {
    const size_t total = (size_t)words * d;
    dilate_ball_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(src, dst, w, h, d, size / 2);
    check_launch("dilate_ball_kernel");
    return;
  }
  const int plane_words = morph_plane_words(w, h);
  if (morph_global(w, h)) {
    if (!scratch) throw DeviceError("dilate_volume: planes above the LDS size need scratch (morph3d_scratch_words)");
    dilate_plane_kernel<true><<<d, 256, 0, stream>>>(src, tmp, w, h, size, plane_words, scratch);
  } else {
    dilate_plane_kernel<false><<<d, 256, (size_t)plane_words * 3 * sizeof(uint64_t), stream>>>(src, tmp, w, h, size,
                                                                                             plane_words, nullptr);
  }
  check_launch("dilate_plane_kernel");
  const size_t total = (size_t)words * d;
  dilate_z_kernel<<<(unsigned)((total + 255) / 256), 256, 0, stream>>>(tmp, dst, words, d, size / 2);
  check_launch("dilate_z_kernel");
}

// z-slab boundary step: one thread per plane word. The 26-connected touch is the 3×3 in-plane
// dilation of the neighbour's plane (dilate_plane3 in volume_slabs.cpp), formed on the fly.
__global__ __launch_bounds__(256) void slab_seed_kernel(const uint64_t* __restrict__ band, uint64_t* __restrict__ region,
                                                        const uint64_t* __restrict__ nb, int w, int h, int wpr,
                                                        int conn26, unsigned long long* __restrict__ added) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  uint64_t add = 0;
  if (i < h * wpr) {
    const int y = i / wpr, k = i - y * wpr;
    uint64_t t = nb[i];
    if (conn26) {
      const uint64_t last = (w & 63) ? ((1ull << (w & 63)) - 1ull) : ~0ull;
      auto hrow = [&](int yy) -> uint64_t {
        if (yy < 0 || yy >= h) return 0ull;
        const uint64_t* r = nb + (size_t)yy * wpr;
        const uint64_t v = r[k], prev = k > 0 ? r[k - 1] : 0ull, next = k + 1 < wpr ? r[k + 1] : 0ull;
        uint64_t acc = v | (v << 1) | (prev >> 63) | (v >> 1) | (next << 63);
        return k == wpr - 1 ? acc & last : acc;
      };
      t = hrow(y - 1) | hrow(y) | hrow(y + 1);
    }
    add = band[i] & t & ~region[i];
    if (add) region[i] |= add;
  }
  unsigned long long c = (unsigned long long)__popcll(add);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(added, c);
}

void launch_slab_seed(const uint64_t* band, uint64_t* region, const uint64_t* nb, int w, int h, bool conn26,
                      unsigned long long* added, hipStream_t stream) {
  const int wpr = (w + 63) / 64, n = h * wpr;
  if (n <= 0) return;
  slab_seed_kernel<<<(n + 255) / 256, 256, 0, stream>>>(band, region, nb, w, h, wpr, conn26 ? 1 : 0, added);
  check_launch("slab_seed_kernel");
}

void preload_volume() {
  hipFuncAttributes a;
  for (const void* f : {reinterpret_cast<const void*>(&srg3d_seed_kernel), reinterpret_cast<const void*>(&srg3d_kernel<false>),
                        reinterpret_cast<const void*>(&srg3d_kernel<true>), reinterpret_cast<const void*>(&dilate_plane_kernel<false>),
                        reinterpret_cast<const void*>(&dilate_plane_kernel<true>), reinterpret_cast<const void*>(&border_plane_kernel<false>),
                        reinterpret_cast<const void*>(&border_plane_kernel<true>), reinterpret_cast<const void*>(&dilate_z_kernel),
                        reinterpret_cast<const void*>(&slab_seed_kernel), reinterpret_cast<const void*>(&dilate_ball_kernel)})
    check_hip(hipFuncGetAttributes(&a, f), "preload volume kernels");
}

}  // namespace nm03::gpu
