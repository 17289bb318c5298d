// K1a — k×k median (VectorMedianFilter, main_sequential.cpp:204-206) on gfx950.
//
// * One workgroup = 256 threads = one 64×64 output tile of one slice (tile list built on host, so
//   slices of any size/type share a launch).
// * The clamp-to-edge input tile (64+k-1)² is staged in LDS as packed u16 PAIRS
//   (pixel[c], pixel[c+32]) so each v_pk_min_u16 / v_pk_max_u16 advances two medians.
//   Row stride is odd (PW|1 words) → the lane→(row, col-group) read pattern is conflict-free for
//   ds_read_b32 (8 rows × 4 groups per 32-lane half hit 32 distinct banks).
// * Thread (g, r) evaluates the generated selection network (tools/gen_median_net.py) for
//   outputs (r, 8g..8g+7) and (r, 32+8g..32+8g+7).
// * Medians are computed on order-preserving 16-bit keys: normalise+clip is monotone, so the
//   median of c(x) is c(median x) exactly (pixel_math.h). The same pass reduces per-slice min/max
//   keys for the original-image render window.
// * Engine batches (`blob` set): the tile is read straight from the uploaded blob — 12-bit packed
//   pairs (nm03/pack12.h) are decoded in the load — and each workgroup writes its 64×64 interior
//   as expanded 16-bit samples to `raw` for the render/JPEG stages. This replaces the separate
//   K0 expansion pass (one launch and one full read + write of the batch's samples less).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {
using nm03::gpu::vmax;
using nm03::gpu::vmin;
#include "nm03/median_net.inc"

template <int K>
__device__ __forceinline__ void run_net(const uint32_t* P, int stride, int r, int g, u16x2* out) {
  auto ld = [&](int rr, int cc) -> u16x2 { return as_u16x2(P[(r + rr) * stride + 8 * g + cc]); };
  if constexpr (K == 3) median_net_k3_w8_h1<u16x2>(ld, out);
  else if constexpr (K == 5) median_net_k5_w8_h1<u16x2>(ld, out);
  else if constexpr (K == 7) median_net_k7_w8_h1<u16x2>(ld, out);
  else median_net_k9_w8_h1<u16x2>(ld, out);
}

template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K <= 7 ? 4 : 2))) void median_kernel(const uint16_t* __restrict__ raw, uint16_t* __restrict__ med,
                                                     const SliceDesc* __restrict__ descs,
                                                     const TileDesc* __restrict__ tiles, SliceStats* stats,
                                                     uint32_t* __restrict__ tile_mm, int dbg,
                                                     const uint16_t* __restrict__ blob, uint16_t* __restrict__ raw_out) {
  constexpr int R = K / 2;
  constexpr int PW = 32 + K - 1;  // pair columns
  constexpr int PS = PW | 1;      // odd stride: conflict-free ds_read_b32
  constexpr int PR = 64 + K - 1;  // rows
  __shared__ uint32_t P[PR * PS];

  const TileDesc t = tiles[blockIdx.x];
  const SliceDesc d = descs[t.slice];
  const int x0 = t.tx * kMedTileW, y0 = t.ty * kMedTileH;
  const int W = d.w, H = d.h;
  // Source: the expanded raw buffer, or (blob set) the slice as uploaded — plain 16-bit samples or
  // a 12-bit little-endian stream (sample p at bits [12p, 12p + 12) from the slice's first byte).
  const bool from_blob = blob != nullptr;
  const bool packed = from_blob && (d.flags & kSliceFlagPacked12);
  const uint16_t* src = from_blob ? blob + d.blob_off : raw + d.raw_off;
  const uint8_t* pb = reinterpret_cast<const uint8_t*>(src);
  auto sample = [&](int y, int x) -> uint16_t {
    const uint32_t p = (uint32_t)y * W + x;
    if (!packed) return src[p];
    const uint32_t o = (3u * p) >> 1;
    const uint32_t v = (uint32_t)pb[o] | ((uint32_t)pb[o + 1] << 8);
    return (uint16_t)((p & 1u) ? (v >> 4) : (v & 0xFFFu));
  };
  // Expanded-sample side output (blob mode): the tile interior, each pixel written by one task.
  uint16_t* rdst = from_blob ? raw_out + d.raw_off : nullptr;
  const int yin_hi = min(y0 + kMedTileH, H), xin_hi = min(x0 + kMedTileW, W);

  uint32_t kmin = 0xFFFFu, kmax = 0u;
  // Keys of the staged samples (key_from_raw, pixel_math.h) without per-pixel type selects: with
  // u = the sample's low stored_bits bits, a signed sample's key (sign-extended, bit 15 flipped) is
  // ((u ^ m) + 0x8000 − m) mod 2^16 with m = 2^(stored_bits − 1) — the sign-extension identity
  // (u ^ m) − m — and an unsigned sample's key is u itself (m = c = 0). Two keys go into one pair
  // word with a byte permute (the high garbage of the signed form dropped), and the tile's key range
  // is kept as packed u16 minima / maxima (one v_pk_min_u16 / v_pk_max_u16 per pair).
  const uint32_t ksb = d.stored_bits;
  const uint32_t km = d.type == kI16 ? 1u << (ksb - 1u) : 0u, kc = d.type == kI16 ? 0x8000u - km : 0u;
  auto key_pair = [&](uint32_t lo, uint32_t hi) -> uint32_t {
    const uint32_t a = (__builtin_amdgcn_ubfe(lo, 0u, ksb) ^ km) + kc;
    const uint32_t b = (__builtin_amdgcn_ubfe(hi, 0u, ksb) ^ km) + kc;
    return __builtin_amdgcn_perm(b, a, 0x05040100u);  // (a & 0xFFFF) | (b << 16)
  };
  u16x2 pmin = as_u16x2(0xFFFFFFFFu), pmax = as_u16x2(0u);
  if ((W & 3) == 0 && (d.raw_off & 3) == 0 && (!from_blob || packed || (d.blob_off & 3) == 0)) {
    // Vector path: window pixels p = 0..71 are image columns x0-4+p (8-byte aligned groups of
    // 4). Pair column c holds window pixels c+4-R (low half) and c+36-R (high half), so a task
    // (row, group gi < 10) takes groups gi and gi+8 and writes up to 4 pair words. W % 4 == 0 and
    // xs ≡ x0 (mod 4), so a group is wholly inside the image or wholly outside — then every pixel
    // clamps to one edge pixel, which the clamped edge group holds: one 8-byte (or, 12-bit packed,
    // two dword) load per group and no per-pixel path. All of a thread's loads are issued first
    // (phase A), then decoded (phase B): every wave of the launch is loading at the same time, so
    // load → use chains would expose the memory latency once per task.
    constexpr int NT = (PR * 10 + 255) / 256;  // tasks per thread
    uint2 ld[NT][2];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int i = threadIdx.x + 256 * t;
      if (i >= PR * 10) break;
      const int r = i / 10, gi = i - r * 10;
      const int y = clampi(y0 - R + r, 0, H - 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int xs = clampi(x0 - 4 + 4 * (gi + 8 * h), 0, W - 4);
        if (packed) {
          // 4 samples = 48 bits at byte o = 1.5·p (p = y·W + xs ≡ 0 mod 4, so o is even): two
          // aligned dword loads from o & ~3 cover them (the device blob has tail slack for the
          // 2 bytes this can read past a slice that ends the blob).
          const size_t o = ((size_t)y * W + xs) * 3 >> 1;
          ld[t][h] = *reinterpret_cast<const uint2*>(pb + (o & ~(size_t)3));
        } else {
          ld[t][h] = *reinterpret_cast<const uint2*>(src + (size_t)y * W + xs);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int i = threadIdx.x + 256 * t;
      if (i >= PR * 10) break;
      const int r = i / 10, gi = i - r * 10;
      const int yy = y0 - R + r;
      const int y = clampi(yy, 0, H - 1);
      const bool row_in = rdst && yy >= y0 && yy < yin_hi;
      uint16_t px[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int g4 = gi + 8 * h;
        const int xs = x0 - 4 + 4 * g4;
        uint2 v = ld[t][h];
        if (packed) {
          const size_t o = ((size_t)y * W + clampi(xs, 0, W - 4)) * 3 >> 1;
          const uint64_t b = ((uint64_t)v.x | ((uint64_t)v.y << 32)) >> ((o & 2) * 8);
          v.x = ((uint32_t)b & 0xFFFu) | (((uint32_t)(b >> 12) & 0xFFFu) << 16);
          v.y = ((uint32_t)(b >> 24) & 0xFFFu) | (((uint32_t)(b >> 36) & 0xFFFu) << 16);
        }
        px[h][0] = (uint16_t)v.x;
        px[h][1] = (uint16_t)(v.x >> 16);
        px[h][2] = (uint16_t)v.y;
        px[h][3] = (uint16_t)(v.y >> 16);
        if (xs < 0) px[h][1] = px[h][2] = px[h][3] = px[h][0];
        if (xs >= W) px[h][0] = px[h][1] = px[h][2] = px[h][3];
        // Expanded-sample side output: groups 8 and 9 are taken twice (as lo and as hi); only the
        // lo copy stores them.
        const bool store = h == 0 ? gi >= 1 : (g4 >= 10 && g4 <= 16);
        if (store && row_in && xs >= x0 && xs < xin_hi) {
          // Non-temporal: read once, by the encoder, after the sharpen and SRG kernels (29.4 → 28.7 µs
          // per 96-slice batch, profiles/r4/median_ntstore/).
          typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
          __builtin_nontemporal_store(u32x2{v.x, v.y}, reinterpret_cast<u32x2*>(rdst + (size_t)yy * W + xs));
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 4 * gi + q - (4 - R);
        if (c < 0 || c >= PW) continue;
        const uint32_t kp = key_pair(px[0][q], px[1][q]);
        P[r * PS + c] = kp;
        pmin = vmin(pmin, as_u16x2(kp));
        pmax = vmax(pmax, as_u16x2(kp));
      }
    }
    kmin = min((uint32_t)pmin.x, (uint32_t)pmin.y);
    kmax = max((uint32_t)pmax.x, (uint32_t)pmax.y);
  } else {
    for (int i = threadIdx.x; i < PR * PW; i += 256) {
      const int r = i / PW, c = i - r * PW;
      const int yy = y0 - R + r;
      const int y = clampi(yy, 0, H - 1);
      const int ul = x0 - R + c, uh = ul + 32;
      const uint16_t sl = sample(y, clampi(ul, 0, W - 1)), sh = sample(y, clampi(uh, 0, W - 1));
      if (rdst && yy >= y0 && yy < yin_hi) {
        if (ul >= x0 && ul < min(x0 + 32, xin_hi)) rdst[(size_t)yy * W + ul] = sl;
        if (uh >= x0 + 32 && uh < xin_hi) rdst[(size_t)yy * W + uh] = sh;
      }
      const uint32_t kl = key_from_raw(sl, d.type, d.stored_bits);
      const uint32_t kh = key_from_raw(sh, d.type, d.stored_bits);
      P[r * PS + c] = kl | (kh << 16);
      kmin = min(kmin, min(kl, kh));
      kmax = max(kmax, max(kl, kh));
    }
  }
  __syncthreads();

  const int g = threadIdx.x & 3, r = threadIdx.x >> 2;
  u16x2 out[8];
  if (dbg == 1) {  // profiling variant: tile load + store only
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = as_u16x2(P[(r + R) * PS + 8 * g + j + R]);
  } else {
    run_net<K>(P, PS, r, g, out);
  }

  const int y = y0 + r;
  if (y < H) {
    uint16_t* dst = med + d.raw_off + (size_t)y * W;
    const int xl = x0 + 8 * g;
    if (xl + 8 <= W && xl + 40 <= W && (W & 7) == 0) {
      // Fast path: two 16-byte stores.
      uint4 lo, hi;
      lo.x = out[0].x | ((uint32_t)out[1].x << 16);
      lo.y = out[2].x | ((uint32_t)out[3].x << 16);
      lo.z = out[4].x | ((uint32_t)out[5].x << 16);
      lo.w = out[6].x | ((uint32_t)out[7].x << 16);
      hi.x = out[0].y | ((uint32_t)out[1].y << 16);
      hi.y = out[2].y | ((uint32_t)out[3].y << 16);
      hi.z = out[4].y | ((uint32_t)out[5].y << 16);
      hi.w = out[6].y | ((uint32_t)out[7].y << 16);
      *reinterpret_cast<uint4*>(dst + xl) = lo;
      *reinterpret_cast<uint4*>(dst + xl + 32) = hi;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (xl + j < W) dst[xl + j] = out[j].x;
        if (xl + 32 + j < W) dst[xl + 32 + j] = out[j].y;
      }
    }
  }

  // Per-slice key range (render window of the original image). Same-address device atomics from
  // every wave of a slice serialise (≈12 us per 64-slice batch): instead each tile stores its
  // range and the sharpen kernel reduces the slice's tiles.
  kmin = wave_min_u32(kmin);
  kmax = wave_max_u32(kmax);
  if (tile_mm) {
    __shared__ uint32_t smm[8];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
      smm[2 * wv] = kmin;
      smm[2 * wv + 1] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t a = smm[0], b = smm[1];
      for (int i = 1; i < 4; ++i) {
        a = min(a, smm[2 * i]);
        b = max(b, smm[2 * i + 1]);
      }
      tile_mm[2 * blockIdx.x] = a;
      tile_mm[2 * blockIdx.x + 1] = b;
    }
  } else if ((threadIdx.x & 63) == 0 && stats) {
    atomicMin(&stats[t.slice].key_min, kmin);
    atomicMax(&stats[t.slice].key_max, kmax);
  }
}

void launch_median(const uint16_t* raw, uint16_t* med, const SliceDesc* descs, const TileDesc* tiles, int ntiles,
                   int k, SliceStats* stats, hipStream_t stream, uint32_t* tile_mm, const uint16_t* blob,
                   uint16_t* raw_out) {
  if (blob && !raw_out) throw DeviceError("launch_median: blob input needs a raw_out buffer");
  if (ntiles <= 0) return;
  dim3 grid(ntiles), block(256);
  static const int dbg = profile_variant("median");  // 1: tile load + store only (output invalid)
  switch (k) {
    case 3: median_kernel<3><<<grid, block, 0, stream>>>(raw, med, descs, tiles, stats, tile_mm, dbg, blob, raw_out); break;
    case 5: median_kernel<5><<<grid, block, 0, stream>>>(raw, med, descs, tiles, stats, tile_mm, dbg, blob, raw_out); break;
    case 7: median_kernel<7><<<grid, block, 0, stream>>>(raw, med, descs, tiles, stats, tile_mm, dbg, blob, raw_out); break;
    case 9: median_kernel<9><<<grid, block, 0, stream>>>(raw, med, descs, tiles, stats, tile_mm, dbg, blob, raw_out); break;
    default: throw DeviceError("median window must be 3, 5, 7 or 9 (got " + std::to_string(k) + ")");
  }
  check_launch("median_kernel");
}

void preload_median() {
  hipFuncAttributes a;
  for (const void* f : {reinterpret_cast<const void*>(&median_kernel<3>), reinterpret_cast<const void*>(&median_kernel<5>),
                        reinterpret_cast<const void*>(&median_kernel<7>), reinterpret_cast<const void*>(&median_kernel<9>)})
    check_hip(hipFuncGetAttributes(&a, f), "preload median_kernel");
}

}  // namespace nm03::gpu
