// K1b — IntensityNormalization + IntensityClipping (applied to the median keys; exact because
// both are monotone), ImageSharpening (9×9 Gaussian unsharp mask, main_sequential.cpp:208-210)
// and the SeededRegionGrowing band test [0.74, 0.91] (main_sequential.cpp:232-233).
//
// One workgroup = 256 threads = two 64×64 output tiles in turn (the second tile's loads issued with
// the first's); the mask radius R is a template parameter (compile-time tile geometry: no runtime
// divisions in the index math).
//  1. the clamp-to-edge (64+2R)² input tile is loaded in 8-byte groups of 4 median keys
//     (per-key clamped loads only where a group leaves the image), normalised+clipped once per
//     key and kept in LDS as f32;
//  2. vertical pass: a thread owns a column pair × 16 rows and slides a (16+2R)-value window of
//     pairs held in registers (each LDS value read once instead of 2R+1 times);
//  3. horizontal pass + combine + band: a thread owns 16 columns of a row (register window of
//     overlapping pairs); the band bits of the four 16-column segments form the row's mask word.
// Both passes compute two outputs per packed f32 instruction (one v_pk_fma_f32 per tap).
// The Gaussian is applied separably in the contract order of golden::sharpen (vertical, then
// horizontal, taps ascending, one fma per tap; no implicit contraction anywhere), so the result is
// bit-identical to the CPU golden model.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/kernels.h"
#include "nm03/pixel_math.h"

namespace nm03::gpu {

constexpr int kMaxR = 7;

// Two adjacent f32 in one register pair: the stencil passes run on packed f32 (v_pk_fma_f32 /
// v_pk_add_f32, per-lane IEEE rounding, so results are those of the scalar ops).
//
// LDS layout: row stride CS ≡ 2 (mod 4) dwords, so every even column pair is 8-byte aligned and
// moves with one ds_read_b64 / ds_write_b64. A b64 access is served 16 lanes at a time; 16 lanes
// on consecutive pairs of one row cover all 32 banks (vertical pass), and 16 lanes on 16
// consecutive rows hit banks (CS·r + {0,1}) mod 32 — distinct for r < 16 because CS/2 is odd
// (horizontal pass). The r2 layout (odd stride, pairs as ds_read2_b32 at stride 2 across lanes)
// ran at 2.49 bank-conflict cycles per LDS instruction (profiles/r2/pmc).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 lds_pair(const float* p) { return f32x2{p[0], p[1]}; }
__device__ __forceinline__ f32x2 lds_pair_a(const float* p) { return *reinterpret_cast<const f32x2*>(p); }
__device__ __forceinline__ void lds_store_pair(float* p, f32x2 v) { *reinterpret_cast<f32x2*>(p) = v; }
// One tap on two outputs: v_pk_fma_f32 (IEEE fma per lane, as std::fma in golden::sharpen).
__device__ __forceinline__ f32x2 pk_fma(float t, f32x2 v, f32x2 acc) {
  return __builtin_elementwise_fma(f32x2{t, t}, v, acc);
}
static_assert(kShpTileW == 64 && kShpTileH == 64, "sharpen tile is 64x64");

template <int R>
__global__ __launch_bounds__(256) void sharpen_band_kernel(const uint16_t* __restrict__ med, uint64_t* __restrict__ band,
                                                           float* __restrict__ sharpened,
                                                           const SliceDesc* __restrict__ descs,
                                                           const TileDesc* __restrict__ tiles, PipeConsts pc,
                                                           SliceStats* stats, const uint32_t* __restrict__ tile_mm,
                                                           const float* __restrict__ lut, int ntiles) {
  constexpr int TW = kShpTileW, TH = kShpTileH;
  constexpr int CW = TW + 2 * R, CH = TH + 2 * R;
  constexpr int CS = CW % 4 == 0 ? CW + 2 : CW;  // LDS row stride ≡ 2 (mod 4)
  constexpr int RA = (R + 3) / 4;                 // 4-key groups of halo on each side
  constexpr int G = TW / 4 + 2 * RA;              // groups per input row
  constexpr int OFS = 4 * RA - R;                 // window column of tile column 0
  // Vertical pass: 7 row blocks of RB rows (the last one starts at TH - RB and recomputes 6 rows),
  // so (32 + R)·7 tasks keep all 256 threads busy for R ≤ 4 (16-row blocks left 112 idle).
  constexpr int RB = 10, NB = (TH + RB - 1) / RB;
  static_assert(CS % 4 == 2, "pair alignment");
  __shared__ __attribute__((aligned(16))) float C[CH * CS];
  __shared__ __attribute__((aligned(16))) float T[TH * CS];
  // Two tiles per workgroup — tiles 2L and 2L+1 of the XCD-ordered list — with the second tile's
  // keys loaded together with the first's, so their latency hides behind the first tile's passes
  // and the launch is one round of workgroups (1536 tiles → 768 workgroups, 4 resident per CU).
  __shared__ uint16_t bm[4 * TH];
  constexpr int NT = (CH * G + 255) / 256;  // tasks per thread
  // Task i → (row r, group g): the first CH·16 tasks are the 16 interior groups of each row, so a
  // 16-lane store group stays on one row (with the rotation below: all 32 banks); the 2·RA halo
  // groups per row follow.
  auto task_rg = [](int i, int& r, int& g) {
    if (i < CH * 16) {
      r = i >> 4;
      g = (i & 15) + RA;
    } else {
      const int k = i - CH * 16;
      if constexpr (RA > 0) {
        r = k / (2 * RA);
        const int hg = k - r * (2 * RA);
        g = hg < RA ? hg : 16 + hg;
      } else {
        r = g = 0;
      }
    }
  };
  auto fast_path = [](const SliceDesc& d) { return (d.w & 3) == 0 && (d.raw_off & 3) == 0; };
  auto load_keys = [&](const TileDesc& tl, const SliceDesc& d, uint2 (&v)[NT]) __attribute__((always_inline)) {
    const int x0 = tl.tx * TW, y0 = tl.ty * TH, W = d.w, H = d.h;
    const uint16_t* src = med + d.raw_off;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int i = threadIdx.x + 256 * t;
      if (i >= CH * G) break;
      int r, g;
      task_rg(i, r, g);
      const int y = clampi(y0 - R + r, 0, H - 1);
      const uint16_t* row = src + (size_t)y * W;
      // W % 4 == 0 and xs ≡ x0 (mod 4): a group is wholly inside or wholly outside the image, and
      // an outside group clamps to one edge pixel — loaded with the edge group (no scalar path).
      const int xs = x0 - 4 * RA + 4 * g;
      v[t] = *reinterpret_cast<const uint2*>(row + clampi(xs, 0, W - 4));
    }
  };
  const uint32_t lw = xcd_tile(blockIdx.x, gridDim.x);
  const bool two = 2 * lw + 1 < (uint32_t)ntiles;
  const TileDesc tA = tiles[2 * lw];
  const TileDesc tB = tiles[two ? 2 * lw + 1 : 2 * lw];
  const SliceDesc dA = descs[tA.slice], dB = descs[tB.slice];
  uint2 vA[NT], vB[NT];
  if (fast_path(dA)) load_keys(tA, dA, vA);
  if (two && fast_path(dB)) load_keys(tB, dB, vB);
  auto tile_body = [&](const TileDesc& t, const SliceDesc& d, const uint2 (&v)[NT]) __attribute__((always_inline)) {
    const int x0 = t.tx * TW, y0 = t.ty * TH;
    const int W = d.w, H = d.h;
    const uint16_t* src = med + d.raw_off;
    NormClip nc;
    nc.slope = d.slope;
    nc.intercept = d.intercept;
    nc.nmin = pc.nmin;
    nc.nmax = pc.nmax;
    nc.nlow = pc.nlow;
    nc.nhigh = pc.nhigh;
    nc.cmin = pc.cmin;
    nc.cmax = pc.cmax;

    // The slice's first tile folds the median tiles' key ranges into stats (render window).
    if (tile_mm && stats && t.tx == 0 && t.ty == 0 && threadIdx.x < 64) {
      const int ntl = ((W + kMedTileW - 1) / kMedTileW) * ((H + kMedTileH - 1) / kMedTileH);
      uint32_t a = 0xFFFFFFFFu, b = 0u;
      for (int i = threadIdx.x; i < ntl; i += 64) {
        a = min(a, tile_mm[2 * (d.med_tile0 + i)]);
        b = max(b, tile_mm[2 * (d.med_tile0 + i) + 1]);
      }
      a = wave_min_u32(a);
      b = wave_max_u32(b);
      if (threadIdx.x == 0) {
        stats[t.slice].key_min = a;
        stats[t.slice].key_max = b;
      }
    }

    // ---- 1. input tile → normalised+clipped f32 in LDS ------------------------------------------
    if ((W & 3) == 0 && (d.raw_off & 3) == 0) {
      // Window columns x0 - 4·RA + 4g + q; tile column c = 4g + q - (4·RA - R). All of a thread's
      // loads are issued before any is consumed: every wave of the launch is in this phase at the
      // same time, so a load → use → load chain would expose the memory latency once per task.
      // Store order rotated per 8-lane group so the lanes of one store instruction spread over the
      // banks: a ds_write_b64 is served 16 lanes at a time, bank (a/4) mod 32; lanes 0–7 write pair
      // h at dwords 4g + 2h, lanes 8–15 pair 1 − h at 4(g + 8) + 2(1 − h) ≡ the other 16 banks.
      const int rot = (threadIdx.x >> 3) & 3;
      // Key → normalised+clipped value: the slice's lookup table (one gather from an L1/L2-resident
      // table built on the host from the same norm_clip_key) or the function itself — its IEEE
      // division alone is ≈13 VALU per key. The choice is workgroup-uniform: two copies of the loop.
      auto stage = [&](auto use_lut) {
      constexpr bool kLut = decltype(use_lut)::value;
      const uint32_t toff = d.lut_off, tbase = d.lut_base;
      auto conv = [&](uint16_t key) -> float {
        if constexpr (kLut) return lut[toff + ((uint32_t)key - tbase)];  // key ≥ lut_base (its key range)
        else return norm_clip_key(key, d.type, nc);
      };
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int i = threadIdx.x + 256 * t;
        if (i >= CH * G) break;
        int r, g;
        task_rg(i, r, g);
        const int xs = x0 - 4 * RA + 4 * g;
        uint16_t px[4] = {(uint16_t)v[t].x, (uint16_t)(v[t].x >> 16), (uint16_t)v[t].y, (uint16_t)(v[t].y >> 16)};
        if (xs < 0) px[1] = px[2] = px[3] = px[0];
        if (xs >= W) px[0] = px[1] = px[2] = px[3];
        if constexpr (OFS % 2 == 0) {
          // Keys (0,1) and (2,3) land on even window columns: two aligned pair stores.
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int h = (j + rot) & 1;
            const int c = 4 * g + 2 * h - OFS;
            const f32x2 kv{conv(h ? px[2] : px[0]), conv(h ? px[3] : px[1])};
            if (c >= 0 && c < CW) lds_store_pair(C + r * CS + c, kv);
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int q = (j + rot) & 3;
            const uint16_t key = q == 0 ? px[0] : q == 1 ? px[1] : q == 2 ? px[2] : px[3];  // selects, no scratch
            const int c = 4 * g + q - OFS;
            if (c >= 0 && c < CW) C[r * CS + c] = conv(key);
          }
        }
      }
      };
      if (lut && d.lut_off != kNoLut) stage(std::true_type{});
      else stage(std::false_type{});
    } else {
      for (int i = threadIdx.x; i < CH * CW; i += 256) {
        const int r = i / CW, c = i - r * CW;
        const int y = clampi(y0 - R + r, 0, H - 1), x = clampi(x0 - R + c, 0, W - 1);
        C[r * CS + c] = norm_clip_key(src[(size_t)y * W + x], d.type, nc);
      }
    }
    __syncthreads();

    // ---- 2. vertical pass: columns (c, c+1), rows [r0, r0 + RB) from a register window of
    //         column pairs; every tap is one v_pk_fma_f32 for two outputs ------------------------------
    constexpr int CP = CW / 2;  // CW = 64 + 2R is even
    // Task → (block, pair): the first 32·NB tasks take pairs 0..31 (a 16-lane group of a b64 access
    // stays inside one row block: conflict-free), the (CP − 32)·NB remaining pairs follow.
    for (int task = threadIdx.x; task < CP * NB; task += 256) {
      int rb, cp;
      if (task < 32 * NB) {
        rb = task >> 5;
        cp = task & 31;
      } else {
        constexpr int X = CP > 32 ? CP - 32 : 1;  // (CP = 32 never gets here)
        const int k = task - 32 * NB;
        rb = k / X;
        cp = 32 + (k - rb * X);
      }
      const int c = 2 * cp;
      const int r0 = min(rb * RB, TH - RB);
      f32x2 win[RB + 2 * R];
#pragma unroll
      for (int k = 0; k < RB + 2 * R; ++k) win[k] = lds_pair_a(C + (r0 + k) * CS + c);
#pragma unroll
      for (int rr = 0; rr < RB; ++rr) {
        f32x2 acc = 0.0f;
#pragma unroll
        for (int k = 0; k <= 2 * R; ++k) acc = pk_fma(pc.taps[k], win[rr + k], acc);
        lds_store_pair(T + (r0 + rr) * CS + c, acc);
      }
    }
    __syncthreads();

    // ---- 3. horizontal pass + combine + band: a thread owns row r, columns [16·seg, 16·seg + 16)
    //         and keeps the overlapping column pairs (a, a+1) of its (16+2R)-value window in
    //         registers, so output pairs (j, j+1) take packed f32 ops as in the vertical pass; band
    //         bits go through LDS to form the 64-bit row words. Wave = segment, lane = row: the
    //         window is read as 8 + R aligned pairs (the odd-offset pairs are register moves).
    const int r = threadIdx.x & (TH - 1), seg = threadIdx.x / TH;
    const int y = y0 + r;
    float smin = INFINITY, smax = -INFINITY;
    {
      f32x2 ev[8 + R];
#pragma unroll
      for (int b = 0; b < 8 + R; ++b) ev[b] = lds_pair_a(T + r * CS + 16 * seg + 2 * b);
      f32x2 pw[16 + 2 * R - 1];
#pragma unroll
      for (int a = 0; a < 16 + 2 * R - 1; ++a) pw[a] = (a & 1) ? f32x2{ev[a >> 1].y, ev[(a >> 1) + 1].x} : ev[a >> 1];
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < 16; j += 2) {
        f32x2 acc = 0.0f;
#pragma unroll
        for (int k = 0; k <= 2 * R; ++k) acc = pk_fma(pc.taps[k], pw[j + k], acc);
        // sharpen_combine (pixel_math.h) on both lanes: s = c + gain·(c − b), same rounding steps.
        const float* cp = C + (r + R) * CS + 16 * seg + j + R;
        f32x2 cv;
        if constexpr (R % 2 == 0) cv = lds_pair_a(cp);
        else cv = lds_pair(cp);
        const f32x2 dd = cv - acc;
        const f32x2 gg = pc.gain * dd;
        const f32x2 sv = cv + gg;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float v = h ? sv.y : sv.x;
          const int xj = x0 + 16 * seg + j + h;
          const bool inside = xj < W && y < H;
          bits |= (inside && in_band(v, pc.band_lo, pc.band_hi)) ? (1u << (j + h)) : 0u;
          if (sharpened && inside) {
            sharpened[d.f32_off + (size_t)y * W + xj] = v;
            smin = fminf(smin, v);
            smax = fmaxf(smax, v);
          }
        }
      }
      bm[seg * TH + r] = (uint16_t)bits;
    }
    __syncthreads();
    if (threadIdx.x < TH && y0 + (int)threadIdx.x < H) {
      const uint16_t* q = bm + threadIdx.x;
      const uint64_t word = (uint64_t)q[0] | ((uint64_t)q[TH] << 16) | ((uint64_t)q[2 * TH] << 32) |
                            ((uint64_t)q[3 * TH] << 48);
      band[d.mask_off + (size_t)(y0 + threadIdx.x) * d.wpr + t.tx] = word;
    }
    if (sharpened && stats) {
      uint32_t a = float_to_ordered(smin), b = float_to_ordered(smax);
      a = wave_min_u32(a);
      b = wave_max_u32(b);
      if ((threadIdx.x & 63) == 0) {
        atomicMin(&stats[t.slice].s_min, a);
        atomicMax(&stats[t.slice].s_max, b);
      }
    }
  };
  tile_body(tA, dA, vA);
  if (two) tile_body(tB, dB, vB);
}

void launch_sharpen_band(const uint16_t* med, uint64_t* band, float* sharpened, const SliceDesc* descs,
                         const TileDesc* tiles, int ntiles, const PipeConsts& pc, SliceStats* stats,
                         hipStream_t stream, const uint32_t* tile_mm, const float* lut) {
  if (ntiles <= 0) return;
#define NM03_SHARPEN_CASE(RR)                                                                              \
  case RR:                                                                                               \
    sharpen_band_kernel<RR><<<(ntiles + 1) / 2, 256, 0, stream>>>(med, band, sharpened, descs, tiles, pc, stats, tile_mm, lut, ntiles); \
    break;
  switch (pc.mask_radius) {
    NM03_SHARPEN_CASE(0)
    NM03_SHARPEN_CASE(1)
    NM03_SHARPEN_CASE(2)
    NM03_SHARPEN_CASE(3)
    NM03_SHARPEN_CASE(4)
    NM03_SHARPEN_CASE(5)
    NM03_SHARPEN_CASE(6)
    NM03_SHARPEN_CASE(7)
    default: throw DeviceError("sharpen mask must be ≤ 15");
  }
#undef NM03_SHARPEN_CASE
  check_launch("sharpen_band_kernel");
}

// Normalise+clip table of one slice format (engine.cpp norm_lut): out[i] = norm_clip_key(base + i)
// for the 2^bits keys of the format, with the very function the sharpen's fallback path and the
// golden model evaluate (pixel_math.h, no FP contraction): bit-identical to a host-built table,
// without a synchronous pageable host→device copy on a slot thread.
__global__ __launch_bounds__(256) void build_norm_lut_kernel(float* __restrict__ out, uint32_t n, uint32_t base,
                                                             uint8_t type, NormClip nc) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = norm_clip_key((uint16_t)(base + i), type, nc);
}

void launch_build_norm_lut(float* out, uint32_t n, uint32_t base, uint8_t type, const NormClip& nc, hipStream_t stream) {
  if (!n) return;
  build_norm_lut_kernel<<<(n + 255) / 256, 256, 0, stream>>>(out, n, base, type, nc);
  check_launch("build_norm_lut_kernel");
}

void preload_sharpen() {
  hipFuncAttributes a;
  for (const void* f : {reinterpret_cast<const void*>(&sharpen_band_kernel<0>), reinterpret_cast<const void*>(&sharpen_band_kernel<1>),
                        reinterpret_cast<const void*>(&sharpen_band_kernel<2>), reinterpret_cast<const void*>(&sharpen_band_kernel<3>),
                        reinterpret_cast<const void*>(&sharpen_band_kernel<4>), reinterpret_cast<const void*>(&sharpen_band_kernel<5>),
                        reinterpret_cast<const void*>(&sharpen_band_kernel<6>), reinterpret_cast<const void*>(&sharpen_band_kernel<7>),
                        reinterpret_cast<const void*>(&build_norm_lut_kernel)})
    check_hip(hipFuncGetAttributes(&a, f), "preload sharpen_band_kernel");
}

}  // namespace nm03::gpu
