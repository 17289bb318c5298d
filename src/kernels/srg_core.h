// Shared LDS bit-plane region-growing core (2D slices: k2_srg_morph.hip, 3D plane sweeps:
// k5_volume.hip). See k2_srg_morph.hip for the algorithm description.
#pragma once

#include <hip/hip_runtime.h>

#include "device_util.h"

namespace nm03::gpu {

__device__ __forceinline__ uint64_t brev64(uint64_t x) { return __builtin_bitreverse64(x); }

__device__ __forceinline__ uint64_t fill_up(uint64_t m, uint64_t s) { return (((m + s) ^ m) & m) | s; }

// Fill runs of M (n words) that intersect R, both directions. Returns true if R changed.
__device__ __forceinline__ bool fill_row(uint64_t* R, const uint64_t* M, int n) {
  bool changed = false;
  uint64_t carry = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t m = M[i], r = R[i];
    const uint64_t s = (r & m) | (carry & m & 1ull);
    const uint64_t f = fill_up(m, s);
    const uint64_t nr = r | f;
    changed |= nr != r;
    R[i] = nr;
    carry = f >> 63;
  }
  carry = 0;
  for (int i = n - 1; i >= 0; --i) {
    const uint64_t m = brev64(M[i]), r = brev64(R[i]);
    const uint64_t s = (r & m) | (carry & m & 1ull);
    const uint64_t f = fill_up(m, s);
    const uint64_t nr = r | f;
    changed |= nr != r;
    R[i] = brev64(nr);
    carry = f >> 63;
  }
  return changed;
}

// fill_row for a compile-time word count: all loads issued up front, both sweeps in registers,
// one store per word (the runtime-n loop above serialises an LDS round trip per word and sweep).
template <int NW>
__device__ __forceinline__ bool fill_row_n(uint64_t* R, const uint64_t* M) {
  uint64_t m[NW], r[NW], o[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    m[i] = M[i];
    r[i] = R[i];
  }
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint64_t s = (r[i] & m[i]) | (carry & m[i] & 1ull);
    const uint64_t f = fill_up(m[i], s);
    o[i] = r[i] | f;
    carry = f >> 63;
  }
  carry = 0;
  bool changed = false;
#pragma unroll
  for (int i = NW - 1; i >= 0; --i) {
    const uint64_t mb = brev64(m[i]), rb = brev64(o[i]);
    const uint64_t s = (rb & mb) | (carry & mb & 1ull);
    const uint64_t f = fill_up(mb, s);
    o[i] = brev64(rb | f);
    carry = f >> 63;
    changed |= o[i] != r[i];
    R[i] = o[i];
  }
  return changed;
}

template <int NW>
__device__ __forceinline__ bool fill_row_any(uint64_t* R, const uint64_t* M, int n) {
  if constexpr (NW > 0) return fill_row_n<NW>(R, M);
  else return fill_row(R, M, n);
}

// Transpose a [rows][wpr] bit-plane (row stride ss words) into [cols][ceil(rows/64)] (row stride
// ds words; 0 = dense). Returns (via flag) whether any destination word changed when `cmp` is set.
__device__ inline void transpose_plane(const uint64_t* src, int rows, int wpr, uint64_t* dst, int cols, bool cmp, int* flag,
                                       int ss = 0, int ds = 0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int hb = (rows + 63) >> 6;
  if (ss == 0) ss = wpr;
  if (ds == 0) ds = hb;
  const int nblocks = hb * wpr;
  bool changed = false;
  for (int b = wave; b < nblocks; b += nw) {
    const int bi = b / wpr, bj = b - bi * wpr;
    const int row = bi * 64 + lane;
    uint64_t x = row < rows ? src[row * ss + bj] : 0ull;
    x = wave_transpose64(x, lane);
    const int drow = bj * 64 + lane;
    if (drow < cols) {
      uint64_t* p = dst + drow * ds + bi;
      if (cmp && *p != x) changed = true;
      *p = x;
    }
  }
  if (cmp && changed) *flag = 1;
}

__device__ __forceinline__ uint64_t last_mask(int w) {
  const int r = w & 63;
  return r ? ((1ull << r) - 1ull) : ~0ull;
}

// Horizontal morphology of one row: OR (dilate) or AND (erode, outside = 1) of shifts by ±1..±r.
// NW > 0: compile-time word count (n ignored), the row is loaded into registers once.
template <int NW = 0>
__device__ __forceinline__ void morph_row_h(const uint64_t* src, uint64_t* dst, int n, int w, int r, bool dil) {
  const uint64_t lm = last_mask(w);
  constexpr int NR = NW > 0 ? NW : 1;
  uint64_t row[NR];
  if constexpr (NW > 0) {
    n = NW;
#pragma unroll
    for (int i = 0; i < NW; ++i) row[i] = src[i];
  }
  auto word = [&](int i) -> uint64_t {
    if constexpr (NW > 0) return row[i];
    else return src[i];
  };
#pragma unroll
  for (int i = 0; i < n; ++i) {
    uint64_t v = word(i);
    uint64_t prev = i > 0 ? word(i - 1) : (dil ? 0ull : ~0ull);
    uint64_t next = i + 1 < n ? word(i + 1) : (dil ? 0ull : ~0ull);
    if (!dil) {
      if (i == n - 1) v |= ~lm;          // bits past the right edge count as "ignored" (=1)
      if (i + 1 == n - 1) next |= ~lm;
    }
    uint64_t acc = v;
    for (int k = 1; k <= r; ++k) {
      const uint64_t left = (v << k) | (prev >> (64 - k));   // pixel x-k
      const uint64_t right = (v >> k) | (next << (64 - k));  // pixel x+k
      acc = dil ? (acc | left | right) : (acc & left & right);
    }
    dst[i] = (i == n - 1) ? (acc & lm) : acc;
  }
}

// Vertical morphology: dst[y] = OP_{|dy|≤r, 0≤y+dy<H} src[y+dy] (row stride s words, 0 = n).
__device__ __forceinline__ void morph_rows_v(const uint64_t* src, uint64_t* dst, int h, int n, int r, bool dil,
                                             int s = 0) {
  if (s == 0) s = n;
  for (int q = threadIdx.x; q < h * n; q += blockDim.x) {
    const int y = q / n, idx = y * s + (q - y * n);
    uint64_t acc = src[idx];
    for (int k = 1; k <= r; ++k) {
      if (y - k >= 0) acc = dil ? (acc | src[idx - k * s]) : (acc & src[idx - k * s]);
      if (y + k < h) acc = dil ? (acc | src[idx + k * s]) : (acc & src[idx + k * s]);
    }
    dst[idx] = acc;
  }
}

template <int NW = 0>
__device__ inline void morph(const uint64_t* src, uint64_t* dst, uint64_t* tmp, int w, int h, int n, int size, bool dil,
                             int s = 0) {
  if (s == 0) s = n;
  const int r = size / 2;
  for (int y = threadIdx.x; y < h; y += blockDim.x) morph_row_h<NW>(src + y * s, tmp + y * s, n, w, r, dil);
  __syncthreads();
  morph_rows_v(tmp, dst, h, n, r, dil, s);
  __syncthreads();
}

// Half-width of the digital disc of radius r at row offset dy: floor(sqrt(r² − dy²)), −1 outside.
__device__ __forceinline__ int disc_halfwidth(int r2_minus) {
  if (r2_minus < 0) return -1;
  int k = 0;
  while ((k + 1) * (k + 1) <= r2_minus) ++k;
  return k;
}

// Word i of the horizontal morphology (radius k) of one row of n words: OR (dilate) or AND (erode,
// pixels outside the row count as 1) of the shifts by ±1..±k. Not masked to the row's width.
__device__ __forceinline__ uint64_t hmorph_word(const uint64_t* row, int i, int n, uint64_t lm, int k, bool dil) {
  uint64_t v = row[i];
  uint64_t prev = i > 0 ? row[i - 1] : (dil ? 0ull : ~0ull);
  uint64_t next = i + 1 < n ? row[i + 1] : (dil ? 0ull : ~0ull);
  if (!dil) {
    if (i == n - 1) v |= ~lm;
    if (i + 1 == n - 1) next |= ~lm;
  }
  uint64_t acc = v;
  for (int j = 1; j <= k; ++j) {
    const uint64_t left = (v << j) | (prev >> (64 - j));
    const uint64_t right = (v >> j) | (next << (64 - j));
    acc = dil ? (acc | left | right) : (acc & left & right);
  }
  return acc;
}

// Morphology with the digital disc of radius r = size/2 (PipelineParams::se_shape = disc): the disc
// is the union of the horizontal segments |dx| ≤ floor(sqrt(r² − dy²)) of its rows, so every output
// word is the OR / AND over the in-image rows y+dy of one horizontally dilated / eroded word. One
// pass, no scratch plane; out-of-image rows are ignored like the square's.
__device__ inline void morph_disc(const uint64_t* src, uint64_t* dst, int w, int h, int n, int size, bool dil, int s = 0) {
  if (s == 0) s = n;
  const int r = size / 2;
  const uint64_t lm = last_mask(w);
  for (int q = threadIdx.x; q < h * n; q += blockDim.x) {
    const int y = q / n, i = q - y * n;
    uint64_t acc = dil ? 0ull : ~0ull;
    for (int dy = -r; dy <= r; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= h) continue;
      const uint64_t v = hmorph_word(src + yy * s, i, n, lm, disc_halfwidth(r * r - dy * dy), dil);
      acc = dil ? (acc | v) : (acc & v);
    }
    dst[y * s + i] = i == n - 1 ? (acc & lm) : acc;
  }
  __syncthreads();
}

// The pipeline's structuring element: square (morph) or disc (morph_disc), PipeConsts::se_disc.
template <int NW = 0>
__device__ inline void morph_se(const uint64_t* src, uint64_t* dst, uint64_t* tmp, int w, int h, int n, int size, bool dil,
                                bool disc, int s = 0) {
  if (disc)
    morph_disc(src, dst, w, h, n, size, dil, s);
  else
    morph<NW>(src, dst, tmp, w, h, n, size, dil, s);
}

// Copy an LDS plane with row stride s (n words per row) to a dense global plane.
__device__ inline void store_plane(const uint64_t* src, uint64_t* dst, int h, int n, int s) {
  for (int q = threadIdx.x; q < h * n; q += blockDim.x) {
    const int y = q / n;
    dst[q] = src[y * s + (q - y * n)];
  }
}


// Grow Rg (seeded, ⊆ M) to the fixpoint of horizontal run fills, vertical run fills on the
// transposed planes and (connectivity 8) diagonal seeding. Mt must hold transpose(M); Rt is
// scratch. All planes in LDS; M/Rg rows are sn words apart, Mt/Rt rows st words apart (0 = dense;
// odd strides keep the thread-per-row sweeps and transposes free of LDS bank conflicts). `flag` is
// an LDS int. Returns the iteration count.
// NW / HB > 0: compile-time words per row of the row / transposed planes (n / ceil(H/64)).
// `flagp` points at TWO LDS ints: iteration k reports changes in flag[k & 1] and clears
// flag[(k + 1) & 1] after its first barrier (every thread read that word at the end of iteration
// k − 1 before reaching it), so the end of an iteration needs one barrier, not three.
template <int NW = 0, int HB = 0>
__device__ inline int srg_fixpoint(uint64_t* M, uint64_t* Rg, const uint64_t* Mt, uint64_t* Rt, int W, int H, int n,
                            int connectivity, int* flagp, int sn = 0, int st = 0) {
  const int hb = (H + 63) >> 6, words = H * n;
  if (sn == 0) sn = n;
  if (st == 0) st = hb;
  int iters = 0;
  const int max_iters = W * H + 4;  // monotone growth ⇒ always terminates earlier
  if (threadIdx.x == 0) flagp[0] = flagp[1] = 0;
  __syncthreads();
  for (;;) {
    int& flag = flagp[iters & 1];
    ++iters;
    bool ch = false;
    for (int y = threadIdx.x; y < H; y += blockDim.x) ch |= fill_row_any<NW>(Rg + y * sn, M + y * sn, n);
    if (ch) flag = 1;
    __syncthreads();
    if (threadIdx.x == 0) flagp[iters & 1] = 0;  // the next iteration's word
    if (connectivity == 8) {
      // Diagonal seeding from a snapshot of the horizontally dilated rows (Rt as scratch).
      for (int y = threadIdx.x; y < H; y += blockDim.x) morph_row_h<NW>(Rg + y * sn, Rt + y * sn, n, W, 1, true);
      __syncthreads();
      bool dch = false;
      for (int q = threadIdx.x; q < words; q += blockDim.x) {
        const int y = q / n, idx = y * sn + (q - y * n);
        uint64_t nb = 0;
        if (y > 0) nb |= Rt[idx - sn];
        if (y + 1 < H) nb |= Rt[idx + sn];
        const uint64_t add = M[idx] & nb & ~Rg[idx];
        if (add) {
          Rg[idx] |= add;
          dch = true;
        }
      }
      if (dch) flag = 1;
      __syncthreads();
    }
    transpose_plane(Rg, H, n, Rt, W, false, nullptr, sn, st);
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) fill_row_any<HB>(Rt + x * st, Mt + x * st, hb);
    __syncthreads();
    transpose_plane(Rt, W, hb, Rg, H, true, &flag, st, sn);
    __syncthreads();
    if (flag == 0 || iters >= max_iters) break;
  }
  return iters;
}

}  // namespace nm03::gpu
