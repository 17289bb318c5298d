// K4 — JPEG export on the GPU (replaces ImageFileExporter → Qt → libjpeg on the host,
// main_sequential.cpp:61-73). Output is byte-identical to libjpeg(-turbo) baseline q75 4:2:0
// (nm03/jpeg_common.h; golden encoder src/io/jpeg.cpp; tests/test_jpeg.py vs Pillow).
//
// Two launches per batch (a batch of 64 slices = 128 canvases = 524k luma blocks):
//  1 jpeg_fused_kernel   workgroup per 256 luma blocks (64 MCUs) of an image, thread per block.
//                        Pixels come from the canvas or — for an exact 2× fit, the common case —
//                        are rendered on the fly from the 6×6 source patch (render_core.h), so the
//                        256 KiB canvas never exists. The workgroup first stages its source rows
//                        in LDS (gray: rescaled f32, 18 × 258 for a 256² slice; labels: the label
//                        and border bit rows) with coalesced loads: 76 → 67 µs per 64-slice batch.
//                        islow FDCT (24-bit multiplies), quantisation by exact reciprocal (umulhi
//                        by ceil(2^32/d): exact for |x|, d < 2^16),
//                        Huffman cost, workgroup scan, decoupled look-back over the image's
//                        earlier workgroups, then the codes are ORed into the zeroed stage words.
//  2 jpeg_stuff_*        grid-stride over (chunk, image) 4 KiB chunks, chunk-major: count 0xFF
//                        bytes; then prefix over previous chunks, in-chunk scan, stuffed bytes
//                        staged in LDS and copied straight into host-mapped pinned memory; the
//                        consumed stage words are cleared for the next launch.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg_common.h"
#include "nm03/kernels.h"
#include "render_core.h"

namespace nm03::gpu {

using namespace nm03::jpeg;

struct QuantRecip {
  uint32_t half[64];  // d/2
  uint32_t m[64];     // ceil(2^32 / d)
};

__device__ __forceinline__ int mag_bits_fast(int v) {
  const unsigned a = (unsigned)(v < 0 ? -v : v);
  return a ? 32 - __builtin_clz(a) : 0;
}
__device__ __forceinline__ uint32_t hlen(uint32_t e) { return e >> 16; }

__device__ __forceinline__ int16_t quant_recip(int32_t x, const QuantRecip& q, int n) {
  const uint32_t a = (uint32_t)(x < 0 ? -x : x) + q.half[n];
  const int32_t v = (int32_t)__umulhi(a, q.m[n]);
  return (int16_t)(x < 0 ? -v : v);
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}


// Look-back status word: hi = state (0 = not yet, 1 = aggregate, 2 = inclusive prefix), lo = bits.
// The stuffing-count kernel (next in the stream) clears the words again for the next launch.
// Relaxed agent-scope atomics: the word itself carries the value, nothing else is published
// through it (the stage bits are consumed by later kernels), and acquire/release would add an L2
// writeback (buffer_wbl2) per store and an L2 invalidate (buffer_inv) per poll on gfx950.
__device__ __forceinline__ uint64_t look_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void look_store(uint64_t* p, uint32_t state, uint32_t v) {
  __hip_atomic_store(p, ((uint64_t)state << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b) {
  const uint32_t s = a + b;
  return s < a ? 0xFFFFFFFFu : s;
}

constexpr int kJpegWG = 256;     // luma blocks (threads) per workgroup = 64 MCUs
constexpr int kAsmWords = 2048;  // LDS assembly buffer for the workgroup's bit range (64 Kbit)

// Gray source staging: the raw rows a workgroup's 64 MCUs read (8 per MCU row + a 1-row halo each
// side, full width + 1-column halos, edge-clamped) are loaded once, coalesced, into LDS; the 6×6
// patches of the exact-2× render then come from LDS instead of 36 scattered global loads per
// block. Pixels are converted to f32 (rescale) once while staging, not once per patch use (2.25×).
constexpr int kPatchLds = 4864;  // f32 elements (19 KiB; 256²: 18 × 258 = 4644); larger footprints use global loads

constexpr int kPrivWords = 5;    // per-block Huffman bits kept in LDS (160 bits, odd stride) ...
constexpr int kSpillWords = 56;  // ... the rest in the block's global spill slot (a block needs ≤ 1700)

// MSB-first bit writer for one block: words [0, kPrivWords) go to LDS, later words (noisy,
// high-detail blocks only) to global memory. Counts every bit.
struct LBitWriter {
  uint32_t* buf;
  uint32_t* spill;
  uint32_t bits = 0;
  uint64_t acc = 0;
  int nacc = 0;
  __device__ LBitWriter(uint32_t* b, uint32_t* s) : buf(b), spill(s) {}
  __device__ __forceinline__ void store(uint32_t wi, uint32_t v) {
    if (wi < (uint32_t)kPrivWords)
      buf[wi] = v;
    else
      spill[wi - kPrivWords] = v;
  }
  // `code` must fit in `len` bits (Huffman codes do; magnitudes are masked by the caller).
  __device__ __forceinline__ void put(uint32_t code, int len) {
    acc = (acc << len) | (uint64_t)code;
    nacc += len;
    bits += (uint32_t)len;
    if (nacc >= 32) {
      store((bits - (uint32_t)nacc) >> 5, (uint32_t)(acc >> (nacc - 32)));
      nacc -= 32;
      acc &= (1ull << nacc) - 1ull;
    }
  }
  __device__ __forceinline__ void put_sym(uint32_t e) { put(e & 0xFFFFu, (int)(e >> 16)); }
  __device__ __forceinline__ void finish() {
    if (nacc > 0) store(bits >> 5, (uint32_t)(acc << (32 - nacc)));
  }
};
__device__ __forceinline__ uint32_t priv_word(const uint32_t* pb, const uint32_t* spill, uint32_t i) {
  return i < (uint32_t)kPrivWords ? pb[i] : spill[i - kPrivWords];
}

// Single-pass encoder: workgroup with ticket L encodes blocks [256p, 256p+256) of image i.
//  1. render (fused 2×) or read the 8×8 block, islow FDCT, reciprocal quantisation;
//  2. Huffman cost of the block (DC needs the previous block's DC: LDS neighbour, and for the
//     first block of the workgroup a wave-0 recomputation of the preceding block's DC = Σ(x-128));
//  3. workgroup exclusive scan of the costs, then a decoupled look-back over the image's earlier
//     workgroups in ticket order (tickets are taken when a workgroup starts, so every workgroup
//     waited on is already resident). The spin is bounded anyway (an image whose look-back
//     times out is re-encoded on the CPU);
//  4. each thread writes its block's codes at its bit offset (atomicOr into the zeroed stage).
// The last workgroup of an image publishes the total (or the overflow marker).
__global__ __launch_bounds__(kJpegWG) __attribute__((amdgpu_waves_per_eu(4))) void jpeg_fused_kernel(const uint8_t* __restrict__ canvas,
                                                             const JpegDesc* __restrict__ jd, int ncanvas, int out_w,
                                                             int out_h, QuantRecip q, JpegWork w, JpegRenderSrc rs,
                                                             int32_t* __restrict__ out_sizes, int dbg) {
  __shared__ uint32_t actab[256];
  __shared__ uint32_t dctab[16];
  __shared__ int32_t sdc[kJpegWG];
  __shared__ uint32_t spriv[kJpegWG * kPrivWords];  // per-block AC Huffman bits
  __shared__ uint32_t swg[kAsmWords + 2];           // the workgroup's bit range
  __shared__ uint32_t sh[17];
  __shared__ uint32_t s_ticket, s_prefix;
  __shared__ int32_t s_prevdc;
  __shared__ __attribute__((aligned(16))) float spatch[kPatchLds];
  const int tid = threadIdx.x;
  if (dbg == 8) {  // profiling variant: empty workgroup
    if (tid == 999) w.total[0] = 1u;
    return;
  }
  actab[tid] = kHuffAcLuma.e[tid];
  if (tid < 16) dctab[tid] = tid < 12 ? kHuffDcLuma.e[tid] : 0u;
  const int bpi = (out_w >> 3) * (out_h >> 3);
  const int parts = (bpi + kJpegWG - 1) / kJpegWG;
  // The image is fixed by the dispatch index; only the part comes from the ticket, so the
  // descriptor loads below overlap the ticket's round trip.
  const int img = (int)(blockIdx.x / (uint32_t)parts);
  const JpegDesc d = jd[img];
  RenderDesc rd;
  RWindow win{0.f, 0.f};
  if (d.render >= 0) {
    rd = rs.rd[d.render];
    if (rd.kind != kRenderLabels) win = render_window(rd, rs.stats);
  }
  if (tid == 0) {
    // Ordered tickets per image: workgroup b encodes image b / parts and takes the next part of
    // that image from the image's counter, so it only ever waits on parts whose workgroups have
    // already started — progress is guaranteed even when other kernels (other streams, other
    // processes on the same GPU) share the CUs or the queue is preempted. (Using the dispatch
    // index as the part is ~5% faster, NM03_JPEG_DBG=9, but two encoders interleaving on the same
    // XCDs can starve each other's predecessors: measured 2.3 s/step stalls with two ranks per
    // GPU.) One counter per image keeps the serialised atomics per address at `parts`.
    uint32_t p = blockIdx.x - (uint32_t)img * (uint32_t)parts;
    if (dbg != 9) {
      p = atomicAdd(&w.ticket[img], 1u);
      if (p == (uint32_t)parts - 1) atomicExch(&w.ticket[img], 0u);  // the image's last ticket
    }
    s_ticket = p;
  }
  __syncthreads();
  // The part is workgroup-uniform: keep it in an SGPR.
  const int part = (int)__builtin_amdgcn_readfirstlane(s_ticket);
  if (dbg == 7) {  // profiling variant: tables + ticket only
    if (part == 0x7FFFFFF1) w.total[0] = 1u;
    return;
  }
  const int mcux = out_w >> 4;
  const int b = part * kJpegWG + tid;
  const bool valid = b < bpi;
  // ---- 0. stage the source rows of this workgroup in LDS (workgroup-uniform decision) ----------
  int ys0 = 0, pcols = 0;
  bool staged = false, lstaged = false;
  uint64_t* const slab = reinterpret_cast<uint64_t*>(spatch);  // label images reuse the area
  if (d.render >= 0 && rd.kind == kRenderLabels && dbg != 12) {
    // Label render rows: 4by .. 4by+3 for the workgroup's block rows → 8 per MCU row.
    const int m0 = part * (kJpegWG / 4), m1 = min(m0 + kJpegWG / 4, bpi >> 2) - 1;
    const int r0 = m0 / mcux, r1 = m1 / mcux;
    const int nrows = 8 * (r1 - r0) + 8, wpr = rd.wpr, nw = nrows * wpr;
    if (2 * nw * 2 <= kPatchLds) {  // two u64 planes in the f32 area
      lstaged = true;
      ys0 = 8 * r0;
      pcols = nw;  // offset of the border plane
      for (int i = tid; i < nw; i += kJpegWG) {
        const int j = i / wpr, k = i - j * wpr;
        const size_t wi = (size_t)clampi(ys0 + j, 0, rd.src_h - 1) * wpr + k;
        slab[i] = rs.bits[rd.src_off + wi];
        slab[nw + i] = rs.bits[rd.border_off + wi];
      }
      __syncthreads();
    }
  }
  if (d.render >= 0 && rd.kind == kRenderRawGray && dbg != 12) {  // dbg 12: A/B with global loads
    const int m0 = part * (kJpegWG / 4), m1 = min(m0 + kJpegWG / 4, bpi >> 2) - 1;
    const int r0 = m0 / mcux, r1 = m1 / mcux;
    const int nrows = 8 * (r1 - r0) + 10;
    pcols = rd.src_w + 2;
    if (nrows * pcols <= kPatchLds && !(rd.src_off & 1)) {
      staged = true;
      ys0 = 8 * r0 - 1;
      const int W = rd.src_w, H = rd.src_h, hw = W >> 1;  // W is a multiple of 8 (exact 2× fit)
      const uint16_t* src = rs.raw + rd.src_off;
      // Interior: 4-byte loads of pixel pairs, all issued before the LDS stores (one latency).
      const int nw = nrows * hw;
      constexpr int kU = 12;  // ≥ 18 rows × 128 pairs / 256 threads for a 256² source: one round of loads
      uint32_t v[kU];
#pragma unroll
      for (int t = 0; t < kU; ++t) {
        const int i = tid + t * kJpegWG;
        v[t] = 0u;
        if (i < nw) {
          const int j = i / hw, k = i - j * hw;
          v[t] = *reinterpret_cast<const uint32_t*>(src + (size_t)clampi(ys0 + j, 0, H - 1) * W + 2 * k);
        }
      }
      auto value = [&](uint16_t r) {
        return rescaled_value(key_from_raw(r, rd.type, rd.stored_bits), rd.type, rd.slope, rd.intercept);
      };
#pragma unroll
      for (int t = 0; t < kU; ++t) {
        const int i = tid + t * kJpegWG;
        if (i < nw) {
          const int j = i / hw, k = i - j * hw;
          spatch[j * pcols + 2 * k + 1] = value((uint16_t)(v[t] & 0xFFFFu));
          spatch[j * pcols + 2 * k + 2] = value((uint16_t)(v[t] >> 16));
        }
      }
      for (int i = tid + kU * kJpegWG; i < nw; i += kJpegWG) {  // larger footprints
        const int j = i / hw, k = i - j * hw;
        const uint32_t u = *reinterpret_cast<const uint32_t*>(src + (size_t)clampi(ys0 + j, 0, H - 1) * W + 2 * k);
        spatch[j * pcols + 2 * k + 1] = value((uint16_t)(u & 0xFFFFu));
        spatch[j * pcols + 2 * k + 2] = value((uint16_t)(u >> 16));
      }
      // Clamped halo columns 0 and W+1.
      for (int i = tid; i < 2 * nrows; i += kJpegWG) {
        const int j = i >> 1, right = i & 1;
        spatch[j * pcols + (right ? W + 1 : 0)] =
            value(src[(size_t)clampi(ys0 + j, 0, H - 1) * W + (right ? W - 1 : 0)]);
      }
      __syncthreads();
    }
  }
  // ---- 1+2. block → DCT → quantisation fused with the AC Huffman coding ------------------------
  // The coefficients never leave registers: the zig-zag walk is unrolled, each coefficient is
  // quantised and — if non-zero in some lane of the wave (else the position is skipped) — coded
  // straight into the block's private bit buffer. The DC code depends on the previous block's DC,
  // so the AC stream is coded first and the DC code is prepended at assembly time.
  uint32_t* const pbuf = spriv + tid * kPrivWords;
  uint32_t* const pspill = w.spill + ((size_t)blockIdx.x * kJpegWG + tid) * kSpillWords;
  int dc0 = 0;
  uint32_t acbits = 0;
  if (valid) {
    const int mcu = b >> 2, sub = b & 3;
    const int bx = 2 * (mcu % mcux) + (sub & 1), by = 2 * (mcu / mcux) + (sub >> 1);
    int32_t blk[64];
    if (dbg == 6) {  // profiling variant: no render
#pragma unroll
      for (int i = 0; i < 64; ++i) blk[i] = (i * 7 + bx + by) & 255;
    } else if (lstaged) {
      const int wpr = rd.wpr;
      render_labels_2x(rd, [&](int y, int k, uint64_t& lab, uint64_t& brd) {
        const int i = (y - ys0) * wpr + k;
        lab = slab[i];
        brd = slab[pcols + i];
      }, bx, by, blk);
    } else if (staged) {
      // Patch element (j, i) = source (4by-1+j, 4bx-1+i) = LDS (4by-1+j-ys0, 4bx+i).
      const float* pp = spatch + (4 * by - 1 - ys0) * pcols + 4 * bx;
      render_patch_2x([&](int j, int i) { return pp[j * pcols + i]; }, win, blk);
    } else if (d.render >= 0) {
      render_block_2x(rd, rs.raw, rs.f32, rs.bits, win, bx, by, blk, dbg == 11);
    } else {
      const uint8_t* src = canvas + d.canvas_off + (size_t)(by * 8) * out_w + bx * 8;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const uint2 v = *reinterpret_cast<const uint2*>(src + (size_t)r * out_w);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          blk[r * 8 + c] = (int32_t)((v.x >> (8 * c)) & 0xFF);
          blk[r * 8 + 4 + c] = (int32_t)((v.y >> (8 * c)) & 0xFF);
        }
      }
    }
    if (dbg == 1 || dbg == 6) {  // profiling variants: stop before the FDCT
      int acc = 0;
#pragma unroll
      for (int i = 0; i < 64; ++i) acc += blk[i] * (i + 1);
      if (acc == 0x7FFFFFF1) w.total[0] = 1u;
      return;
    }
    // Level shift (x − 128) folded into the DC term: the islow FDCT is linear and its only
    // rounding of the DC is a shift that divides the constant exactly, so fdct(x − 128) ==
    // fdct(x) with DC − 64·128 (checked for all-extreme and random blocks). Saves 64 VALU ops.
    fdct_islow(blk);
    blk[0] -= 64 * 128;
    // Quantise into packed int16 pairs first (frees the 64 int32 DCT registers), then walk the
    // zig-zag order from those registers.
    uint32_t zp[32];
#pragma unroll
    for (int k = 0; k < 64; k += 2) {
      const int16_t a = quant_recip(blk[kNatural[k]], q, kNatural[k]);
      const int16_t c = quant_recip(blk[kNatural[k + 1]], q, kNatural[k + 1]);
      zp[k >> 1] = (uint32_t)(uint16_t)a | ((uint32_t)(uint16_t)c << 16);
    }
    dc0 = (int16_t)(zp[0] & 0xFFFFu);
    LBitWriter lw(pbuf, pspill);
    int last = 0;
    // Outer loop not unrolled: zp[j] is indexed by a wave-uniform counter (register indexing, no
    // scratch), keeping the code compact.
#pragma unroll 1
    for (int j = 0; j < 32; ++j) {
      const uint32_t word = zp[j];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = 2 * j + h;
        const int v = (int16_t)(word >> (16 * h));
        if (k > 0 && __ballot(v != 0)) {
          if (v != 0) {
            int run = k - last - 1;
            while (run > 15) {
              lw.put_sym(actab[0xF0]);
              run -= 16;
            }
            const int nb = mag_bits_fast(v);
            const uint32_t e = actab[(run << 4) + nb];  // symbol and magnitude in one put (≤ 27 bits)
            const uint32_t mag = (uint32_t)(v < 0 ? v - 1 : v) & ((1u << nb) - 1u);
            lw.put(((e & 0xFFFFu) << nb) | mag, (int)(e >> 16) + nb);
            last = k;
          }
        }
      }
    }
    if (last < 63) lw.put_sym(actab[0x00]);
    if ((b & 3) == 3) {  // the MCU's Cb and Cr blocks of a gray image: DC diff 0 + EOB each
      lw.put_sym(kHuffDcChroma.e[0]);
      lw.put_sym(kHuffAcChroma.e[0]);
      lw.put_sym(kHuffDcChroma.e[0]);
      lw.put_sym(kHuffAcChroma.e[0]);
    }
    lw.finish();
    acbits = lw.bits;
  }
  if (dbg == 2) {  // profiling variant: stop after FDCT + quantisation + AC coding
    if (dc0 == 0x7FFFFFF1 || acbits == 0x7FFFFFF1u) w.total[0] = 1u;
    return;
  }
  sdc[tid] = dc0;
  // DC of the block preceding this workgroup's first block (0 at the start of the image).
  if (tid < 64) {
    int dcp = 0;
    if (part > 0) {
      const int pb = part * kJpegWG - 1;
      const int mcu = pb >> 2, sub = pb & 3;
      const int u = 8 * (2 * (mcu % mcux) + (sub & 1)) + (tid & 7);
      const int v = 8 * (2 * (mcu / mcux) + (sub >> 1)) + (tid >> 3);
      const int px = d.render >= 0 ? (int)render_pixel(rd, rs.raw, rs.f32, rs.bits, win, u, v)
                                   : (int)canvas[d.canvas_off + (size_t)v * out_w + u];
      dcp = quant_recip(wave_sum_i32(px - 128), q, 0);
    }
    if (tid == 0) s_prevdc = dcp;
  }
  __syncthreads();
  // DC code (Huffman symbol + magnitude bits, ≤ 20 bits, right-aligned).
  const int diff = dc0 - (tid ? sdc[tid - 1] : s_prevdc);
  const int dn = mag_bits_fast(diff);
  const uint32_t dce = dctab[dn];
  const int dclen = valid ? (int)(dce >> 16) + dn : 0;
  const uint32_t dccode = ((dce & 0xFFFFu) << dn) | ((uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << dn) - 1u));
  const uint32_t bits = valid ? (uint32_t)dclen + acbits : 0u;
  // ---- 3. workgroup scan + look-back --------------------------------------------------------
  uint32_t agg = 0;
  const uint32_t excl = block_exclusive_scan(bits, sh, &agg);  // ends with a barrier
  uint64_t* look = w.look + (size_t)img * parts;
  if (tid < 64) {
    // Wave 0 looks back through a window of 64 predecessors per round trip: lane l reads the
    // status of part (hi - l); the nearest inclusive prefix ends the window and the aggregates up
    // to it are summed across the wave. (A serial walk costs one device-scope load latency per
    // predecessor — the critical path of images whose parts all run concurrently.)
    const int lane = tid;
    uint32_t prefix = 0;
    if (part == 0 || dbg == 4) {  // dbg 4: profiling variant without the look-back wait
      if (lane == 0) look_store(&look[part], 2u, agg);
    } else {
      if (lane == 0) look_store(&look[part], 1u, agg);
      int hi = part - 1;
      uint32_t spins = 0;
      for (;;) {
        const int p = hi - lane;
        const uint64_t st = p >= 0 ? look_load(&look[p]) : (2ull << 32);  // before part 0: inclusive 0
        const uint32_t state = (uint32_t)(st >> 32);
        const uint64_t incl = __ballot(state == 2u);
        const int stop = incl ? __builtin_ctzll(incl) : 64;  // nearest inclusive prefix
        const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1ull);
        if (__ballot(state == 0u) & need) {  // a needed predecessor has not published yet
          if (++spins > (1u << 26)) {  // cannot happen with ordered tickets; never hang the GPU
            prefix = 0xFFFFFFFFu;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        uint32_t lo32 = lane <= stop ? (uint32_t)st : 0u, hi32 = 0u;  // 64-bit wave sum
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const uint32_t l2 = __shfl_xor(lo32, o, 64), h2 = __shfl_xor(hi32, o, 64);
          const uint32_t s = lo32 + l2;
          hi32 += h2 + (s < lo32 ? 1u : 0u);
          lo32 = s;
        }
        prefix = sat_add(prefix, hi32 ? 0xFFFFFFFFu : lo32);
        if (stop < 64) break;
        hi -= 64;
      }
      if (lane == 0) look_store(&look[part], 2u, sat_add(prefix, agg));
    }
    if (lane == 0) s_prefix = prefix;
  }
  // Meanwhile: assemble the workgroup's contiguous bit range in LDS: each block's DC code, then
  // its AC words shifted behind it.
  const uint32_t nlocal = (agg + 31) >> 5;
  const bool in_lds = nlocal < (uint32_t)kAsmWords;  // workgroup-uniform
  const uint32_t nwp = (acbits + 31) >> 5;
  const uint32_t acpos = excl + (uint32_t)dclen;
  if (in_lds) {
    for (uint32_t i = tid; i <= nlocal; i += kJpegWG) swg[i] = 0u;
    __syncthreads();
    if (valid) {
      const uint32_t dv = dclen ? dccode << (32 - dclen) : 0u, sh0 = excl & 31u, w0 = excl >> 5;
      atomicOr(&swg[w0], dv >> sh0);
      if (sh0) atomicOr(&swg[w0 + 1], dv << (32u - sh0));
      const uint32_t shf = acpos & 31u, wa = acpos >> 5;
      for (uint32_t i = 0; i < nwp; ++i) {
        const uint32_t v = priv_word(pbuf, pspill, i);
        atomicOr(&swg[wa + i], v >> shf);
        if (shf) atomicOr(&swg[wa + i + 1], v << (32u - shf));
      }
    }
  }
  __syncthreads();
  const uint32_t prefix = s_prefix;
  const uint32_t end = sat_add(prefix, agg);
  const uint32_t cap_bits = d.stage_words * 32u;
  uint32_t* stage = w.stage + d.stage_off;
  // ---- 4. emission: coalesced word stores (only the two edge words, shared with the
  //         neighbouring workgroups, are atomic) --------------------------------------------------
  if (end <= cap_bits && agg) {
    if (in_lds) {
      const uint32_t sft = prefix & 31u, base = prefix >> 5;
      const uint32_t nw = ((prefix + agg + 31u) >> 5) - base;
      for (uint32_t j = tid; j < nw; j += kJpegWG) {
        uint32_t v = j < nlocal ? swg[j] >> sft : 0u;
        if (sft && j > 0) v |= swg[j - 1] << (32u - sft);
        if (j == 0 || j == nw - 1)
          atomicOr(&stage[base + j], v);
        else
          stage[base + j] = v;
      }
    } else if (valid) {
      // Very detailed workgroup (> 64 Kbit): each block ORs its bits straight into the stage.
      const uint32_t p0 = prefix + excl;
      const uint32_t dv = dclen ? dccode << (32 - dclen) : 0u;
      atomicOr(&stage[p0 >> 5], dv >> (p0 & 31u));
      if (p0 & 31u) atomicOr(&stage[(p0 >> 5) + 1], dv << (32u - (p0 & 31u)));
      const uint32_t pa = prefix + acpos;
      for (uint32_t i = 0; i < nwp; ++i) {
        const uint32_t v = priv_word(pbuf, pspill, i), dst = pa + 32u * i, wi = dst >> 5, shf = dst & 31u;
        atomicOr(&stage[wi], v >> shf);
        if (shf) atomicOr(&stage[wi + 1], v << (32u - shf));
      }
    }
  }
  if (part == parts - 1 && tid == 0) {
    const uint32_t nbytes = (end + 7) >> 3;
    const bool overflow = end == 0xFFFFFFFFu || end > cap_bits || 2u * nbytes + 16u > d.out_cap ||
                          (nbytes + kStuffChunk - 1) / kStuffChunk > (uint32_t)w.max_chunks;
    w.total[img] = overflow ? 0xFFFFFFFFu : end;
    if (overflow) out_sizes[img] = -1;
  }
}

// Byte i of the entropy-coded segment (MSB-first words), final byte padded with 1-bits.
__device__ __forceinline__ uint32_t seg_byte(const uint32_t* stage, uint32_t i, uint32_t nbytes, uint32_t padbits) {
  uint32_t v = (stage[i >> 2] >> (24 - 8 * (i & 3))) & 0xFFu;
  if (padbits && i == nbytes - 1) v |= 0xFFu >> padbits;
  return v;
}

constexpr int kStuffThreads = 256;
constexpr int kBytesPerThread = kStuffChunk / kStuffThreads;  // 16
constexpr int kStuffGrid = 512;                               // persistent-style: 2 workgroups per CU

// Bytes of the largest image of the launch (an overflowed image forces the full sweep: its
// partially written stage must be cleared). Every workgroup reduces the ≤ few hundred totals.
__device__ __forceinline__ uint32_t launch_max_bytes(const JpegWork& w, int ncanvas, uint32_t* sh) {
  uint32_t m = 0;
  for (int i = threadIdx.x; i < ncanvas; i += blockDim.x) {
    const uint32_t t = w.total[i];
    m = max(m, t == 0xFFFFFFFFu ? 0x7FFFFFFFu : (t + 7) >> 3);
  }
  m = wave_max_u32(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  uint32_t r = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = max(r, sh[i]);
  __syncthreads();
  return r;
}

// Work items are (chunk, image) in chunk-major order, so the valid chunks of every image come first
// and the grid-stride loop stops at the largest image instead of sweeping max_chunks × images.
__global__ __launch_bounds__(kStuffThreads) void jpeg_stuff_count_kernel(const JpegDesc* __restrict__ jd, int ncanvas,
                                                                         JpegWork w) {
  __shared__ uint32_t cnt;
  __shared__ uint32_t shm[16];
  // The encoder's look-back words are done with: clear them for the next launch.
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < w.look_used; i += (size_t)gridDim.x * blockDim.x)
    w.look[i] = 0ull;
  const uint32_t maxb = launch_max_bytes(w, ncanvas, shm);
  const int n = ncanvas * w.max_chunks;
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const int chunk = it / ncanvas, img = it - chunk * ncanvas;
    const uint32_t c0 = (uint32_t)chunk * kStuffChunk;
    if (c0 >= maxb) break;
    const uint32_t total = w.total[img];
    if (total == 0xFFFFFFFFu) continue;
    const uint32_t nbytes = (total + 7) >> 3;
    if (c0 >= nbytes) continue;
    const uint32_t* stage = w.stage + jd[img].stage_off;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    uint32_t ff = 0;
    const uint32_t b0 = c0 + threadIdx.x * kBytesPerThread;
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
      const uint32_t i = b0 + k;
      if (i < nbytes) ff += seg_byte(stage, i, nbytes, total & 7u) == 0xFFu;
    }
    if (ff) atomicAdd(&cnt, ff);
    __syncthreads();
    if (threadIdx.x == 0) w.chunk_ff[(size_t)img * w.max_chunks + chunk] = cnt;
  }
}

// Writes the stuffed chunk into host-mapped memory and clears the stage words it consumed, so the
// stage is all-zero again for the next launch (the encoder ORs bits into it).
__global__ __launch_bounds__(kStuffThreads) void jpeg_stuff_write_kernel(const JpegDesc* __restrict__ jd, int ncanvas,
                                                                         JpegWork w, uint8_t* __restrict__ out,
                                                                         int32_t* __restrict__ out_sizes) {
  __shared__ uint32_t sh[17];
  __shared__ uint8_t buf[2 * kStuffChunk];
  const uint32_t maxb = launch_max_bytes(w, ncanvas, sh);
  const int n = ncanvas * w.max_chunks;
  for (int it = blockIdx.x; it < n; it += gridDim.x) {
    const int chunk = it / ncanvas, img = it - chunk * ncanvas;
    const uint32_t c0 = (uint32_t)chunk * kStuffChunk;
    if (c0 >= maxb) break;
    const JpegDesc d = jd[img];
    uint32_t* stage = w.stage + d.stage_off;
    const uint32_t total = w.total[img];
    if (total == 0xFFFFFFFFu) {  // overflowed image (rare): clear whatever the encoder wrote
      for (uint32_t i = c0 / 4 + threadIdx.x; i < (c0 + kStuffChunk) / 4 && i < d.stage_words; i += blockDim.x)
        stage[i] = 0u;
      continue;
    }
    const uint32_t nbytes = (total + 7) >> 3;
    if (c0 >= nbytes) continue;
    const uint32_t* ffc = w.chunk_ff + (size_t)img * w.max_chunks;
    // Output offset of this chunk = bytes before it + 0xFF stuffing inserted before it.
    uint32_t before = 0;
    for (int c = 0; c < chunk; ++c) before += ffc[c];
    const uint32_t obase = c0 + before;
    const uint32_t b0 = c0 + threadIdx.x * kBytesPerThread;
    uint32_t v[kBytesPerThread];
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
      const uint32_t i = b0 + k;
      v[k] = i < nbytes ? seg_byte(stage, i, nbytes, total & 7u) : 0x100u;  // 0x100 = past the end
      mine += v[k] < 0x100u ? (v[k] == 0xFFu ? 2u : 1u) : 0u;
    }
    uint32_t chunk_len = 0;
    uint32_t o = block_exclusive_scan(mine, sh, &chunk_len);  // ends with a barrier: stage reads done
#pragma unroll
    for (int k = 0; k < kBytesPerThread; ++k) {
      if (v[k] >= 0x100u) continue;
      buf[o++] = (uint8_t)v[k];
      if (v[k] == 0xFFu) buf[o++] = 0;
    }
    const uint32_t w0 = c0 / 4, w1 = min((nbytes + 3) / 4, (c0 + kStuffChunk) / 4);
    for (uint32_t i = w0 + threadIdx.x; i < w1; i += blockDim.x) stage[i] = 0u;
    __syncthreads();
    uint8_t* dst = out + d.out_off + obase;
    for (uint32_t i = threadIdx.x; i < chunk_len; i += blockDim.x) dst[i] = buf[i];
    if (c0 + kStuffChunk >= nbytes && threadIdx.x == 0) out_sizes[img] = (int32_t)(obase + chunk_len);
    __syncthreads();  // buf is reused by the next iteration
  }
}

bool render_is_exact_2x(const RenderDesc& r, int out_w, int out_h) {
  return r.invx == 0.5f && r.invy == 0.5f && r.ox == 0.0f && r.oy == 0.0f && 2 * r.src_w == out_w &&
         2 * r.src_h == out_h && (r.src_w % 4) == 0;
}

void launch_jpeg(const uint8_t* canvas, const JpegDesc* jd, int ncanvas, int out_w, int out_h, const int32_t* div_luma,
                 JpegWork& w, uint8_t* out, int32_t* out_sizes, hipStream_t stream, const JpegRenderSrc* fused) {
  if (ncanvas <= 0) return;
  if (out_w % 16 || out_h % 16) throw DeviceError("GPU JPEG encoder needs canvas dims that are multiples of 16");
  if (w.max_chunks <= 0 || !w.total || !w.chunk_ff || !w.stage || !w.look || !w.ticket || !w.spill)
    throw DeviceError("launch_jpeg: JpegWork incomplete");
  QuantRecip q;
  for (int i = 0; i < 64; ++i) {
    const uint32_t dv = (uint32_t)div_luma[i];
    q.half[i] = dv >> 1;
    q.m[i] = (uint32_t)(((1ull << 32) + dv - 1) / dv);
  }
  JpegRenderSrc rs;
  if (fused) rs = *fused;
  const int bpi = (out_w / 8) * (out_h / 8);
  const int parts = (bpi + kJpegWG - 1) / kJpegWG;
  if ((size_t)parts * ncanvas > w.look_cap) throw DeviceError("launch_jpeg: look-back capacity exceeded");
  w.look_used = (size_t)parts * ncanvas;
  // NM03_JPEG_DBG selects truncated profiling variants (output invalid; tools/gpu_jpeg_split.sh).
  static const int dbg = [] {
    const char* e = std::getenv("NM03_JPEG_DBG");
    return e ? std::atoi(e) : 0;
  }();
  // NM03_JPEG_LDS_PAD: extra dynamic LDS per workgroup (caps the encoder's residency per CU so
  // other streams' kernels keep LDS to run alongside it).
  static const int pad = [] {
    const char* e = std::getenv("NM03_JPEG_LDS_PAD");
    return e ? std::atoi(e) : 0;
  }();
  jpeg_fused_kernel<<<parts * ncanvas, kJpegWG, pad, stream>>>(canvas, jd, ncanvas, out_w, out_h, q, w, rs,
                                                                out_sizes, dbg);
  check_launch("jpeg_fused_kernel");
  jpeg_stuff_count_kernel<<<kStuffGrid, kStuffThreads, 0, stream>>>(jd, ncanvas, w);
  check_launch("jpeg_stuff_count_kernel");
  jpeg_stuff_write_kernel<<<kStuffGrid, kStuffThreads, 0, stream>>>(jd, ncanvas, w, out, out_sizes);
  check_launch("jpeg_stuff_write_kernel");
}

}  // namespace nm03::gpu
