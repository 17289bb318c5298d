// K4 — JPEG export on the GPU (replaces ImageFileExporter → Qt → libjpeg on the host,
// main_sequential.cpp:61-73). Output is byte-identical to libjpeg(-turbo) baseline q75 4:2:0
// (nm03/jpeg_common.h; golden encoder src/io/jpeg.cpp; tests/test_jpeg.py vs Pillow).
//
// One launch per batch (a batch of 64 slices = 128 canvases = 524k luma blocks), after a clear of
// the look-back records:
//    jpeg_fused_kernel   workgroup per 256 luma blocks (64 MCUs) of an image, thread per block.
//                        Pixels come from the canvas or — for an exact 2× fit, the common case —
//                        are rendered on the fly from the 6×6 source patch (render_core.h), so the
//                        256 KiB canvas never exists. The workgroup first stages its source rows
//                        in LDS (gray: rescaled f32, 18 × 258 for a 256² slice; labels: the label
//                        and border bit rows) with coalesced loads: 76 → 67 µs per 64-slice batch.
//                        islow FDCT as v_dot2_i32_i16 dot products (label waves of one flat colour
//                        skip FDCT, quantisation and coding), quantisation by exact reciprocal (umulhi
//                        by ceil(2^32/d): exact for |x|, d < 2^16),
//                        Huffman cost, workgroup scan, the workgroup's bit range assembled in LDS,
//                        its 0xFF-byte counts for all 8 byte alignments, a decoupled look-back
//                        over the image's earlier workgroups that resolves both the bit offset and
//                        the number of stuffing bytes before it, and the 0xFF-stuffed bytes it
//                        owns written straight into host-mapped pinned memory. (Earlier versions
//                        ORed the codes into an HBM stage and ran two more launches to count and
//                        insert the stuffing: 2.65 MB written + read back per batch, two launches.)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

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

// i / d for 0 ≤ i < 2^16 and 1 ≤ d < 2^16 as one multiply-high by m = ceil(2^32 / d): with
// e = m·d − 2^32 < d, i·m / 2^32 = i/d + i·e / (d·2^32), and the error term stays below
// 2^-16 ≤ 1/d, so it never carries i/d past the next integer. The divisors here (staged row
// widths, MCUs per row) are workgroup-uniform: m is computed once instead of the compiler's
// ≈10-instruction float-reciprocal division per use (24 per thread in the gray staging alone).
struct Div16 {
  uint32_t d, m;
  __device__ __forceinline__ explicit Div16(uint32_t dv) : d(dv), m(dv > 1u ? 0xFFFFFFFFu / dv + 1u : 0u) {}
  __device__ __forceinline__ uint32_t q(uint32_t i) const { return d > 1u ? __umulhi(i, m) : i; }
};

// |quantised x| (the same quotient as quant_recip, without the sign).
__device__ __forceinline__ uint32_t quant_mag(int32_t x, const QuantRecip& q, int n) {
  const uint32_t a = (uint32_t)(x < 0 ? -x : x) + q.half[n];
  return __umulhi(a, q.m[n]);
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}


// Look-back records: 3 words per workgroup, each tagged in its top 2 bits (0 = not yet, 1 =
// aggregate, 2 = inclusive; word 0 is rewritten with the inclusive record). Cleared (memset)
// before every launch.
// Relaxed agent-scope atomics: the word itself carries the value, nothing else is published
// through it (the stage bits are consumed by later kernels), and acquire/release would add an L2
// writeback (buffer_wbl2) per store and an L2 invalidate (buffer_inv) per poll on gfx950.
__device__ __forceinline__ uint64_t look_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void look_store64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// `n` ≤ 8 bits at bit offset `o` of an MSB-first word buffer (right-aligned). Reads word o/32 + 1:
// the buffer is zeroed one word past its end.
__device__ __forceinline__ uint32_t lds_bits(const uint32_t* buf, uint32_t o, uint32_t n) {
  if (n == 0) return 0u;
  const uint32_t w = o >> 5, sh = o & 31u;
  uint32_t v = buf[w] << sh;
  if (sh) v |= buf[w + 1] >> (32u - sh);
  return v >> (32u - n);
}
__device__ __forceinline__ uint32_t lds_byte(const uint32_t* buf, uint32_t o) { return lds_bits(buf, o, 8); }

constexpr int kJpegWG = 256;     // luma blocks (threads) per workgroup = 64 MCUs

// Gray source staging: the raw rows a workgroup's 64 MCUs read (8 per MCU row + a 1-row halo each
// side, full width + 1-column halos, edge-clamped) are loaded once, coalesced, into LDS; the 6×6
// patches of the exact-2× render then come from LDS instead of 36 scattered global loads per
// block. Pixels are converted to f32 (rescale) once while staging, not once per patch use (2.25×).
// Staged gray rows are swizzled: source column c (0..W+1 with the halos) sits at c + c/4 of a row of
// stride ≡ 4 (mod 8) words. A half-wave's patch reads then hit distinct banks: its 16 blocks step
// 5 words apart (16 distinct banks mod 32) and its two block rows, 4 source rows apart, are offset
// by 16 banks (disjoint sets) — the plain layout's 4-byte stride put 4 addresses on each bank.
constexpr int kPatchLds = 5832;  // f32 elements (22.8 KiB; 256²: 18 × 324); larger footprints use global loads
__device__ __forceinline__ int swz_col(int c) { return c + (c >> 2); }
// One LDS region serves the render (source patch above) and then, once every block is rendered,
// the workgroup's assembled bit range followed by its staged stuffed output bytes.
constexpr int kUnionWords = kPatchLds + 1080;  // 27 KiB as before (4 workgroups per CU): bit ranges up to ~220 Kbit

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
// kOcc: target waves per SIMD (= workgroups per CU); kUnion: LDS words of the patch / bit-range
// union; kSamp: jpeg::Sampling — 4:2:0 scans MCUs of 2×2 luma blocks followed by the MCU's two
// all-zero chroma blocks; 4:4:4 scans the luma blocks in raster order, each followed by its two
// chroma blocks; gray scans them in raster order alone. (One instance per layout: the default
// 4:2:0 code is unchanged by the other two.) 5 workgroups per CU (31.7 KiB, ≤ 96 VGPRs with spills) measured no better than 4 once
// images were dealt round-robin (profiles/r3/jpeg_spread/split_and_occ5.txt).
template <int kOcc, int kUnion, int kSamp, bool kNearest>
__global__ __launch_bounds__(kJpegWG) __attribute__((amdgpu_waves_per_eu(kOcc))) void jpeg_fused_kernel(const uint8_t* __restrict__ canvas,
                                                             const JpegDesc* __restrict__ jd, int ncanvas, int out_w,
                                                             int out_h, QuantRecip q, JpegWork w, JpegRenderSrc rs,
                                                             uint8_t* __restrict__ out, int32_t* __restrict__ out_sizes,
                                                             int dbg) {
  // dbg: profiling variant (NM03_PROFILE_VARIANT=jpeg=N; output invalid), 0 = the real encoder.
  // kWG blocks (threads) per workgroup = kWG / 4 MCUs. (512-block workgroups, 8 waves and 2 per
  // CU, halve the per-workgroup fixed costs but measured no faster: 116.8–117.6 vs 119.2 µs per
  // 96-slice batch in the bench, profiles/r4/jpeg_wg512/.)
  constexpr int kWG = kJpegWG;
  constexpr int kPatch = kPatchLds;
  constexpr bool k420 = kSamp == kSampling420;
  // Scan units (MCUs) per workgroup and the canvas rows (source rows of the 2× render: half) of one
  // row of units.
  constexpr int kUnitBlocks = k420 ? 4 : 1, kUnitRows = k420 ? 16 : 8;
  static_assert(kPatch <= kUnion, "staging area exceeds the LDS union");
  __shared__ uint32_t actab[256];
  __shared__ uint32_t dctab[16];
  __shared__ int32_t sdc[kWG];
  __shared__ uint32_t spriv[kWG * kPrivWords];  // per-block AC Huffman bits
  __shared__ uint32_t sh[17];
  __shared__ uint32_t sff[(kWG / 64) * 8];
  __shared__ uint32_t s_ticket, s_obase, s_nown, s_strad_v, s_fin_v, s_f, s_nwords;
  __shared__ bool s_bad, s_strad, s_fin;
  __shared__ int32_t s_prevdc;
  __shared__ __attribute__((aligned(16))) float spatch[kUnion];  // render patch, then swg + output
  uint32_t* const swg = reinterpret_cast<uint32_t*>(spatch);             // the workgroup's bit range
  const int tid = threadIdx.x;
  // Records of the previous launch (the other half of the look area) are dead: clear them here
  // for the next launch instead of a separate memset launch.
  if (w.clear_words) {
    uint64_t* other = w.look + w.clear_base;
    for (size_t i = (size_t)blockIdx.x * kWG + tid; i < w.clear_words; i += (size_t)gridDim.x * kWG) other[i] = 0ull;
  }
  if (dbg == 8) {  // profiling variant: empty workgroup
    if (tid == 999) out_sizes[0] = 1;
    return;
  }
  const int bpi = (out_w >> 3) * (out_h >> 3);
  const int parts = (bpi + kWG - 1) / kWG;
  // The image is fixed by the dispatch index; only the part comes from the ticket. The ticket's
  // device-scope atomic is issued first, so its round trip overlaps the table and descriptor
  // loads below (issued after them it waited behind three dependent descriptor loads).
  // Images are dealt round-robin over the dispatch order (workgroup b encodes image b mod
  // ncanvas): consecutive workgroups hit different ticket counters instead of `parts` of them
  // queueing on one address, and an image's parts start one `ncanvas` stride apart, so a part's
  // predecessors have mostly finished encoding when it looks back (blocked order: 137.8–138.5 vs
  // 118.9–119.0 µs per 96-slice batch, profiles/r3/jpeg_spread/).
  const int img = (int)(blockIdx.x % (uint32_t)ncanvas);
  uint32_t ticket = 0;
  if (tid == 0) {
    // The address goes through a VGPR the compiler cannot prove uniform: a uniform-address atomic
    // is rewritten into a wave-aggregated one whose result is waited for on the spot.
    // (Kept in the global address space: a flat atomic would also count in lgkmcnt and hold up
    // the LDS waits behind it.)
    auto* tp = (__attribute__((address_space(1))) uint32_t*)&w.ticket[img];
    asm volatile("" : "+v"(tp));
    ticket = __hip_atomic_fetch_add(tp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  actab[tid] = kHuffAcLuma.e[tid];
  if (tid < 16) dctab[tid] = tid < 12 ? kHuffDcLuma.e[tid] : 0u;
  // JpegDesc::render is -1 or img itself, so the render descriptor loads alongside the JPEG one
  // (no dependent round trip); the render window (stats of the slice) is computed where the render
  // first needs it, so its load overlaps the staging below.
  const JpegDesc d = jd[img];
  RenderDesc rd;
  if (rs.rd) rd = rs.rd[img];
  RWindow win{0.f, 0.f};
  if (tid == 0) {
    // Ordered tickets per image: workgroup b encodes image b / parts and takes the next part of
    // that image from the image's counter, so it only ever waits on parts whose workgroups have
    // already started — progress is guaranteed even when other kernels (other streams, other
    // processes on the same GPU) share the CUs or the queue is preempted. (Using the dispatch
    // index as the part is ~5% faster, but two encoders interleaving on the same XCDs can starve
    // each other's predecessors: measured 2.3 s/step stalls with two ranks per GPU.) One counter per
    // image keeps the serialised atomics per address at `parts`.
    if (ticket == (uint32_t)parts - 1) atomicExch(&w.ticket[img], 0u);  // the image's last ticket
    s_ticket = ticket;
  }
  __syncthreads();
  // The part is workgroup-uniform: keep it in an SGPR.
  const int part = (int)__builtin_amdgcn_readfirstlane(s_ticket);
  if (dbg == 7) {  // profiling variant: tables + ticket only
    if (part == 0x7FFFFFF1) out_sizes[0] = 1;
    return;
  }
  // Profiling variants 40 / 41: only the gray (original) / only the label (processed) images are
  // encoded; the other kind's workgroups leave after taking their ticket (their images' output is
  // invalid). Splits the encoder's time by image kind.
  if ((dbg == 40 && d.render >= 0 && rd.kind == kRenderLabels) || (dbg == 41 && !(d.render >= 0 && rd.kind == kRenderLabels))) {
    if (part == 0x7FFFFFF1) out_sizes[0] = 1;
    return;
  }
  // Units (MCUs) per row: 16×16 (4:2:0) or 8×8 (4:4:4, gray) canvas pixels each.
  const int mcux = k420 ? out_w >> 4 : out_w >> 3;
  const Div16 dmx((uint32_t)mcux);
  // Scan block b → luma block column/row of the canvas.
  auto block_xy = [&](int bb, int& bx, int& by) {
    if (k420) {
      const int mcu = bb >> 2, sub = bb & 3;
      const int my = (int)dmx.q((uint32_t)mcu), mx = mcu - my * mcux;
      bx = 2 * mx + (sub & 1);
      by = 2 * my + (sub >> 1);
    } else {
      by = (int)dmx.q((uint32_t)bb);
      bx = bb - by * mcux;
    }
  };
  const int b = part * kWG + tid;
  const bool valid = b < bpi;
  // ---- 0. stage the source rows of this workgroup in LDS (workgroup-uniform decision) ----------
  int ys0 = 0, pcols = 0;
  bool staged = false, lstaged = false;
  // (A flat-label-workgroup shortcut — a workgroup whose label rows were all background or all
  // region filled its bit range with the repeating MCU pattern instead of coding — was removed in
  // round 5: its extra live state gave the kernel a 36-byte private segment, and the kernel without
  // it measured 105.2–105.8 vs 106.8–107.2 µs per 96-slice batch, profiles/r5/jpeg_flat/.)
  uint64_t* const slab = reinterpret_cast<uint64_t*>(spatch);  // label images reuse the area
  if (d.render >= 0 && rd.kind == kRenderLabels) {
    // Label render rows: 4by .. 4by+3 for the workgroup's block rows → 8 per MCU row (4:2:0).
    const int m0 = part * (kWG / kUnitBlocks), m1 = min(m0 + kWG / kUnitBlocks, bpi / kUnitBlocks) - 1;
    const int r0 = m0 / mcux, r1 = m1 / mcux;
    const int nrows = (kUnitRows / 2) * (r1 - r0 + 1), wpr = rd.wpr, nw = nrows * wpr;
    if (2 * nw * 2 <= kPatch) {  // two u64 planes in the f32 area
      lstaged = true;
      ys0 = (kUnitRows / 2) * r0;
      pcols = nw;  // offset of the border plane
      const Div16 dw((uint32_t)wpr);
      for (int i = tid; i < nw; i += kWG) {
        const int j = (int)dw.q((uint32_t)i), k = i - j * wpr;
        const size_t wi = (size_t)clampi(ys0 + j, 0, rd.src_h - 1) * wpr + k;
        slab[i] = rs.bits[rd.src_off + wi];
        slab[nw + i] = rs.bits[rd.border_off + wi];
      }
      __syncthreads();
    }
  }
  if (d.render >= 0 && rd.kind == kRenderRawGray) {
    const int m0 = part * (kWG / kUnitBlocks), m1 = min(m0 + kWG / kUnitBlocks, bpi / kUnitBlocks) - 1;
    const int r0 = m0 / mcux, r1 = m1 / mcux;
    const int nrows = (kUnitRows / 2) * (r1 - r0 + 1) + 2;
    pcols = swz_col(rd.src_w + 1) + 1;
    pcols += (4 - pcols % 8 + 8) % 8;  // row stride ≡ 4 (mod 8)
    if (nrows * pcols <= kPatch && !(rd.src_off & 1)) {
      staged = true;
      ys0 = (kUnitRows / 2) * r0 - 1;
      const int W = rd.src_w, H = rd.src_h, hw = W >> 1;  // W is a multiple of 8 (exact 2× fit)
      const uint16_t* src = rs.raw + rd.src_off;
      // Interior: 4-byte loads of pixel pairs, all issued before the LDS stores (one latency).
      const int nw = nrows * hw;
      const Div16 dh((uint32_t)hw);
      constexpr int kU = 12;  // ≥ 18 rows × 128 pairs / 256 threads for a 256² source: one round
      uint32_t v[kU];
#pragma unroll
      for (int t = 0; t < kU; ++t) {
        const int i = tid + t * kWG;
        v[t] = 0u;
        if (i < nw) {
          const int j = (int)dh.q((uint32_t)i), k = i - j * hw;
          v[t] = *reinterpret_cast<const uint32_t*>(src + (size_t)clampi(ys0 + j, 0, H - 1) * W + 2 * k);
        }
      }
      // rescaled_value(key_from_raw(r)) per staged pixel (pixel_math.h), without the key round
      // trip: the value is the low stored_bits bits of the sample, sign-extended for signed data —
      // one shift up and one arithmetic or logical shift down, selected as integers, then one
      // int → f32 conversion; the rescale only when the image has one (workgroup-uniform).
      // (Written with __builtin_amdgcn_sbfe / _ubfe and the select between the two conversions,
      // the compiler folded both into one unsigned conversion and signed slices rendered wrong:
      // profiles/r4/bfe_probe/, test_engine_norm_tables_vs_golden.)
      const bool sgn = rd.type == kI16, affine = rd.slope != 1.0f || rd.intercept != 0.0f;
      const uint32_t vsh = 32u - rd.stored_bits;
      auto value = [&](uint32_t r) {
        const uint32_t up = r << vsh;
        const int32_t xi = sgn ? (int32_t)up >> vsh : (int32_t)(up >> vsh);
        float x = (float)xi;
        if (affine) {
          const float t = x * rd.slope;
          x = t + rd.intercept;
        }
        return x;
      };
#pragma unroll
      for (int t = 0; t < kU; ++t) {
        const int i = tid + t * kWG;
        if (i < nw) {
          const int j = (int)dh.q((uint32_t)i), k = i - j * hw;
          spatch[j * pcols + swz_col(2 * k + 1)] = value(v[t] & 0xFFFFu);
          spatch[j * pcols + swz_col(2 * k + 2)] = value(v[t] >> 16);
        }
      }
      for (int i = tid + kU * kWG; i < nw; i += kWG) {  // larger footprints
        const int j = (int)dh.q((uint32_t)i), k = i - j * hw;
        const uint32_t u = *reinterpret_cast<const uint32_t*>(src + (size_t)clampi(ys0 + j, 0, H - 1) * W + 2 * k);
        spatch[j * pcols + swz_col(2 * k + 1)] = value(u & 0xFFFFu);
        spatch[j * pcols + swz_col(2 * k + 2)] = value(u >> 16);
      }
      // Clamped halo columns 0 and W+1.
      for (int i = tid; i < 2 * nrows; i += kWG) {
        const int j = i >> 1, right = i & 1;
        spatch[j * pcols + (right ? swz_col(W + 1) : 0)] =
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
  if (d.render >= 0 && rd.kind != kRenderLabels) win = render_window(rd, rs.stats);
  uint32_t* const pbuf = spriv + tid * kPrivWords;
  uint32_t* const pspill = w.spill + ((size_t)blockIdx.x * kWG + tid) * kSpillWords;
  int dc0 = 0;
  uint32_t acbits = 0;
  if (valid) {
    int bx, by;
    block_xy(b, bx, by);
    int32_t blk[64];
    // Label images are mostly background: when every block of the wave is one flat colour (76% of
    // the phantom cohort's label waves, 97.5% of its blocks) the islow FDCT of a constant block is
    // exactly DC = 64·x with every AC coefficient 0 (all butterfly differences vanish), so the
    // wave skips the FDCT, the quantisation and the zig-zag walk (wave-uniform branch).
    bool flat = false;
    if (dbg == 6) {  // profiling variant: no render
#pragma unroll
      for (int i = 0; i < 64; ++i) blk[i] = (i * 7 + bx + by) & 255;
    } else if (lstaged) {  // d.render ≥ 0: the fit is exactly 2× (render_is_exact_2x)
      const int wpr = rd.wpr;
      render_labels_exact2x(rd, [&](int y, int k, uint64_t& lab, uint64_t& brd) {
        const int i = (y - ys0) * wpr + k;
        lab = slab[i];
        brd = slab[pcols + i];
      }, bx, by, blk);
      bool same = true;
#pragma unroll
      for (int i = 1; i < 64; ++i) same = same && blk[i] == blk[0];  // 15 distinct cells after CSE
      flat = __ballot(!same) == 0;
    } else if (staged) {
      // Patch element (j, i) = source (4by-1+j, 4bx-1+i) = staged row 4by-1+j-ys0, column 4bx+i.
      // Patch column i = source column 4bx-1+i = staged column 4bx+i → swizzled 5bx + i + (i ≥ 4).
      const float* pp = spatch + (4 * by - 1 - ys0) * pcols + 5 * bx;
      auto fetch = [&](int j, int i) { return pp[j * pcols + i + (i >= 4 ? 1 : 0)]; };
      if (kNearest)  // --render-filter nearest: its own instance (launch_jpeg)
        render_patch_2x_nearest(fetch, win, blk);
      else
        render_patch_2x(fetch, win, blk);
    } else if (d.render >= 0) {
      render_block_2x<kNearest>(rd, rs.raw, rs.f32, rs.bits, win, bx, by, blk);
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
      if (acc == 0x7FFFFFF1) out_sizes[0] = 1;
      return;
    }
    LBitWriter lw(pbuf, pspill);
    int last = 0;
    if (flat) {
      dc0 = quant_recip(64 * (blk[0] - 128), q, 0);  // == fdct_islow's DC − 64·128 for a flat block
      if (dbg == 16) {  // profiling variant (below): every wave must stop here, or the look-back of
        // the flat waves would wait for records the stopped waves never publish
        if (dc0 == 0x7FFFFFF1) out_sizes[0] = 1;
        return;
      }
    } else {
      // Level shift (x − 128) folded into the DC term: the islow FDCT is linear and its only
      // rounding of the DC is a shift that divides the constant exactly, so fdct(x − 128) ==
      // fdct(x) with DC − 64·128 (checked for all-extreme and random blocks). Saves 64 VALU ops.
      // islow FDCT as 16-bit dot products (jpeg_common.h fdct_islow_dot): 63 fewer static VALU
      // instructions than the multiply/add form and no scratch spills (20 scratch instructions).
      fdct_islow_dot(blk);
      blk[0] -= 64 * 128;
      // Quantise into packed pairs first (frees the 64 int32 DCT registers), then walk the zig-zag
      // order from those registers. Sign-magnitude halves: |q| in bits 0–14 (16–30), the
      // coefficient's sign in bit 15 (31) — the coder needs |q| for the category and the sign only
      // to complement the magnitude bits, so the quotient is never negated back (|q| < 2^14: the
      // islow coefficients of 8-bit samples stay below 2^15 and every divisor is ≥ 2). Per pair:
      // 2 × (abs, add, mul_hi) + one byte permute for the signs + one bit-field insert.
      uint32_t zp[32];
#pragma unroll
      for (int k = 0; k < 64; k += 2) {
        const int32_t xa = blk[kNatural[k]], xc = blk[kNatural[k + 1]];
        const uint32_t mags = quant_mag(xa, q, kNatural[k]) | (quant_mag(xc, q, kNatural[k + 1]) << 16);
        const uint32_t signs = ((uint32_t)xa >> 16) | ((uint32_t)xc & 0xFFFF0000u);
        zp[k >> 1] = (mags & ~0x80008000u) | (signs & 0x80008000u);
      }
      {
        const int a0 = (int)(zp[0] & 0x7FFFu);
        dc0 = (zp[0] & 0x8000u) ? -a0 : a0;
      }
      if (dbg == 16) {  // profiling variant: stop after the FDCT and quantisation
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) acc ^= zp[i] * (uint32_t)(2 * i + 1);
        if (acc == 0x7FFFFFF1u) out_sizes[0] = 1;
        return;
      }
      // Outer loop not unrolled: zp[j] is indexed by a wave-uniform counter (register indexing, no
      // scratch), keeping the code compact.
#pragma unroll 1
      for (int j = 0; j < 32; ++j) {
        const uint32_t word = zp[j];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int k = 2 * j + h;
          const uint32_t half = word >> (16 * h);
          const uint32_t av = half & 0x7FFFu;  // |q|; bit 15 of `half`: its sign
          if (k > 0 && __ballot(av != 0)) {
            if (av != 0) {
              int run = k - last - 1;
              while (run > 15) {
                lw.put_sym(actab[0xF0]);
                run -= 16;
              }
              const int nb = 32 - __builtin_clz(av);
              const uint32_t e = actab[(run << 4) + nb];  // symbol and magnitude in one put (≤ 27 bits)
              // Magnitude bits: q for q > 0, q − 1 = ~|q| for q < 0 (low nb bits).
              const uint32_t mag = (av ^ (0u - ((half >> 15) & 1u))) & ((1u << nb) - 1u);
              lw.put(((e & 0xFFFFu) << nb) | mag, (int)(e >> 16) + nb);
              last = k;
            }
          }
        }
      }
    }
    if (last < 63) lw.put_sym(actab[0x00]);
    if (kSamp == kSampling444 || (k420 && (b & 3) == 3)) {  // the MCU's Cb and Cr blocks of a gray image: DC diff 0 + EOB each
      lw.put_sym(kHuffDcChroma.e[0]);
      lw.put_sym(kHuffAcChroma.e[0]);
      lw.put_sym(kHuffDcChroma.e[0]);
      lw.put_sym(kHuffAcChroma.e[0]);
    }
    lw.finish();
    acbits = lw.bits;
  }
  if (dbg == 2) {  // profiling variant: stop after FDCT + quantisation + AC coding
    if (dc0 == 0x7FFFFFF1 || acbits == 0x7FFFFFF1u) out_sizes[0] = 1;
    return;
  }
  sdc[tid] = dc0;
  // DC of the block preceding this workgroup's first block (0 at the start of the image).
  if (tid < 64) {
    int dcp = 0;
    if (part > 0 && dbg != 17) {  // dbg 17: profiling variant without the predecessor's DC (output invalid)
      int pbx, pby;
      block_xy(part * kWG - 1, pbx, pby);
      const int u = 8 * pbx + (tid & 7);
      const int v = 8 * pby + (tid >> 3);
      const int px = d.render >= 0 ? (int)render_pixel(rd, rs.raw, rs.f32, rs.bits, win, u, v)
                                   : (int)canvas[d.canvas_off + (size_t)v * out_w + u];
      dcp = quant_recip(wave_sum_i32(px - 128), q, 0);
    }
    if (tid == 0) s_prevdc = dcp;
  }
  __syncthreads();
  uint32_t agg = 0, nlocal = 0;
  bool in_lds = true;
  // DC code (Huffman symbol + magnitude bits, ≤ 20 bits, right-aligned).
  const int diff = dc0 - (tid ? sdc[tid - 1] : s_prevdc);
  const int dn = mag_bits_fast(diff);
  const uint32_t dce = dctab[dn];
  const int dclen = valid ? (int)(dce >> 16) + dn : 0;
  const uint32_t dccode = ((dce & 0xFFFFu) << dn) | ((uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << dn) - 1u));
  const uint32_t bits = valid ? (uint32_t)dclen + acbits : 0u;
  // ---- 3. workgroup scan, bit range assembled in LDS ----------------------------------------
  const uint32_t excl = block_exclusive_scan(bits, sh, &agg);  // ends with a barrier
  // Each block's DC code, then its AC words shifted behind it, into the workgroup's contiguous
  // bit range (MSB-first words), in the LDS region the render patch used. A range too long for
  // it (> ~220 Kbit: pathological detail) poisons the image, which the host then re-encodes.
  nlocal = (agg + 31) >> 5;
  in_lds = nlocal + 2u <= (uint32_t)kUnion;  // workgroup-uniform
  const uint32_t nwp = (acbits + 31) >> 5;
  const uint32_t acpos = excl + (uint32_t)dclen;
  if (in_lds) {
    for (uint32_t i = tid; i <= nlocal; i += kWG) swg[i] = 0u;
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
  // ---- 4. this workgroup's stuffing record -------------------------------------------------
  // Output byte k (bits 8k..8k+7 of the image's segment) belongs to the workgroup holding its
  // last bit; its offset in the stuffed output is k + (0xFF bytes before k). Whether a byte is
  // 0xFF depends on where the workgroup's range starts inside a byte (a = start mod 8), known only
  // after the look-back — so the record carries, for all eight alignments, the number of 0xFF
  // bytes lying wholly inside the range (ff[a]), plus its leading-ones count and last 7 bits
  // (the byte that straddles two workgroups). Successors then resolve any chain of aggregates.
  const uint32_t A = agg;
  uint32_t ffc[8];
#pragma unroll
  for (int al = 0; al < 8; ++al) ffc[al] = 0;
  if (in_lds) {
    // All eight alignments in one pass over the range's 32-bit words: bit q (MSB first) of
    // `r` says whether the 8 bits starting at range bit 32j + q are all ones (three shift-ANDs on
    // the word and the next one); a byte of alignment `al` starts at f + 8i, f = (8 − al) & 7, and
    // must end within the range (p + 8 ≤ A), so its count is popcount(r & (0x80808080 >> f)) over
    // the valid positions — instead of one LDS byte extraction per byte and alignment.
    const uint32_t nw = (A + 31u) >> 5;  // the range buffer has ≥ 2 words of slack (in_lds)
    for (uint32_t j = tid; j < nw; j += kWG) {
      const int32_t lim = (int32_t)A - 8 - 32 * (int32_t)j;  // last q whose byte fits in the range
      if (lim < 0) continue;
      const uint64_t v = ((uint64_t)swg[j] << 32) | swg[j + 1];
      uint64_t run = v & (v << 1);
      run &= run << 2;
      run &= run << 4;  // bit k: bits k .. k−7 of v all set
      uint32_t r = (uint32_t)(run >> 32);
      if (lim < 31) r &= ~((1u << (31 - lim)) - 1u);
#pragma unroll
      for (int al = 0; al < 8; ++al) ffc[al] += (uint32_t)__popc(r & (0x80808080u >> ((8 - al) & 7)));
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int al = 0; al < 8; ++al) ffc[al] = (uint32_t)wave_sum_i32((int)ffc[al]);
  if (lane == 0) {
#pragma unroll
    for (int al = 0; al < 8; ++al) sff[wv * 8 + al] = ffc[al];
  }
  __syncthreads();
  uint64_t* look = w.look + w.look_base + (size_t)img * parts * 3;
  if (tid < 64) {
    uint32_t ff[8];
#pragma unroll
    for (int al = 0; al < 8; ++al) {
      ff[al] = 0;
#pragma unroll
      for (int wq = 0; wq < kWG / 64; ++wq) ff[al] += sff[wq * 8 + al];
    }
    const uint32_t w0 = in_lds ? swg[0] : 0u;
    const uint32_t lead = ~w0 ? (uint32_t)__builtin_clz(~w0) : 32u;
    const uint32_t head = min(min(lead, 8u), A);  // leading ones of the range
    const uint32_t tail = in_lds && A >= 7 ? lds_bits(swg, A - 7, 7) : (in_lds ? lds_bits(swg, 0, A) : 0u);
    const bool poison = !in_lds || A >= (1u << 20) || ff[0] > 0x7FFFu;
    // ---- 5. publish the aggregate (3 words), then the decoupled look-back ----------------------
    if (lane == 0 && part < parts - 1) {
      look_store64(&look[3 * part + 1], (1ull << 62) | ((uint64_t)(ff[2] & 0x7FFF) << 45) |
                                            ((uint64_t)(ff[3] & 0x7FFF) << 30) | ((uint64_t)(ff[4] & 0x7FFF) << 15) |
                                            (uint64_t)(ff[5] & 0x7FFF));
      look_store64(&look[3 * part + 2], (1ull << 62) | ((uint64_t)(ff[6] & 0x7FFF) << 15) | (uint64_t)(ff[7] & 0x7FFF));
      look_store64(&look[3 * part], (1ull << 62) | ((uint64_t)poison << 61) | ((uint64_t)(A & 0xFFFFF) << 41) |
                                        ((uint64_t)tail << 34) | ((uint64_t)head << 30) |
                                        ((uint64_t)(ff[0] & 0x7FFF) << 15) | (uint64_t)(ff[1] & 0x7FFF));
    }
    // Lane l looks at part (hi − l): the nearest inclusive record ends the window; the aggregates
    // after it are resolved in order (their start bits are the inclusive end plus a suffix sum of
    // aggregate lengths, which fixes every alignment). Part −1 is an inclusive (0, 0) sentinel.
    uint32_t p_start = 0, ff_before = 0, tail_prev = 0;
    bool bad = poison;
    if (part > 0) {
      const int hi = part - 1;
      uint32_t spins = 0;
      uint64_t r0 = 0, r1 = 0, r2 = 0;
      int stop;
      for (;;) {
        const int q = hi - lane;
        uint32_t tag = 2;
        r0 = 2ull << 62;
        r1 = r2 = 0;
        if (q >= 0) {
          r0 = look_load(&look[3 * q]);
          tag = (uint32_t)(r0 >> 62);
          if (tag == 1u) {
            r1 = look_load(&look[3 * q + 1]);
            r2 = look_load(&look[3 * q + 2]);
            if ((r1 >> 62) != 1u || (r2 >> 62) != 1u) tag = 0;  // words land one by one
          }
        }
        const uint64_t incl = __ballot(tag == 2u);
        stop = incl ? __builtin_ctzll(incl) : 64;
        const uint64_t need = stop >= 63 ? ~0ull : ((2ull << stop) - 1ull);
        if ((__ballot(tag == 0u) & need) || stop == 64) {  // a needed record is not published yet
          if (++spins > (1u << 26)) {  // cannot happen with ordered tickets; never hang the GPU
            bad = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        break;
      }
      if (!bad) {
        const bool isagg = lane < stop;
        const uint32_t alen = isagg ? (uint32_t)(r0 >> 41) & 0xFFFFFu : 0u;
        uint32_t suf = alen;  // inclusive suffix sum over lanes l..63
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t t = (uint32_t)__shfl_down((int)suf, o, 64);
          if (lane + o < 64) suf += t;
        }
        // Inclusive record at lane `stop`: end bit, 0xFF count, last 7 bits.
        const uint32_t iend = (uint32_t)__shfl((int)((uint32_t)(r0 >> 39) & 0x3FFFFFu), stop, 64);
        const uint32_t iff = (uint32_t)__shfl((int)((uint32_t)(r0 >> 19) & 0xFFFFFu), stop, 64);
        const uint32_t mytail = isagg ? (uint32_t)(r0 >> 34) & 0x7Fu : (uint32_t)(r0 >> 12) & 0x7Fu;
        const uint32_t prevtail = (uint32_t)__shfl_down((int)mytail, 1, 64);  // part q − 1's last bits
        const uint32_t qstart = iend + (suf - alen);
        const uint32_t al = qstart & 7u;
        uint32_t fq = 0;
        if (isagg) {
          const uint32_t sel = al < 2 ? (uint32_t)(r0 >> (al ? 0 : 15)) : al < 6 ? (uint32_t)(r1 >> (15 * (5 - al)))
                                                                                : (uint32_t)(r2 >> (15 * (7 - al)));
          fq = sel & 0x7FFFu;
          const uint32_t hq = (uint32_t)(r0 >> 30) & 0xFu, m = (1u << al) - 1u;
          if (al && (prevtail & m) == m && hq >= 8u - al) ++fq;  // the straddling byte
        }
        const bool pois = __ballot(lane <= stop && ((r0 >> 61) & 1ull)) != 0;
        bad = bad || pois;
        ff_before = iff + (uint32_t)wave_sum_i32((int)fq);
        p_start = iend + (uint32_t)__shfl((int)suf, 0, 64);
        tail_prev = (uint32_t)__shfl((int)mytail, 0, 64);
      }
    }
    // ---- 6. own 0xFF count, inclusive record ---------------------------------------------------
    const uint32_t al = p_start & 7u, f = (8u - al) & 7u;
    const bool last = part == parts - 1;
    uint32_t own = 0, nown = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) own = al == (uint32_t)k ? ff[k] : own;  // select: ff stays in VGPRs (no scratch)
    bool strad = false, fin = false;
    uint32_t strad_v = 0, fin_v = 0;
    if (al) {  // the byte shared with the previous workgroup
      strad = true;
      const uint32_t take = min(8u - al, A);
      strad_v = ((tail_prev & ((1u << al) - 1u)) << (8u - al)) | (lds_bits(swg, 0, take) << (8u - al - take));
      if (take < 8u - al) strad_v |= (1u << (8u - al - take)) - 1u;  // final byte: pad with ones
      own += strad_v == 0xFFu;
    }
    const uint32_t nfull = A >= f ? (A - f) >> 3 : 0u;
    const uint32_t rem = A >= f ? A - f - 8u * nfull : 0u;
    if (last && rem) {  // the image's final partial byte, padded with 1-bits
      fin = true;
      fin_v = (lds_bits(swg, f + 8u * nfull, rem) << (8u - rem)) | ((1u << (8u - rem)) - 1u);
      own += fin_v == 0xFFu;
    }
    nown = (uint32_t)strad + nfull + (uint32_t)fin;
    const uint32_t end = p_start + A;
    bad = bad || end >= (1u << 22) || ff_before + own >= (1u << 20);
    const uint32_t obase = (p_start >> 3) + ff_before;
    // Exact end of this workgroup's stuffed bytes (own = its 0xFF count). It must be exact, not a
    // bound: a later workgroup that saw this one only as an aggregate never learns its flag, so the
    // flag has to follow from positions alone (ends are monotone along the image: once one
    // workgroup's end passes the capacity every later start does, and the last part reports -1).
    // A conservative 2 × nown bound let a workgroup drop its bytes while the image still reported
    // a size (tests/test_gpu.py::test_engine_jpeg_d2h_identical, capacity 20000).
    bad = bad || obase + nown + own > d.out_cap;
    if (lane == 0) {
      look_store64(&look[3 * part], (2ull << 62) | ((uint64_t)bad << 61) | ((uint64_t)(end & 0x3FFFFF) << 39) |
                                        ((uint64_t)((ff_before + own) & 0xFFFFF) << 19) |
                                        ((uint64_t)(in_lds ? (A >= 7 ? lds_bits(swg, A - 7, 7) : 0u) : 0u) << 12));
      s_bad = bad;
      s_obase = obase;
      s_nown = nown;
      s_strad = strad;
      s_fin = fin;
      s_strad_v = strad_v;
      s_fin_v = fin_v;
      s_f = f;
      s_nwords = nlocal + 2u;
      if (last) out_sizes[img] = bad ? -1 : (int32_t)(((end + 7u) >> 3) + ff_before + own);
    }
  }
  __syncthreads();
  if (dbg == 4 || s_bad) return;
  // ---- 7. stuffed bytes straight into the host-mapped output --------------------------------
  // Thread t takes a contiguous run of the owned bytes; a block scan of (bytes + 0xFF count) gives
  // every run its output position; the stuffed bytes are staged in LDS behind the bit range and
  // copied out with consecutive lanes on consecutive bytes.
  const uint32_t nown = s_nown, f = s_f, hs = s_strad ? 1u : 0u;
  const uint32_t per = (nown + kWG - 1) / kWG;
  const uint32_t j0 = min(nown, tid * per), j1 = min(nown, j0 + per);
  auto owned = [&](uint32_t j) -> uint32_t {
    if (j < hs) return s_strad_v;
    const uint32_t i = j - hs;
    const uint32_t nfull = nown - hs - (s_fin ? 1u : 0u);
    return i < nfull ? lds_byte(swg, f + 8u * i) : s_fin_v;
  };
  uint32_t cnt = 0;
  for (uint32_t j = j0; j < j1; ++j) cnt += owned(j) == 0xFFu ? 2u : 1u;
  uint32_t tot = 0;
  uint32_t o = block_exclusive_scan(cnt, sh, &tot);
  uint8_t* dst = out + d.out_off + s_obase;
  // Staged bytes sit at the destination's 16-byte phase behind the bit range, so 16-byte chunks of
  // the output are 16-byte chunks of LDS (one ds_read_b128 + one dwordx4 host store per lane).
  const uint32_t phase = (uint32_t)((uintptr_t)dst & 15u);
  uint8_t* sbuf = reinterpret_cast<uint8_t*>(swg + ((s_nwords + 3u) & ~3u)) + phase;  // behind the bit range
  const bool staged_out = tot + phase <= (uint32_t)(kUnion - ((s_nwords + 3u) & ~3u)) * 4u;
  for (uint32_t j = j0; j < j1; ++j) {
    const uint32_t v = owned(j);
    if (staged_out) {
      sbuf[o++] = (uint8_t)v;
      if (v == 0xFFu) sbuf[o++] = 0;
    } else {
      dst[o++] = (uint8_t)v;
      if (v == 0xFFu) dst[o++] = 0;
    }
  }
  if (staged_out) {
    __syncthreads();
    if (dbg == 15) {  // profiling variant: staged, not stored
      if (tot == 0x7FFFFFF1u) out_sizes[0] = sbuf[tid];
      return;
    }
    // Chunk c covers destination bytes [16c − phase, 16c + 16 − phase) of the range; the first and
    // last chunks may be partial (byte stores), the rest move whole.
    const uint32_t nchunks = (phase + tot + 15u) >> 4;
    uint8_t* const dbase = dst - phase;  // 16-byte aligned
    const uint8_t* const lbase = sbuf - phase;
    for (uint32_t c = tid; c < nchunks; c += kWG) {
      const uint32_t b0 = 16u * c, lo = max(b0, phase), hi = min(b0 + 16u, phase + tot);
      if (lo == b0 && hi == b0 + 16u) {
        // Non-temporal: the bytes go to host memory over PCIe and are never read back on the GPU.
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(lbase + b0), reinterpret_cast<u32x4*>(dbase + b0));
      } else {
        for (uint32_t k = lo; k < hi; ++k) dbase[k] = lbase[k];
      }
    }
  }
}

bool render_is_exact_2x(const RenderDesc& r, int out_w, int out_h) {
  return r.invx == 0.5f && r.invy == 0.5f && r.ox == 0.0f && r.oy == 0.0f && 2 * r.src_w == out_w &&
         2 * r.src_h == out_h && (r.src_w % 4) == 0;
}

void launch_jpeg(const uint8_t* canvas, const JpegDesc* jd, int ncanvas, int out_w, int out_h, const int32_t* div_luma,
                 JpegWork& w, uint8_t* out, int32_t* out_sizes, hipStream_t stream, const JpegRenderSrc* fused,
                 int sampling, bool nearest) {
  if (ncanvas <= 0) return;
  if (sampling < kSampling420 || sampling > kSamplingGray) throw DeviceError("launch_jpeg: unknown sampling");
  if (out_w % 16 || out_h % 16) throw DeviceError("GPU JPEG encoder needs canvas dims that are multiples of 16");
  if (!w.look || !w.ticket || !w.spill) throw DeviceError("launch_jpeg: JpegWork incomplete");
  if (w.look_base && w.look_base != 3 * w.look_cap) throw DeviceError("launch_jpeg: look area state corrupt");
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
  // NM03_PROFILE_VARIANT=jpeg=N selects truncated profiling variants (output invalid; time them
  // with rocprofv3 --kernel-trace --stats).
  static const int dbg = profile_variant("jpeg") & 0xFF;
  if (rs.rd && rs.nrd < ncanvas) throw DeviceError("launch_jpeg: fewer render descriptors than canvases");
  // The look-back records (3 words per workgroup) start unpublished. Eager launches alternate
  // between two halves of the look area, each launch clearing the half the previous one used
  // (stream order makes that safe); captured launches (hipGraph replay repeats the arguments)
  // clear their own half with a memset node instead.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cap);
  const size_t words = (size_t)parts * ncanvas * 3;
  if (cap != hipStreamCaptureStatusNone) {
    w.look_base = 0;
    w.clear_words = 0;
    check_hip(hipMemsetAsync(w.look, 0, words * sizeof(uint64_t), stream), "clear look-back");
  } else {
    const size_t half = 3 * w.look_cap;
    w.clear_base = w.look_base;
    w.clear_words = w.prev_words;
    w.look_base = w.look_base ? 0 : half;
    w.prev_words = words;
  }
  // Fused gray renders with --render-filter nearest have their own 4:2:0 instance; callers send the
  // other layouts' nearest renders through canvases (jpeg_fuses_nearest).
  if (nearest && sampling != kSampling420) throw DeviceError("launch_jpeg: fused nearest renders need 4:2:0");
  auto* kern = nearest                    ? &jpeg_fused_kernel<4, kUnionWords, kSampling420, true>
               : sampling == kSampling420 ? &jpeg_fused_kernel<4, kUnionWords, kSampling420, false>
               : sampling == kSampling444 ? &jpeg_fused_kernel<4, kUnionWords, kSampling444, false>
                                          : &jpeg_fused_kernel<4, kUnionWords, kSamplingGray, false>;
  kern<<<parts * ncanvas, kJpegWG, 0, stream>>>(canvas, jd, ncanvas, out_w, out_h, q, w, rs, out, out_sizes, dbg);
  check_launch("jpeg_fused_kernel");
}

void preload_kernels(bool with_volume) {
  // NM03_PRELOAD_TRACE=1: milliseconds per translation unit on stderr (what a cold start pays for
  // each code object).
  static const int trace = [] {
    const char* e = std::getenv("NM03_PRELOAD_TRACE");
    return e && *e ? std::atoi(e) : 0;  // 2: the same loads in reverse order (first-use cost vs size)
  }();
  auto t = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!trace) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[nm03 preload] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  };
  if (trace == 2) {
    preload_render();
    lap("k3_render");
    preload_srg();
    lap("k2_srg_morph");
    preload_sharpen();
    lap("k1_sharpen");
  }
  preload_median();
  lap("k1_median");
  preload_sharpen();
  lap("k1_sharpen");
  preload_srg();
  lap("k2_srg_morph");
  preload_render();
  lap("k3_render");
  if (with_volume) {
    preload_volume();
    preload_threshold();
    lap("k5_volume+k6_threshold");
  }
  hipFuncAttributes a;
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&jpeg_fused_kernel<4, kUnionWords, kSampling420, false>)),
            "preload jpeg_fused_kernel");
  lap("k4_jpeg (first instance)");
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&jpeg_fused_kernel<4, kUnionWords, kSampling420, true>)),
            "preload jpeg_fused_kernel nearest");
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&jpeg_fused_kernel<4, kUnionWords, kSampling444, false>)),
            "preload jpeg_fused_kernel 4:4:4");
  check_hip(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&jpeg_fused_kernel<4, kUnionWords, kSamplingGray, false>)),
            "preload jpeg_fused_kernel gray");
  lap("k4_jpeg (other instances)");
}

}  // namespace nm03::gpu
