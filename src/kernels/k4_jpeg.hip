// K4 — JPEG export on the GPU (replaces ImageFileExporter → Qt → libjpeg on the host,
// main_sequential.cpp:61-73). Output is byte-identical to libjpeg(-turbo) baseline q75 4:2:0
// (nm03/jpeg_common.h; golden encoder src/io/jpeg.cpp; tests/test_jpeg.py vs Pillow).
//
// Every stage is massively parallel (a batch of 64 slices = 128 canvases = 524k luma blocks):
//  1 jpeg_block_kernel   thread per 8×8 luma block (MCU order). Pixels come from the canvas, or
//                        — for an exact 2× fit, the common case — are rendered on the fly from the
//                        6×6 source patch (render_core.h), so the 256 KiB canvas never exists.
//                        islow FDCT, quantisation by exact reciprocal multiply (umulhi by
//                        ceil(2^32/d): exact for |x| < 2^16, d < 2^16), zig-zag, non-zero mask and
//                        the predictor-independent Huffman cost (AC codes, ZRLs, EOB).
//  2 jpeg_scan_kernel    workgroup per image: DC-difference costs, MCU bit counts (chroma of a
//                        gray canvas is 8 zero bits per MCU), workgroup exclusive scan → bit
//                        offset of every block; zero the image's staging words.
//  3 jpeg_emit_kernel    thread per luma block: writes its codes at its bit offset (atomicOr only
//                        touches words shared with neighbouring blocks' ranges).
//  4 jpeg_stuff_*        workgroup per 4 KiB chunk: count 0xFF bytes; then prefix over previous
//                        chunks, in-chunk scan, stuffed bytes staged in LDS and copied with
//                        64-byte-coalesced stores straight into host-mapped pinned memory.
#include <hip/hip_runtime.h>

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

__global__ __launch_bounds__(256) void jpeg_block_kernel(const uint8_t* __restrict__ canvas,
                                                         const JpegDesc* __restrict__ jd, int ncanvas, int out_w,
                                                         int out_h, QuantRecip q, JpegWork w, JpegRenderSrc rs) {
  // AC code lengths in LDS: 63 per-lane lookups per block become ds_read_u8 instead of gathers.
  __shared__ uint8_t aclen[256];
  aclen[threadIdx.x] = (uint8_t)hlen(kHuffAcLuma.e[threadIdx.x]);
  __syncthreads();
  const int bpi = (out_w >> 3) * (out_h >> 3);
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= bpi * ncanvas) return;
  const int img = gid / bpi, b = gid - img * bpi;
  const JpegDesc d = jd[img];
  const int mcux = out_w >> 4;
  const int mcu = b >> 2, sub = b & 3;
  const int bx = 2 * (mcu % mcux) + (sub & 1), by = 2 * (mcu / mcux) + (sub >> 1);
  int32_t blk[64];
  if (d.render >= 0) {
    const RenderDesc rd = rs.rd[d.render];
    const RWindow win = rd.kind == kRenderLabels ? RWindow{0.f, 0.f} : render_window(rd, rs.stats);
    render_block_2x(rd, rs.raw, rs.f32, rs.bits, win, bx, by, blk);
#pragma unroll
    for (int i = 0; i < 64; ++i) blk[i] -= 128;
  } else {
    const uint8_t* src = canvas + d.canvas_off + (size_t)(by * 8) * out_w + bx * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint2 v = *reinterpret_cast<const uint2*>(src + (size_t)r * out_w);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        blk[r * 8 + c] = (int32_t)((v.x >> (8 * c)) & 0xFF) - 128;
        blk[r * 8 + 4 + c] = (int32_t)((v.y >> (8 * c)) & 0xFF) - 128;
      }
    }
  }
  fdct_islow(blk);
  int16_t zz[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const int n = kNatural[k];
    const int32_t x = blk[n];
    const uint32_t a = (uint32_t)(x < 0 ? -x : x) + q.half[n];
    const int32_t qv = (int32_t)__umulhi(a, q.m[n]);
    zz[k] = (int16_t)(x < 0 ? -qv : qv);
  }
  uint64_t nz = 0;
  uint32_t bits = 0;
  int run = 0;
#pragma unroll
  for (int k = 1; k < 64; ++k) {
    const int v = zz[k];
    if (v == 0) {
      ++run;
    } else {
      nz |= 1ull << k;
      bits += (uint32_t)(run >> 4) * aclen[0xF0];
      const int n = mag_bits_fast(v);
      bits += aclen[((run & 15) << 4) + n] + (uint32_t)n;
      run = 0;
    }
  }
  if (run) bits += aclen[0x00];
  const size_t bi = (size_t)d.coef_off + b;
  uint4* dst = reinterpret_cast<uint4*>(w.coef + bi * 64);
#pragma unroll
  for (int qd = 0; qd < 8; ++qd) {
    uint4 v;
    v.x = (uint16_t)zz[qd * 8 + 0] | ((uint32_t)(uint16_t)zz[qd * 8 + 1] << 16);
    v.y = (uint16_t)zz[qd * 8 + 2] | ((uint32_t)(uint16_t)zz[qd * 8 + 3] << 16);
    v.z = (uint16_t)zz[qd * 8 + 4] | ((uint32_t)(uint16_t)zz[qd * 8 + 5] << 16);
    v.w = (uint16_t)zz[qd * 8 + 6] | ((uint32_t)(uint16_t)zz[qd * 8 + 7] << 16);
    dst[qd] = v;
  }
  w.nzmask[bi] = nz;
  w.acbits[bi] = bits;
  w.dc[bi] = zz[0];
}

__global__ __launch_bounds__(1024) void jpeg_scan_kernel(const JpegDesc* __restrict__ jd, int mcus, JpegWork w,
                                                         int32_t* __restrict__ out_sizes) {
  __shared__ uint32_t sh[17];
  const JpegDesc d = jd[blockIdx.x];
  const int tid = threadIdx.x;
  const int per = (mcus + (int)blockDim.x - 1) / (int)blockDim.x;
  const int m0 = min(tid * per, mcus), m1 = min(m0 + per, mcus);
  const int16_t* dc = w.dc + d.coef_off;
  const uint32_t* acb = w.acbits + d.coef_off;
  const uint32_t chroma_bits = 2u * (hlen(kHuffDcChroma.e[0]) + hlen(kHuffAcChroma.e[0]));
  uint32_t bits = 0;
  for (int m = m0; m < m1; ++m) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int b = 4 * m + s;
      const int diff = (int)dc[b] - (b ? (int)dc[b - 1] : 0);
      const int n = mag_bits_fast(diff);
      bits += hlen(kHuffDcLuma.e[n]) + (uint32_t)n + acb[b];
    }
    bits += chroma_bits;
  }
  uint32_t total = 0;
  uint32_t pos = block_exclusive_scan(bits, sh, &total);
  const uint32_t nbytes = (total + 7) >> 3;
  const bool overflow = nbytes > d.stage_words * 4u || 2u * nbytes + 16u > d.out_cap ||
                        (nbytes + kStuffChunk - 1) / kStuffChunk > (uint32_t)w.max_chunks;
  if (tid == 0) {
    w.total[blockIdx.x] = overflow ? 0xFFFFFFFFu : total;
    if (overflow) out_sizes[blockIdx.x] = -1;
  }
  if (overflow) return;
  uint32_t* boff = w.boff + d.coef_off;
  for (int m = m0; m < m1; ++m) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int b = 4 * m + s;
      boff[b] = pos;
      const int diff = (int)dc[b] - (b ? (int)dc[b - 1] : 0);
      const int n = mag_bits_fast(diff);
      pos += hlen(kHuffDcLuma.e[n]) + (uint32_t)n + acb[b];
    }
    pos += chroma_bits;
  }
  uint32_t* stage = w.stage + d.stage_off;
  const uint32_t nwords = (total + 31) >> 5;
  for (uint32_t i = tid; i < nwords; i += blockDim.x) stage[i] = 0u;
}

struct GBitWriter {
  uint32_t* words;
  uint32_t widx;
  uint64_t acc;
  int nacc;
  __device__ GBitWriter(uint32_t* w, uint32_t pos) : words(w), widx(pos >> 5), acc(0), nacc((int)(pos & 31)) {}
  __device__ __forceinline__ void put(uint32_t code, int len) {
    acc = (acc << len) | (uint64_t)(code & ((1u << len) - 1u));
    nacc += len;
    if (nacc >= 32) {
      const uint32_t wv = (uint32_t)(acc >> (nacc - 32));
      if (wv) atomicOr(&words[widx], wv);
      ++widx;
      nacc -= 32;
      acc &= (1ull << nacc) - 1ull;
    }
  }
  __device__ __forceinline__ void put_sym(uint32_t e) { put(e & 0xFFFFu, (int)(e >> 16)); }
  __device__ __forceinline__ void flush() {
    if (nacc > 0) {
      const uint32_t wv = (uint32_t)(acc << (32 - nacc));
      if (wv) atomicOr(&words[widx], wv);
    }
  }
};

__global__ __launch_bounds__(256) void jpeg_emit_kernel(const JpegDesc* __restrict__ jd, int ncanvas, int bpi,
                                                        JpegWork w) {
  __shared__ uint32_t actab[256];
  __shared__ uint32_t dctab[16];
  actab[threadIdx.x] = kHuffAcLuma.e[threadIdx.x];
  if (threadIdx.x < 16) dctab[threadIdx.x] = kHuffDcLuma.e[threadIdx.x];
  __syncthreads();
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= bpi * ncanvas) return;
  const int img = gid / bpi, b = gid - img * bpi;
  if (w.total[img] == 0xFFFFFFFFu) return;
  const JpegDesc d = jd[img];
  const size_t bi = (size_t)d.coef_off + b;
  const int16_t* dc = w.dc + d.coef_off;
  GBitWriter bw(w.stage + d.stage_off, w.boff[bi]);
  const int diff = (int)dc[b] - (b ? (int)dc[b - 1] : 0);
  const int n = mag_bits_fast(diff);
  bw.put_sym(dctab[n]);
  if (n) bw.put((uint32_t)(diff < 0 ? diff - 1 : diff), n);
  uint64_t nz = w.nzmask[bi] & ~1ull;
  const int16_t* cf = w.coef + bi * 64;
  int last = 0;
  while (nz) {
    const int k = __builtin_ctzll(nz);
    nz &= nz - 1;
    int run = k - last - 1;
    while (run > 15) {
      bw.put_sym(actab[0xF0]);
      run -= 16;
    }
    const int v = cf[k];
    const int nb = mag_bits_fast(v);
    bw.put_sym(actab[(run << 4) + nb]);
    bw.put((uint32_t)(v < 0 ? v - 1 : v), nb);
    last = k;
  }
  if (last < 63) bw.put_sym(actab[0x00]);
  bw.flush();
}

// Byte i of the entropy-coded segment (MSB-first words), final byte padded with 1-bits.
__device__ __forceinline__ uint32_t seg_byte(const uint32_t* stage, uint32_t i, uint32_t nbytes, uint32_t padbits) {
  uint32_t v = (stage[i >> 2] >> (24 - 8 * (i & 3))) & 0xFFu;
  if (padbits && i == nbytes - 1) v |= 0xFFu >> padbits;
  return v;
}

constexpr int kStuffThreads = 256;
constexpr int kBytesPerThread = kStuffChunk / kStuffThreads;  // 16

__global__ __launch_bounds__(kStuffThreads) void jpeg_stuff_count_kernel(const JpegDesc* __restrict__ jd, JpegWork w) {
  __shared__ uint32_t cnt;
  const int img = blockIdx.y, chunk = blockIdx.x;
  const uint32_t total = w.total[img];
  if (total == 0xFFFFFFFFu) return;
  const uint32_t nbytes = (total + 7) >> 3;
  const uint32_t c0 = (uint32_t)chunk * kStuffChunk;
  if (c0 >= nbytes) return;
  const JpegDesc d = jd[img];
  const uint32_t* stage = w.stage + d.stage_off;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  uint32_t ff = 0;
  const uint32_t b0 = c0 + threadIdx.x * kBytesPerThread;
  for (int k = 0; k < kBytesPerThread; ++k) {
    const uint32_t i = b0 + k;
    if (i < nbytes) ff += seg_byte(stage, i, nbytes, total & 7u) == 0xFFu;
  }
  if (ff) atomicAdd(&cnt, ff);
  __syncthreads();
  if (threadIdx.x == 0) w.chunk_ff[(size_t)img * w.max_chunks + chunk] = cnt;
}

__global__ __launch_bounds__(kStuffThreads) void jpeg_stuff_write_kernel(const JpegDesc* __restrict__ jd, JpegWork w,
                                                                         uint8_t* __restrict__ out,
                                                                         int32_t* __restrict__ out_sizes) {
  __shared__ uint32_t sh[17];
  __shared__ uint8_t buf[2 * kStuffChunk];
  const int img = blockIdx.y, chunk = blockIdx.x;
  const uint32_t total = w.total[img];
  if (total == 0xFFFFFFFFu) return;
  const uint32_t nbytes = (total + 7) >> 3;
  const uint32_t c0 = (uint32_t)chunk * kStuffChunk;
  if (c0 >= nbytes) return;
  const JpegDesc d = jd[img];
  const uint32_t* stage = w.stage + d.stage_off;
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
  uint32_t o = block_exclusive_scan(mine, sh, &chunk_len);
#pragma unroll
  for (int k = 0; k < kBytesPerThread; ++k) {
    if (v[k] >= 0x100u) continue;
    buf[o++] = (uint8_t)v[k];
    if (v[k] == 0xFFu) buf[o++] = 0;
  }
  __syncthreads();
  uint8_t* dst = out + d.out_off + obase;
  for (uint32_t i = threadIdx.x; i < chunk_len; i += blockDim.x) dst[i] = buf[i];
  if (c0 + kStuffChunk >= nbytes && threadIdx.x == 0) out_sizes[img] = (int32_t)(obase + chunk_len);
}

bool render_is_exact_2x(const RenderDesc& r, int out_w, int out_h) {
  return r.invx == 0.5f && r.invy == 0.5f && r.ox == 0.0f && r.oy == 0.0f && 2 * r.src_w == out_w &&
         2 * r.src_h == out_h && (r.src_w % 4) == 0;
}

void launch_jpeg(const uint8_t* canvas, const JpegDesc* jd, int ncanvas, int out_w, int out_h, const int32_t* div_luma,
                 const JpegWork& w, uint8_t* out, int32_t* out_sizes, hipStream_t stream, const JpegRenderSrc* fused) {
  if (ncanvas <= 0) return;
  if (out_w % 16 || out_h % 16) throw DeviceError("GPU JPEG encoder needs canvas dims that are multiples of 16");
  if (w.max_chunks <= 0 || !w.boff || !w.total || !w.chunk_ff) throw DeviceError("launch_jpeg: JpegWork incomplete");
  QuantRecip q;
  for (int i = 0; i < 64; ++i) {
    const uint32_t dv = (uint32_t)div_luma[i];
    q.half[i] = dv >> 1;
    q.m[i] = (uint32_t)(((1ull << 32) + dv - 1) / dv);
  }
  JpegRenderSrc rs;
  if (fused) rs = *fused;
  const int bpi = (out_w / 8) * (out_h / 8);
  const int nblk = bpi * ncanvas;
  jpeg_block_kernel<<<(nblk + 255) / 256, 256, 0, stream>>>(canvas, jd, ncanvas, out_w, out_h, q, w, rs);
  check_launch("jpeg_block_kernel");
  jpeg_scan_kernel<<<ncanvas, 1024, 0, stream>>>(jd, (out_w / 16) * (out_h / 16), w, out_sizes);
  check_launch("jpeg_scan_kernel");
  jpeg_emit_kernel<<<(nblk + 255) / 256, 256, 0, stream>>>(jd, ncanvas, bpi, w);
  check_launch("jpeg_emit_kernel");
  dim3 sg(w.max_chunks, ncanvas);
  jpeg_stuff_count_kernel<<<sg, kStuffThreads, 0, stream>>>(jd, w);
  check_launch("jpeg_stuff_count_kernel");
  jpeg_stuff_write_kernel<<<sg, kStuffThreads, 0, stream>>>(jd, w, out, out_sizes);
  check_launch("jpeg_stuff_write_kernel");
}

}  // namespace nm03::gpu
