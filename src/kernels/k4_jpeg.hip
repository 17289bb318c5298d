// K4 — JPEG export on the GPU (replaces ImageFileExporter → Qt → libjpeg on the host,
// main_sequential.cpp:61-73). Output is byte-identical to libjpeg(-turbo) baseline q75 4:2:0
// (see nm03/jpeg_common.h and the golden encoder src/io/jpeg.cpp).
//
// Stage 1 (jpeg_dct_kernel): one thread per 8×8 luma block, blocks in MCU order. islow integer
//   FDCT + rounding quantisation, zig-zag, plus everything of the Huffman cost that does not
//   depend on the DC predictor (AC run/size codes, ZRLs, EOB) and a 64-bit non-zero mask.
// Stage 2 (jpeg_huff_kernel): one 1024-thread workgroup per image. Each thread owns a run of MCUs:
//   DC differences + MCU bit counts → workgroup exclusive scan → every thread knows its bit
//   offset and emits its codes straight into a zeroed word buffer (atomicOr only where words are
//   shared with neighbours' bit ranges). A second scan inserts the 0x00 stuffing after every
//   0xFF byte; the finished segment is copied with 4-byte coalesced stores into host-mapped
//   pinned memory, so no D2H copy and no size round-trip are needed.
// Chroma of a gray canvas is constant 128 → each Cb/Cr block is "DC diff 0, EOB" (4 bits).
#include <hip/hip_runtime.h>

#include "device_util.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg_common.h"
#include "nm03/kernels.h"

namespace nm03::gpu {

using namespace nm03::jpeg;

struct Divs {
  int32_t d[64];
};

__device__ __forceinline__ int mag_bits_fast(int v) {
  const unsigned a = (unsigned)(v < 0 ? -v : v);
  return a ? 32 - __builtin_clz(a) : 0;
}
__device__ __forceinline__ uint32_t hlen(uint32_t e) { return e >> 16; }

__global__ __launch_bounds__(256) void jpeg_dct_kernel(const uint8_t* __restrict__ canvas,
                                                       const JpegDesc* __restrict__ jd, int ncanvas, int out_w,
                                                       int out_h, Divs divs, JpegWork w) {
  const int bpi = (out_w >> 3) * (out_h >> 3);
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= bpi * ncanvas) return;
  const int img = gid / bpi, b = gid - img * bpi;
  const JpegDesc d = jd[img];
  const int mcux = out_w >> 4;
  const int mcu = b >> 2, sub = b & 3;
  const int bx = 2 * (mcu % mcux) + (sub & 1), by = 2 * (mcu / mcux) + (sub >> 1);
  const uint8_t* src = canvas + d.canvas_off + (size_t)(by * 8) * out_w + bx * 8;
  int32_t blk[64];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint2 v = *reinterpret_cast<const uint2*>(src + (size_t)r * out_w);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      blk[r * 8 + c] = (int32_t)((v.x >> (8 * c)) & 0xFF) - 128;
      blk[r * 8 + 4 + c] = (int32_t)((v.y >> (8 * c)) & 0xFF) - 128;
    }
  }
  fdct_islow(blk);
  int16_t zz[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) zz[k] = quantize(blk[kNatural[k]], divs.d[kNatural[k]]);
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
      bits += (uint32_t)(run >> 4) * hlen(kHuffAcLuma.e[0xF0]);
      const int n = mag_bits_fast(v);
      bits += hlen(kHuffAcLuma.e[((run & 15) << 4) + n]) + (uint32_t)n;
      run = 0;
    }
  }
  if (run) bits += hlen(kHuffAcLuma.e[0x00]);
  const size_t bi = (size_t)d.coef_off + b;
  uint4* dst = reinterpret_cast<uint4*>(w.coef + bi * 64);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint4 v;
    v.x = (uint16_t)zz[q * 8 + 0] | ((uint32_t)(uint16_t)zz[q * 8 + 1] << 16);
    v.y = (uint16_t)zz[q * 8 + 2] | ((uint32_t)(uint16_t)zz[q * 8 + 3] << 16);
    v.z = (uint16_t)zz[q * 8 + 4] | ((uint32_t)(uint16_t)zz[q * 8 + 5] << 16);
    v.w = (uint16_t)zz[q * 8 + 6] | ((uint32_t)(uint16_t)zz[q * 8 + 7] << 16);
    dst[q] = v;
  }
  w.nzmask[bi] = nz;
  w.acbits[bi] = bits;
  w.dc[bi] = zz[0];
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

__device__ __forceinline__ uint32_t coherent_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t stage_byte(const uint32_t* stage, uint32_t i) {
  const uint32_t wv = coherent_load(stage + (i >> 2));
  return (wv >> (24 - 8 * (i & 3))) & 0xFFu;
}

__global__ __launch_bounds__(1024) void jpeg_huff_kernel(const JpegDesc* __restrict__ jd, int mcus, JpegWork w,
                                                         uint8_t* __restrict__ out, int32_t* __restrict__ out_sizes) {
  __shared__ uint32_t sh[17];
  const JpegDesc d = jd[blockIdx.x];
  const int tid = threadIdx.x;
  const int per = (mcus + (int)blockDim.x - 1) / (int)blockDim.x;
  const int m0 = min(tid * per, mcus), m1 = min(m0 + per, mcus);
  const int16_t* dc = w.dc + d.coef_off;
  const uint32_t* acb = w.acbits + d.coef_off;
  const uint32_t chroma_bits =
      2u * (hlen(kHuffDcChroma.e[0]) + hlen(kHuffAcChroma.e[0]));  // Cb + Cr: DC diff 0 + EOB each
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
  const uint32_t pos = block_exclusive_scan(bits, sh, &total);
  const uint32_t nbytes = (total + 7) >> 3;
  if (nbytes > d.stage_words * 4u || 2u * nbytes + 16u > d.out_cap) {
    if (tid == 0) out_sizes[blockIdx.x] = -1;
    return;
  }
  uint32_t* stage = w.stage + d.stage_off;
  const uint32_t nwords = (total + 31) >> 5;
  for (uint32_t i = tid; i < nwords; i += blockDim.x) stage[i] = 0u;
  __threadfence();
  __syncthreads();

  GBitWriter bw(stage, pos);
  for (int m = m0; m < m1; ++m) {
    for (int s = 0; s < 4; ++s) {
      const int b = 4 * m + s;
      const size_t bi = (size_t)d.coef_off + b;
      const int diff = (int)dc[b] - (b ? (int)dc[b - 1] : 0);
      const int n = mag_bits_fast(diff);
      bw.put_sym(kHuffDcLuma.e[n]);
      if (n) bw.put((uint32_t)(diff < 0 ? diff - 1 : diff), n);
      uint64_t nz = w.nzmask[bi] & ~1ull;
      const int16_t* cf = w.coef + bi * 64;
      int last = 0;
      while (nz) {
        const int k = __builtin_ctzll(nz);
        nz &= nz - 1;
        int run = k - last - 1;
        while (run > 15) {
          bw.put_sym(kHuffAcLuma.e[0xF0]);
          run -= 16;
        }
        const int v = cf[k];
        const int nb = mag_bits_fast(v);
        bw.put_sym(kHuffAcLuma.e[(run << 4) + nb]);
        bw.put((uint32_t)(v < 0 ? v - 1 : v), nb);
        last = k;
      }
      if (last < 63) bw.put_sym(kHuffAcLuma.e[0x00]);
    }
    bw.put_sym(kHuffDcChroma.e[0]);
    bw.put_sym(kHuffAcChroma.e[0]);
    bw.put_sym(kHuffDcChroma.e[0]);
    bw.put_sym(kHuffAcChroma.e[0]);
  }
  bw.flush();
  __threadfence();
  __syncthreads();

  // Byte stuffing: bytes [b0,b1) per thread; the final partial byte is padded with 1-bits.
  const uint32_t per_b = (nbytes + blockDim.x - 1) / blockDim.x;
  const uint32_t b0 = min(tid * per_b, nbytes), b1 = min(b0 + per_b, nbytes);
  const uint32_t padbits = total & 7u;
  auto byte_at = [&](uint32_t i) -> uint32_t {
    uint32_t v = stage_byte(stage, i);
    if (padbits && i == nbytes - 1) v |= 0xFFu >> padbits;
    return v;
  };
  uint32_t cnt = 0;
  for (uint32_t i = b0; i < b1; ++i) cnt += 1u + (byte_at(i) == 0xFFu ? 1u : 0u);
  uint32_t out_total = 0;
  const uint32_t opos = block_exclusive_scan(cnt, sh, &out_total);
  uint8_t* tmp = w.tmp + d.out_off;
  uint32_t o = opos;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t v = byte_at(i);
    tmp[o++] = (uint8_t)v;
    if (v == 0xFFu) tmp[o++] = 0;
  }
  __threadfence();
  __syncthreads();
  const uint32_t nw = (out_total + 3) >> 2;
  const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tmp);
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out + d.out_off);
  for (uint32_t i = tid; i < nw; i += blockDim.x) o32[i] = coherent_load(t32 + i);
  if (tid == 0) out_sizes[blockIdx.x] = (int32_t)out_total;
}

void launch_jpeg(const uint8_t* canvas, const JpegDesc* jd, int ncanvas, int out_w, int out_h, const int32_t* div_luma,
                 const JpegWork& w, uint8_t* out, int32_t* out_sizes, hipStream_t stream) {
  if (ncanvas <= 0) return;
  if (out_w % 16 || out_h % 16) throw DeviceError("GPU JPEG encoder needs canvas dims that are multiples of 16");
  Divs dv;
  for (int i = 0; i < 64; ++i) dv.d[i] = div_luma[i];
  const int bpi = (out_w / 8) * (out_h / 8);
  const int nblk = bpi * ncanvas;
  jpeg_dct_kernel<<<(nblk + 255) / 256, 256, 0, stream>>>(canvas, jd, ncanvas, out_w, out_h, dv, w);
  check_launch("jpeg_dct_kernel");
  jpeg_huff_kernel<<<ncanvas, 1024, 0, stream>>>(jd, (out_w / 16) * (out_h / 16), w, out, out_sizes);
  check_launch("jpeg_huff_kernel");
}

}  // namespace nm03::gpu
