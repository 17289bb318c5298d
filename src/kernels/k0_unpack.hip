// K0 — expand the uploaded raw region of a batch into the 16-bit sample buffer every later kernel
// reads (nm03/pack12.h): slices shipped as 12-bit pairs are unpacked, 16-bit slices are copied.
// One thread per 16 samples: 24 packed bytes (three 8-byte loads) → 32 bytes (two 16-byte stores).
// HBM-bound and tiny next to the upload it shortens (≈6 MB read, 8 MB written per 64-slice batch).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "nm03/gpu_types.h"
#include "nm03/kernels.h"

namespace nm03::gpu {

__global__ __launch_bounds__(256) void unpack_kernel(const uint16_t* __restrict__ blob_raw, uint16_t* __restrict__ raw,
                                                     const SliceDesc* __restrict__ descs) {
  const SliceDesc d = descs[blockIdx.y];
  const uint32_t npix = (uint32_t)d.w * d.h;
  const uint32_t p0 = (blockIdx.x * blockDim.x + threadIdx.x) * 16u;
  if (p0 >= npix) return;
  uint16_t* dst = raw + d.raw_off + p0;
  if (d.flags & kSliceFlagPacked12) {
    // npix % 16 == 0 for packed slices; byte offset of the group = 1.5 * p0 (8-byte aligned).
    const uint64_t* s = reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(blob_raw + d.blob_off) +
                                                          (size_t)p0 * 3 / 2);
    const uint64_t w0 = s[0], w1 = s[1], w2 = s[2];
    // 192-bit little-endian stream; sample j occupies bits [12j, 12j + 12).
    auto field = [&](int j) -> uint32_t {
      const int b = 12 * j;
      uint64_t v;
      if (b + 12 <= 64) v = w0 >> b;
      else if (b < 64) v = (w0 >> b) | (w1 << (64 - b));
      else if (b + 12 <= 128) v = w1 >> (b - 64);
      else if (b < 128) v = (w1 >> (b - 64)) | (w2 << (128 - b));
      else v = w2 >> (b - 128);
      return (uint32_t)(v & 0xFFFu);
    };
    uint4 a, c;
    a.x = field(0) | (field(1) << 16);
    a.y = field(2) | (field(3) << 16);
    a.z = field(4) | (field(5) << 16);
    a.w = field(6) | (field(7) << 16);
    c.x = field(8) | (field(9) << 16);
    c.y = field(10) | (field(11) << 16);
    c.z = field(12) | (field(13) << 16);
    c.w = field(14) | (field(15) << 16);
    reinterpret_cast<uint4*>(dst)[0] = a;
    reinterpret_cast<uint4*>(dst)[1] = c;
  } else {
    // Plain 16-bit slice: both offsets are multiples of 8 samples; the allocation pads to 8.
    const uint4* s = reinterpret_cast<const uint4*>(blob_raw + d.blob_off + p0);
    uint4* o = reinterpret_cast<uint4*>(dst);
    o[0] = s[0];
    if (p0 + 8 < npix) o[1] = s[1];
  }
}

void launch_unpack(const uint16_t* blob_raw, uint16_t* raw, const SliceDesc* descs, int nslices, int max_pixels,
                   hipStream_t stream) {
  if (nslices <= 0) return;
  const int groups = (max_pixels + 15) / 16;
  dim3 grid((unsigned)((groups + 255) / 256), (unsigned)nslices), block(256);
  unpack_kernel<<<grid, block, 0, stream>>>(blob_raw, raw, descs);
  check_launch("unpack_kernel");
}

// Upload of a small batch as a shader copy from host-mapped pinned memory (engine: batches up to
// NM03_SHADER_UPLOAD_KB). The copy runs on the batch's compute queue, so the median starts without
// an SDMA → compute dependency and does not queue behind other slots' SDMA uploads (a 15-slice
// batch's copy measured 36 µs when alone and up to ≈180 µs beside three others, plus ≈12 µs from
// its end to the first kernel: profiles/r3/single_pass/).
__global__ __launch_bounds__(256) void copy_from_host_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                             size_t n16, const uint8_t* __restrict__ src_tail,
                                                             uint8_t* __restrict__ dst_tail, int tail) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) dst[i] = src[i];
  if (blockIdx.x == 0 && (int)threadIdx.x < tail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
}

void launch_copy_from_host(const void* src, void* dst, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return;
  if (((uintptr_t)src | (uintptr_t)dst) & 15) throw DeviceError("launch_copy_from_host: pointers must be 16-byte aligned");
  const size_t n16 = bytes / 16;
  const int tail = (int)(bytes % 16);
  const size_t groups = std::max<size_t>(1, std::min<size_t>((n16 + 255) / 256, 2048));
  copy_from_host_kernel<<<(unsigned)groups, 256, 0, stream>>>(
      static_cast<const uint4*>(src), static_cast<uint4*>(dst), n16, static_cast<const uint8_t*>(src) + n16 * 16,
      static_cast<uint8_t*>(dst) + n16 * 16, tail);
  check_launch("copy_from_host_kernel");
}

}  // namespace nm03::gpu
