// nm03/pack12.h — 12-bit transfer packing of 16-bit samples for the host→device upload.
//
// MR series store 12-bit samples in 16-bit words (BitsStored = 12 on typical T1 acquisitions); the
// raw pixels are the one large PCIe transfer of the pipeline (128 KiB per 256² slice), and the
// upload engine is the step's bottleneck (ARCHITECTURE.md §6). When every sample of a slice fits in
// 12 bits, the loader ships it as 12-bit pairs — 3 bytes per 2 samples, 25% fewer bytes on PCIe
// and in host memory — and the GPU expands it back to the identical 16-bit words before the first
// kernel (k0_unpack.hip). With BitsStored ≤ 12 the low 12 bits are the sample — every consumer
// masks to the stored bits (key_from_raw) — so such slices are always packed; wider slices are
// packed when every sample fits and otherwise shipped unchanged. Lossless by construction: every
// stage sees the same keys either way.
//
// Layout: pair k = samples (2k, 2k+1) → 24-bit little-endian value s[2k] | s[2k+1] << 12 at byte 3k.
#pragma once

#include <cstddef>
#include <cstdint>

namespace nm03::pack12 {

// True when the CPU has the vector unit the packer uses (AVX2); otherwise pack() always declines.
bool available();

// Packs n samples (n % 16 == 0) into dst (capacity ≥ n * 3 / 2 + 32: the vector stores write up to
// 32 bytes past the packed end) when all fit in 12 bits; returns the packed byte count n * 3 / 2, or
// 0 (dst untouched beyond scratch use) when some sample needs more bits or n % 16 != 0.
size_t pack(const uint16_t* src, size_t n, uint8_t* dst);

// True when n % 16 == 0, the packer is available and every sample fits in 12 bits.
bool fits12(const uint16_t* src, size_t n);

// Packs the low 12 bits of n samples (n % 16 == 0) straight into dst — pinned upload memory — through an
// L1-sized bounce buffer and streaming stores: no full-size intermediate, and exactly n * 3 / 2
// bytes are written (nothing past the end: neighbouring slices may be written concurrently).
void pack_stream(const uint16_t* src, size_t n, uint8_t* dst);

// pack_stream and the range check in one pass over the samples (the engine's path): returns
// whether every sample fit in 12 bits; if not, the n * 3 / 2 bytes written to dst are garbage.
bool pack_stream_checked(const uint16_t* src, size_t n, uint8_t* dst);

// Scalar reference of the inverse (tests; the device expands with k0_unpack.hip).
void unpack(const uint8_t* src, size_t n, uint16_t* dst);

}  // namespace nm03::pack12
