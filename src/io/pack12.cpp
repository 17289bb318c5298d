// 12-bit transfer packing (include/nm03/pack12.h).
#include "nm03/pack12.h"

#include <immintrin.h>

#include <cstring>

#include "nm03/dicom.h"

namespace nm03::pack12 {

namespace {

// One pass to test the range (OR of all samples), one to pack 16 samples (32 bytes) into 24: within
// each 32-bit lane the pair (lo, hi) becomes lo | hi << 12 (24 bits), then a byte shuffle drops the
// top byte of every lane and the two 12-byte halves are stored back to back.
__attribute__((target("avx2"))) size_t pack_avx2(const uint16_t* src, size_t n, uint8_t* dst) {
  __m256i acc = _mm256_setzero_si256();
  for (size_t i = 0; i < n; i += 16) acc = _mm256_or_si256(acc, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  if (!_mm256_testz_si256(acc, _mm256_set1_epi16((short)0xF000))) return 0;
  const __m256i lo_mask = _mm256_set1_epi32(0x00000FFF), hi_mask = _mm256_set1_epi32(0x00FFF000);
  const __m256i shuf = _mm256_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1,  //
                                        0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1);
  uint8_t* d = dst;
  for (size_t i = 0; i < n; i += 16, d += 24) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i p = _mm256_or_si256(_mm256_and_si256(v, lo_mask), _mm256_and_si256(_mm256_srli_epi32(v, 4), hi_mask));
    const __m256i c = _mm256_shuffle_epi8(p, shuf);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(d), _mm256_castsi256_si128(c));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(d + 12), _mm256_extracti128_si256(c, 1));
  }
  return n / 2 * 3;
}

__attribute__((target("avx2"))) bool fits_avx2(const uint16_t* src, size_t n) {
  __m256i acc = _mm256_setzero_si256();
  for (size_t i = 0; i < n; i += 16) acc = _mm256_or_si256(acc, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  return _mm256_testz_si256(acc, _mm256_set1_epi16((short)0xF000));
}

// 16 samples → 24 bytes at d (stores 28: callers keep 4 bytes of slack).
__attribute__((target("avx2"))) inline void pack16(const uint16_t* src, uint8_t* d) {
  const __m256i lo_mask = _mm256_set1_epi32(0x00000FFF), hi_mask = _mm256_set1_epi32(0x00FFF000);
  const __m256i shuf = _mm256_setr_epi8(0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1,  //
                                        0, 1, 2, 4, 5, 6, 8, 9, 10, 12, 13, 14, -1, -1, -1, -1);
  const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src));
  const __m256i p = _mm256_or_si256(_mm256_and_si256(v, lo_mask), _mm256_and_si256(_mm256_srli_epi32(v, 4), hi_mask));
  const __m256i c = _mm256_shuffle_epi8(p, shuf);
  _mm_storeu_si128(reinterpret_cast<__m128i*>(d), _mm256_castsi256_si128(c));
  _mm_storeu_si128(reinterpret_cast<__m128i*>(d + 12), _mm256_extracti128_si256(c, 1));
}

// Packs and range-checks in the same pass (one read of the samples): returns false — dst then
// holds garbage the caller must not use — when some sample needs more than 12 bits.
__attribute__((target("avx2"))) bool pack_stream_avx2(const uint16_t* src, size_t n, uint8_t* dst) {
  constexpr size_t kChunk = 2048;  // samples per bounce (3 KiB packed: stays in L1)
  alignas(64) uint8_t bounce[kChunk / 2 * 3 + 32];
  __m256i acc = _mm256_setzero_si256();
  for (size_t i = 0; i < n; i += kChunk) {
    const size_t m = n - i < kChunk ? n - i : kChunk;
    for (size_t k = 0; k < m; k += 16) {
      acc = _mm256_or_si256(acc, _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + k)));
      pack16(src + i + k, bounce + k / 2 * 3);
    }
    dicom::stream_copy_unfenced(dst + i / 2 * 3, bounce, m / 2 * 3);
  }
  _mm_sfence();  // one fence for the whole slice
  return _mm256_testz_si256(acc, _mm256_set1_epi16((short)0xF000));
}

}  // namespace

bool fits12(const uint16_t* src, size_t n) { return n && !(n & 15) && available() && fits_avx2(src, n); }

void pack_stream(const uint16_t* src, size_t n, uint8_t* dst) { (void)pack_stream_avx2(src, n, dst); }

bool pack_stream_checked(const uint16_t* src, size_t n, uint8_t* dst) {
  return n && !(n & 15) && available() && pack_stream_avx2(src, n, dst);
}

bool available() {
  static const bool ok = __builtin_cpu_supports("avx2");
  return ok;
}

size_t pack(const uint16_t* src, size_t n, uint8_t* dst) {
  if (n == 0 || (n & 15) || !available()) return 0;
  return pack_avx2(src, n, dst);
}

void unpack(const uint8_t* src, size_t n, uint16_t* dst) {
  for (size_t k = 0; 2 * k < n; ++k) {
    const uint32_t v = (uint32_t)src[3 * k] | ((uint32_t)src[3 * k + 1] << 8) | ((uint32_t)src[3 * k + 2] << 16);
    dst[2 * k] = (uint16_t)(v & 0xFFFu);
    if (2 * k + 1 < n) dst[2 * k + 1] = (uint16_t)(v >> 12);
  }
}

}  // namespace nm03::pack12
