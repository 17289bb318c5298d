// 12-bit transfer packing (include/nm03/pack12.h).
#include "nm03/pack12.h"

#include <immintrin.h>

#include <cstdlib>
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

// Bounce → destination copy with streaming (non-temporal) stores. Cached stores were measured in
// round 3 (would the DMA upload read recently packed lines from the CPU caches instead of DRAM?):
// 292–314k vs 369–389k slices/s — they read every destination line for ownership and evict the
// loaders' working set (profiles/r3/pack_nt/ab.txt).
inline void bounce_out(uint8_t* dst, const uint8_t* src, size_t bytes) { dicom::stream_copy_unfenced(dst, src, bytes); }

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
    bounce_out(dst + i / 2 * 3, bounce, m / 2 * 3);
  }
  _mm_sfence();  // one fence for the whole slice
  return _mm256_testz_si256(acc, _mm256_set1_epi16((short)0xF000));
}

// AVX-512 VBMI form of pack_stream_avx2 (Zen 5 hosts of the MI355X boxes run 512-bit ops at full
// width): 32 samples → 48 bytes per step, one cross-lane byte permute (vpermb) instead of an
// in-lane shuffle + two 16-byte stores. The 64-byte store writes 16 bytes past the step's output
// into the bounce buffer; the next step overwrites them. Samples of a last odd 16 go through pack16.
__attribute__((target("avx2,avx512f,avx512bw,avx512vbmi"))) bool pack_stream_avx512(const uint16_t* src, size_t n,
                                                                                     uint8_t* dst) {
  constexpr size_t kChunk = 2048;
  alignas(64) uint8_t bounce[kChunk / 2 * 3 + 64];
  alignas(64) static const uint8_t kIdx[64] = {
      0,  1,  2,  4,  5,  6,  8,  9,  10, 12, 13, 14, 16, 17, 18, 20, 21, 22, 24, 25, 26, 28,
      29, 30, 32, 33, 34, 36, 37, 38, 40, 41, 42, 44, 45, 46, 48, 49, 50, 52, 53, 54, 56, 57,
      58, 60, 61, 62, 0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0};
  const __m512i idx = _mm512_load_si512(kIdx);
  const __m512i lo_mask = _mm512_set1_epi32(0x00000FFF), hi_mask = _mm512_set1_epi32(0x00FFF000);
  __m512i acc = _mm512_setzero_si512();
  for (size_t i = 0; i < n; i += kChunk) {
    const size_t m = n - i < kChunk ? n - i : kChunk;
    const size_t m32 = m & ~(size_t)31;
    for (size_t k = 0; k < m32; k += 32) {
      const __m512i v = _mm512_loadu_si512(src + i + k);
      acc = _mm512_or_si512(acc, v);
      const __m512i p = _mm512_or_si512(_mm512_and_si512(v, lo_mask), _mm512_and_si512(_mm512_srli_epi32(v, 4), hi_mask));
      _mm512_storeu_si512(bounce + k / 2 * 3, _mm512_permutexvar_epi8(idx, p));
    }
    if (m32 < m) {  // m % 32 == 16
      acc = _mm512_or_si512(acc, _mm512_zextsi256_si512(_mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + m32))));
      pack16(src + i + m32, bounce + m32 / 2 * 3);
    }
    bounce_out(dst + i / 2 * 3, bounce, m / 2 * 3);
  }
  _mm_sfence();
  return _mm512_test_epi16_mask(acc, _mm512_set1_epi16((short)0xF000)) == 0;
}

bool use_avx512() {
  static const bool ok = [] {
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512vbmi");
  }();
  return ok;
}

bool pack_stream_any(const uint16_t* src, size_t n, uint8_t* dst) {
  return use_avx512() ? pack_stream_avx512(src, n, dst) : pack_stream_avx2(src, n, dst);
}

}  // namespace

bool fits12(const uint16_t* src, size_t n) { return n && !(n & 15) && available() && fits_avx2(src, n); }

void pack_stream(const uint16_t* src, size_t n, uint8_t* dst) { (void)pack_stream_any(src, n, dst); }

bool pack_stream_checked(const uint16_t* src, size_t n, uint8_t* dst) {
  return n && !(n & 15) && available() && pack_stream_any(src, n, dst);
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
