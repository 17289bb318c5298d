// nm03/jpeg_common.h — baseline JPEG (ITU T.81) building blocks shared by the CPU encoder
// (src/io/jpeg.cpp) and the gfx950 encoder (src/kernels/k4_jpeg.hip).
//
// The reference exports through FAST's ImageFileExporter → Qt QImage::save (libjpeg, quality 75,
// 4:2:0, standard Huffman tables, JDCT_ISLOW) — main_sequential.cpp:61-73, SURVEY App. A.9.
// We reproduce libjpeg's arithmetic exactly: the LL&M integer "islow" forward DCT (CONST_BITS=13,
// PASS1_BITS=2, outputs scaled by 8), rounding division by 8·Q, the Annex K tables scaled for
// quality 75, zig-zag order and the standard (Annex K.3) Huffman codes.  A gray canvas maps to
// Y = gray, Cb = Cr = 128 exactly under libjpeg's RGB→YCbCr, so chroma blocks are all-zero.
//
// Acknowledgement: the forward DCT below follows the arithmetic of the Independent JPEG Group's
// jfdctint.c ("islow", the Loeffler–Ligtenberg–Moschytz algorithm as implemented by the IJG) step
// for step, because byte identity with libjpeg requires the same rounding at every stage, and the
// quality scaling follows IJG jcparam.c. This software is based in part on the work of the
// Independent JPEG Group. The tables are ITU T.81 Annex K.
#pragma once

#include <cstdint>

#include "nm03/common.h"

namespace nm03::jpeg {

// Component layout of the exported file. The reference's Qt writer is not pinned on this point
// (SURVEY §7.6 risk 1): an RGB(A) QImage goes out as YCbCr 4:2:0 (libjpeg's default, the
// default here), a Grayscale8 one as a single-component file. 4:4:4 is libjpeg with
// 1×1 chroma sampling. Gray canvases make the chroma blocks all-zero in both YCbCr forms.
enum Sampling : int { kSampling420 = 0, kSampling444 = 1, kSamplingGray = 2 };

// Zig-zag index → natural (row-major) index.
inline constexpr uint8_t kNatural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Annex K.1 tables, natural order.
inline constexpr uint8_t kStdLuma[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
inline constexpr uint8_t kStdChroma[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
    99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// Annex K.3 Huffman specifications: BITS (counts per length 1..16) and HUFFVAL.
inline constexpr uint8_t kDcLumaBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
inline constexpr uint8_t kDcLumaVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
inline constexpr uint8_t kDcChromaBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
inline constexpr uint8_t kDcChromaVals[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
inline constexpr uint8_t kAcLumaBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
inline constexpr uint8_t kAcLumaVals[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61,
    0x07, 0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52,
    0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25,
    0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45,
    0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64,
    0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99,
    0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6,
    0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3,
    0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8,
    0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
inline constexpr uint8_t kAcChromaBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
inline constexpr uint8_t kAcChromaVals[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61,
    0x71, 0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33,
    0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18,
    0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44,
    0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63,
    0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97,
    0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4,
    0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca,
    0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7,
    0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

// Encoder code table: entry = (length << 16) | code, 0 when the symbol is absent.
struct HuffEnc {
  uint32_t e[256];
};

constexpr HuffEnc build_huff(const uint8_t* bits, const uint8_t* vals) {
  HuffEnc h{};
  uint32_t code = 0;
  int k = 0;
  for (int len = 1; len <= 16; ++len) {
    for (int i = 0; i < bits[len - 1]; ++i) {
      h.e[vals[k++]] = ((uint32_t)len << 16) | code;
      ++code;
    }
    code <<= 1;
  }
  return h;
}

inline constexpr HuffEnc kHuffDcLuma = build_huff(kDcLumaBits, kDcLumaVals);
inline constexpr HuffEnc kHuffAcLuma = build_huff(kAcLumaBits, kAcLumaVals);
inline constexpr HuffEnc kHuffDcChroma = build_huff(kDcChromaBits, kDcChromaVals);
inline constexpr HuffEnc kHuffAcChroma = build_huff(kAcChromaBits, kAcChromaVals);

// libjpeg jpeg_quality_scaling + jpeg_add_quant_table(force_baseline=TRUE).
inline void quality_table(const uint8_t* base, int quality, uint16_t* out) {
  if (quality <= 0) quality = 1;
  if (quality > 100) quality = 100;
  int scale = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int i = 0; i < 64; ++i) {
    long t = ((long)base[i] * scale + 50L) / 100L;
    if (t <= 0L) t = 1L;
    if (t > 255L) t = 255L;
    out[i] = (uint16_t)t;
  }
}

// Number of bits of |v| (JPEG magnitude category), v != 0 → 1..15.
NM03_HD int mag_bits(int v) {
  unsigned a = (unsigned)(v < 0 ? -v : v);
  int n = 0;
  while (a) {
    ++n;
    a >>= 1;
  }
  return n;
}

// Products inside the FDCT: every operand fits in 24 signed bits (pass-1 inputs are |x| ≤ 128 sums,
// pass-2 inputs ≤ 2^15) and every product in 31 bits, so the device uses the full-rate
// v_mul_i32_i24 instead of the quarter-rate v_mul_lo_u32 — the results are identical.
NM03_HD int32_t fdct_mul(int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __mul24(a, b);
#else
  return a * b;
#endif
}

// LL&M integer forward DCT, libjpeg jfdctint "islow" arithmetic.  `d` holds 64 level-shifted
// samples (x-128) in natural order; on return it holds coefficients scaled up by 8.
// libjpeg's jfdctint.c islow forward DCT, in two passes (rows, then columns); fdct_islow = both.
#define NM03_DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))
constexpr int kFdctCB = 13, kFdctP1 = 2;
constexpr int32_t kF0_298 = 2446, kF0_390 = 3196, kF0_541 = 4433, kF0_765 = 6270, kF0_899 = 7373, kF1_175 = 9633,
                  kF1_501 = 12299, kF1_847 = 15137, kF1_961 = 16069, kF2_053 = 16819, kF2_562 = 20995, kF3_072 = 25172;

NM03_HD void fdct_islow_pass1(int32_t* d) {
  constexpr int CB = kFdctCB, P1 = kFdctP1;
  for (int r = 0; r < 8; ++r) {
    int32_t* p = d + r * 8;
    int32_t t0 = p[0] + p[7], t7 = p[0] - p[7];
    int32_t t1 = p[1] + p[6], t6 = p[1] - p[6];
    int32_t t2 = p[2] + p[5], t5 = p[2] - p[5];
    int32_t t3 = p[3] + p[4], t4 = p[3] - p[4];
    int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    p[0] = (t10 + t11) * (1 << P1);
    p[4] = (t10 - t11) * (1 << P1);
    int32_t z1 = fdct_mul(t12 + t13, kF0_541);
    p[2] = NM03_DESCALE(z1 + fdct_mul(t13, kF0_765), CB - P1);
    p[6] = NM03_DESCALE(z1 + fdct_mul(t12, -kF1_847), CB - P1);
    z1 = t4 + t7;
    int32_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
    int32_t z5 = fdct_mul(z3 + z4, kF1_175);
    t4 = fdct_mul(t4, kF0_298);
    t5 = fdct_mul(t5, kF2_053);
    t6 = fdct_mul(t6, kF3_072);
    t7 = fdct_mul(t7, kF1_501);
    z1 = fdct_mul(z1, -kF0_899);
    z2 = fdct_mul(z2, -kF2_562);
    z3 = fdct_mul(z3, -kF1_961);
    z4 = fdct_mul(z4, -kF0_390);
    z3 += z5;
    z4 += z5;
    p[7] = NM03_DESCALE(t4 + z1 + z3, CB - P1);
    p[5] = NM03_DESCALE(t5 + z2 + z4, CB - P1);
    p[3] = NM03_DESCALE(t6 + z2 + z3, CB - P1);
    p[1] = NM03_DESCALE(t7 + z1 + z4, CB - P1);
  }
}

NM03_HD void fdct_islow_pass2(int32_t* d) {
  constexpr int CB = kFdctCB, P1 = kFdctP1;
  for (int c = 0; c < 8; ++c) {
    int32_t* p = d + c;
    int32_t t0 = p[0] + p[56], t7 = p[0] - p[56];
    int32_t t1 = p[8] + p[48], t6 = p[8] - p[48];
    int32_t t2 = p[16] + p[40], t5 = p[16] - p[40];
    int32_t t3 = p[24] + p[32], t4 = p[24] - p[32];
    int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    p[0] = NM03_DESCALE(t10 + t11, P1);
    p[32] = NM03_DESCALE(t10 - t11, P1);
    int32_t z1 = fdct_mul(t12 + t13, kF0_541);
    p[16] = NM03_DESCALE(z1 + fdct_mul(t13, kF0_765), CB + P1);
    p[48] = NM03_DESCALE(z1 + fdct_mul(t12, -kF1_847), CB + P1);
    z1 = t4 + t7;
    int32_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
    int32_t z5 = fdct_mul(z3 + z4, kF1_175);
    t4 = fdct_mul(t4, kF0_298);
    t5 = fdct_mul(t5, kF2_053);
    t6 = fdct_mul(t6, kF3_072);
    t7 = fdct_mul(t7, kF1_501);
    z1 = fdct_mul(z1, -kF0_899);
    z2 = fdct_mul(z2, -kF2_562);
    z3 = fdct_mul(z3, -kF1_961);
    z4 = fdct_mul(z4, -kF0_390);
    z3 += z5;
    z4 += z5;
    p[56] = NM03_DESCALE(t4 + z1 + z3, CB + P1);
    p[40] = NM03_DESCALE(t5 + z2 + z4, CB + P1);
    p[24] = NM03_DESCALE(t6 + z2 + z3, CB + P1);
    p[8] = NM03_DESCALE(t7 + z1 + z4, CB + P1);
  }
}
NM03_HD void fdct_islow(int32_t* d) {
  fdct_islow_pass1(d);
  fdct_islow_pass2(d);
}

// The same islow FDCT in dot-product form. With the z-terms distributed out, each odd output is a
// fixed integer combination of t4..t7 and the even pair (2, 6) one of t12, t13 — the very same
// integers (distributivity; no intermediate leaves int32). Every butterfly term fits int16 (pass 1:
// |t| ≤ 510 for 8-bit samples; pass 2: |t| ≤ 16320, pass-1 outputs being ≤ 8160) and so does every
// combined constant (≤ 11363), so on gfx950 an output is one or two v_dot2_i32_i16 (16-bit pairs,
// 32-bit accumulate, the rounding bias as the accumulator seed) instead of the multiply/add chain.
// Host builds evaluate the identical sums with plain int32 arithmetic (tests/native: bit-equal to
// fdct_islow over random and extreme blocks).
NM03_HD int32_t fdct_dot2(int32_t a, int32_t b, int32_t ca, int32_t cb, int32_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef short s2 __attribute__((ext_vector_type(2)));
  const s2 x = {(short)a, (short)b}, c = {(short)ca, (short)cb};
  return __builtin_amdgcn_sdot2(x, c, acc, false);
#else
  return a * ca + b * cb + acc;
#endif
}
namespace fdct_dot {
constexpr int32_t kE2[2] = {kF0_541, kF0_541 + kF0_765}, kE6[2] = {kF0_541 - kF1_847, kF0_541};
// Odd outputs 1, 3, 5, 7 as coefficients of (t4, t5, t6, t7).
constexpr int32_t kO1[4] = {kF1_175 - kF0_899, kF1_175 - kF0_390, kF1_175, kF1_501 - kF0_899 - kF0_390 + kF1_175};
constexpr int32_t kO3[4] = {kF1_175 - kF1_961, kF1_175 - kF2_562, kF3_072 - kF2_562 - kF1_961 + kF1_175, kF1_175};
constexpr int32_t kO5[4] = {kF1_175, kF2_053 - kF2_562 - kF0_390 + kF1_175, kF1_175 - kF2_562, kF1_175 - kF0_390};
constexpr int32_t kO7[4] = {kF0_298 - kF0_899 - kF1_961 + kF1_175, kF1_175, kF1_175 - kF1_961, kF1_175 - kF0_899};
static_assert(kO7[0] == -11363 && kO1[3] == 11363 && kE6[0] == -10704, "combined FDCT constants");

// One 1-D transform of p[0], p[s], ..., p[7s]; pass 2 descales the even outputs by P1 and the
// rotated ones by CB + P1, pass 1 scales the even ones up by P1 and the rotated ones down by CB − P1.
template <bool kPass2>
NM03_HD void fdct_1d(int32_t* p, int s) {
  constexpr int sh = kPass2 ? kFdctCB + kFdctP1 : kFdctCB - kFdctP1;
  constexpr int32_t R = 1 << (sh - 1);
  const int32_t t0 = p[0] + p[7 * s], t7 = p[0] - p[7 * s];
  const int32_t t1 = p[s] + p[6 * s], t6 = p[s] - p[6 * s];
  const int32_t t2 = p[2 * s] + p[5 * s], t5 = p[2 * s] - p[5 * s];
  const int32_t t3 = p[3 * s] + p[4 * s], t4 = p[3 * s] - p[4 * s];
  const int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  if (kPass2) {
    p[0] = NM03_DESCALE(t10 + t11, kFdctP1);
    p[4 * s] = NM03_DESCALE(t10 - t11, kFdctP1);
  } else {
    p[0] = (t10 + t11) * (1 << kFdctP1);
    p[4 * s] = (t10 - t11) * (1 << kFdctP1);
  }
  p[2 * s] = fdct_dot2(t12, t13, kE2[0], kE2[1], R) >> sh;
  p[6 * s] = fdct_dot2(t12, t13, kE6[0], kE6[1], R) >> sh;
  p[1 * s] = fdct_dot2(t6, t7, kO1[2], kO1[3], fdct_dot2(t4, t5, kO1[0], kO1[1], R)) >> sh;
  p[3 * s] = fdct_dot2(t6, t7, kO3[2], kO3[3], fdct_dot2(t4, t5, kO3[0], kO3[1], R)) >> sh;
  p[5 * s] = fdct_dot2(t6, t7, kO5[2], kO5[3], fdct_dot2(t4, t5, kO5[0], kO5[1], R)) >> sh;
  p[7 * s] = fdct_dot2(t6, t7, kO7[2], kO7[3], fdct_dot2(t4, t5, kO7[0], kO7[1], R)) >> sh;
}
}  // namespace fdct_dot

// `d` holds 64 unshifted 8-bit samples (0..255; the int16 bounds above assume it).
NM03_HD void fdct_islow_dot(int32_t* d) {
  for (int r = 0; r < 8; ++r) fdct_dot::fdct_1d<false>(d + 8 * r, 1);
  for (int c = 0; c < 8; ++c) fdct_dot::fdct_1d<true>(d + c, 8);
}
#undef NM03_DESCALE

// Rounding division by the islow divisor (8·Q), sign-symmetric (libjpeg forward_DCT).
NM03_HD int16_t quantize(int32_t v, int32_t divisor) {
  if (v < 0) {
    int32_t t = -v;
    t += divisor >> 1;
    t /= divisor;
    return (int16_t)(-t);
  }
  int32_t t = v + (divisor >> 1);
  t /= divisor;
  return (int16_t)t;
}

// Bits a Huffman-coded luma/chroma block takes (DC diff + AC run/size codes + EOB).
// `zz` is the quantised block in zig-zag order.
NM03_HD int block_bits(const int16_t* zz, int dc_diff, const HuffEnc& dc, const HuffEnc& ac) {
  int nb = mag_bits(dc_diff);
  int bits = (int)(dc.e[nb] >> 16) + nb;
  int run = 0;
  for (int k = 1; k < 64; ++k) {
    int v = zz[k];
    if (v == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bits += (int)(ac.e[0xF0] >> 16);
      run -= 16;
    }
    int n = mag_bits(v);
    bits += (int)(ac.e[(run << 4) + n] >> 16) + n;
    run = 0;
  }
  if (run > 0) bits += (int)(ac.e[0] >> 16);
  return bits;
}

}  // namespace nm03::jpeg
