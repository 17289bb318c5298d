// nm03/pixel_math.h — the numerical contract shared bit-for-bit by the CPU golden model
// (src/golden) and the gfx950 HIP kernels (src/kernels). Every function here is NM03_HD and is
// compiled with -ffp-contract=off on both sides, so a given input produces identical f32 bits.
//
// Operational semantics follow SURVEY.md Appendix A (the FAST ops used by the reference,
// main_sequential.cpp:175-262):
//   A.3 normalise + clip   n = ((x-min)/(max-min))*(high-low)+low ; c = min(max(n,cmin),cmax)
//   A.4 median             7×7 median, clamp-to-edge (== FAST VectorMedianFilter on 1-channel data)
//   A.5 sharpen            s = c + gain*(c - G*c), G = normalised 9×9 Gaussian σ=0.5, computed
//                          separably (vertical pass, then horizontal), taps in ascending order
//   A.7 SRG band           0.74 <= s <= 0.91
//   A.9 render             bilinear original (window = slice min/max), nearest labels
#pragma once

#include <cmath>
#include <cstdint>

#include "nm03/common.h"
#include "nm03/params.h"

namespace nm03 {

// ---------------------------------------------------------------------------------------------
// Order-preserving 16-bit keys.  The median of an odd-sized window commutes with any monotone
// map, and raw→(rescale)→normalise→clip is monotone (every step is a correctly-rounded monotone
// f32 op, or a negated one when slope<0, which still maps the median to the median).  So the
// median is computed on raw integer keys (packed v_pk_min/max_u16 on gfx950) and mapped once.
// ---------------------------------------------------------------------------------------------
// `stored_bits` = DICOM BitsStored: unsigned data is masked to it, signed data sign-extended.
NM03_HD uint16_t key_from_raw(uint16_t raw_bits, uint8_t type, uint8_t stored_bits) {
  const int sh = 16 - (int)stored_bits;
  if (type == kI16) {
    int16_t v = (int16_t)(uint16_t)(raw_bits << sh);
    v = (int16_t)(v >> sh);
    return (uint16_t)((uint16_t)v ^ 0x8000u);
  }
  return (uint16_t)(raw_bits & (uint16_t)(0xFFFFu >> sh));
}
NM03_HD float raw_value_from_key(uint16_t key, uint8_t type) {
  if (type == kI16) return (float)(int16_t)(uint16_t)(key ^ 0x8000u);
  return (float)key;
}

struct NormClip {
  float slope, intercept;  // modality rescale (1,0 when absent / disabled)
  float nmin, nmax, nlow, nhigh;
  float cmin, cmax;
};

NM03_HD float rescaled_value(uint16_t key, uint8_t type, float slope, float intercept) {
  float x = raw_value_from_key(key, type);
  if (slope != 1.0f || intercept != 0.0f) {
    float t = x * slope;
    x = t + intercept;
  }
  return x;
}

NM03_HD float norm_clip_value(float x, const NormClip& p) {
  float t = x - p.nmin;
  float r = p.nmax - p.nmin;
  t = t / r;
  float h = p.nhigh - p.nlow;
  t = t * h;
  t = t + p.nlow;
  t = t < p.cmin ? p.cmin : t;
  t = t > p.cmax ? p.cmax : t;
  return t;
}

NM03_HD float norm_clip_key(uint16_t key, uint8_t type, const NormClip& p) {
  return norm_clip_value(rescaled_value(key, type, p.slope, p.intercept), p);
}

// Unsharp mask combine: s = c + gain*(c - b)   (no FMA: -ffp-contract=off everywhere)
NM03_HD float sharpen_combine(float c, float b, float gain) {
  float d = c - b;
  float g = gain * d;
  return c + g;
}

NM03_HD bool in_band(float s, float lo, float hi) { return s >= lo && s <= hi; }

// Normalised 1D Gaussian taps g[i], i = -R..R (R = mask/2), computed in double and rounded once.
// The 2D FAST mask exp(-(i²+j²)/2σ²)/Σ is exactly g[i]·g[j]; we apply it separably.
inline void gaussian_taps(float sigma, int mask, float* out) {
  const int R = mask / 2;
  double sum = 0.0, w[64];
  for (int i = -R; i <= R; ++i) {
    w[i + R] = std::exp(-(double)(i * i) / (2.0 * (double)sigma * (double)sigma));
    sum += w[i + R];
  }
  for (int i = 0; i < mask; ++i) out[i] = (float)(w[i] / sum);
}

// ---------------------------------------------------------------------------------------------
// Render: canvas Wc×Hc black, slice fitted preserving physical aspect, centred.
// ---------------------------------------------------------------------------------------------
struct RenderGeom {
  float ox, oy;      // canvas offset of the displayed rectangle (pixels)
  float invx, invy;  // source pixels per canvas pixel
  int src_w, src_h;
  int out_w, out_h;
};

inline RenderGeom make_render_geom(int src_w, int src_h, float spacing_x, float spacing_y,
                                   int out_w, int out_h) {
  RenderGeom g{};
  if (!(spacing_x > 0.f)) spacing_x = 1.f;
  if (!(spacing_y > 0.f)) spacing_y = 1.f;
  double ew = (double)src_w * spacing_x, eh = (double)src_h * spacing_y;
  double scale = std::fmin((double)out_w / ew, (double)out_h / eh);
  double dw = ew * scale, dh = eh * scale;
  g.ox = (float)(((double)out_w - dw) * 0.5);
  g.oy = (float)(((double)out_h - dh) * 0.5);
  g.invx = (float)((double)src_w / dw);
  g.invy = (float)((double)src_h / dh);
  g.src_w = src_w;
  g.src_h = src_h;
  g.out_w = out_w;
  g.out_h = out_h;
  return g;
}

// Continuous source coordinate (pixel units, pixel centres at k+0.5) of canvas pixel centre u.
NM03_HD float render_src_coord(int u, float o, float inv) {
  float t = (float)u + 0.5f;
  t = t - o;
  return t * inv;
}

// Window mapping of the gray renderers: g = (v - lo) * inv, inv = 1/(hi - lo) computed once per
// image (window_inv). FAST's GLSL shader divides per fragment, which GLSL does not round correctly
// anyway; a per-image reciprocal is the contract here (golden, kernels and torch reference agree).
NM03_HD float window_inv(float lo, float hi) {
  const float r = hi - lo;
  return r > 0.0f ? 1.0f / r : 0.0f;
}

NM03_HD uint8_t gray_u8(float v, float lo, float inv) {
  float g = v - lo;
  g = g * inv;
  g = g < 0.0f ? 0.0f : g;
  g = g > 1.0f ? 1.0f : g;
  float t = g * 255.0f;
  t = t + 0.5f;
  return (uint8_t)(int)t;  // t ∈ [0.5, 255.5]: truncation == floor
}

// Bilinear lerp in the order: rows first, then between rows.
NM03_HD float bilerp(float a, float b, float c, float d, float wx, float wy) {
  float ix = 1.0f - wx, iy = 1.0f - wy;
  float t0 = ix * a;
  float t1 = wx * b;
  float top = t0 + t1;
  float t2 = ix * c;
  float t3 = wx * d;
  float bot = t2 + t3;
  float u0 = iy * top;
  float u1 = wy * bot;
  return u0 + u1;
}

NM03_HD int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// Opacity → u8 colour over black background (label colour White).
inline uint8_t opacity_u8(float alpha) {
  float t = alpha * 255.0f;
  t = t + 0.5f;
  int v = (int)std::floor(t);
  return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

}  // namespace nm03
