// CPU golden model (see include/nm03/golden.h). Straightforward, obviously-correct code: the
// point is to be an independent oracle for the gfx950 kernels, not to be fast.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>

#include "nm03/dicom.h"
#include "nm03/golden.h"
#include "nm03/jpeg.h"

namespace nm03::golden {

SliceInput load_slice(const std::string& path, int min_dim, int frame) {
  std::vector<uint8_t> buf = dicom::read_file(path);
  dicom::Header h = dicom::parse(buf.data(), buf.size());
  const int f = dicom::select_frame(h, frame);
  if (min_dim > 0 && (h.cols < min_dim || h.rows < min_dim))
    throw SliceError("Image dimensions too small: " + std::to_string(h.cols) + "x" + std::to_string(h.rows));
  SliceInput s;
  s.w = h.cols;
  s.h = h.rows;
  s.type = h.type;
  s.stored_bits = h.type == kU8 ? 8 : h.bits_stored;
  s.slope = h.slope;
  s.intercept = h.intercept;
  s.spacing_x = h.spacing_x;
  s.spacing_y = h.spacing_y;
  s.raw.resize((size_t)s.w * s.h);
  dicom::copy_pixels16(h, buf.data(), buf.size(), s.raw.data(), f);
  if (s.type == kU8) s.type = kU16;  // widened; stored_bits keeps the 8-bit mask
  return s;
}

NormClip make_normclip(const SliceInput& s, const PipelineParams& p) {
  NormClip n;
  n.slope = p.apply_rescale ? s.slope : 1.f;
  n.intercept = p.apply_rescale ? s.intercept : 0.f;
  n.nmin = p.norm_min;
  n.nmax = p.norm_max;
  n.nlow = p.norm_low;
  n.nhigh = p.norm_high;
  n.cmin = p.clip_min;
  n.cmax = p.clip_max;
  return n;
}

std::vector<uint16_t> keys(const SliceInput& s) {
  std::vector<uint16_t> k(s.raw.size());
  for (size_t i = 0; i < k.size(); ++i) k[i] = key_from_raw(s.raw[i], s.type, (uint8_t)s.stored_bits);
  return k;
}

std::vector<float> norm_clip(const SliceInput& s, const PipelineParams& p) {
  NormClip n = make_normclip(s, p);
  std::vector<float> out(s.raw.size());
  for (size_t i = 0; i < out.size(); ++i)
    out[i] = norm_clip_key(key_from_raw(s.raw[i], s.type, (uint8_t)s.stored_bits), s.type, n);
  return out;
}

std::vector<float> rescaled(const SliceInput& s, const PipelineParams& p) {
  NormClip n = make_normclip(s, p);
  std::vector<float> out(s.raw.size());
  for (size_t i = 0; i < out.size(); ++i)
    out[i] = rescaled_value(key_from_raw(s.raw[i], s.type, (uint8_t)s.stored_bits), s.type, n.slope, n.intercept);
  return out;
}

template <class T>
static std::vector<T> median_t(const std::vector<T>& img, int w, int h, int k) {
  const int r = k / 2;
  std::vector<T> out(img.size()), win((size_t)k * k);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int n = 0;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx)
          win[n++] = img[(size_t)clampi(y + dy, 0, h - 1) * w + clampi(x + dx, 0, w - 1)];
      std::nth_element(win.begin(), win.begin() + n / 2, win.begin() + n);
      out[(size_t)y * w + x] = win[n / 2];
    }
  return out;
}

std::vector<float> median(const std::vector<float>& img, int w, int h, int k) { return median_t(img, w, h, k); }
std::vector<uint16_t> median_u16(const std::vector<uint16_t>& img, int w, int h, int k) {
  return median_t(img, w, h, k);
}

std::vector<float> vector_median(const std::vector<float>& img, int w, int h, int k) {
  const int r = k / 2;
  std::vector<float> out(img.size()), win((size_t)k * k);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int n = 0;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx)
          win[n++] = img[(size_t)clampi(y + dy, 0, h - 1) * w + clampi(x + dx, 0, w - 1)];
      int best = 0;
      float best_s = INFINITY;
      for (int a = 0; a < n; ++a) {
        float s = 0.f;
        for (int b = 0; b < n; ++b) s += std::fabs(win[a] - win[b]);
        if (s < best_s) {
          best_s = s;
          best = a;
        }
      }
      out[(size_t)y * w + x] = win[best];
    }
  return out;
}

// Contract order shared with K1b: vertical pass, then horizontal, taps ascending, each tap one fused
// multiply-add (IEEE fma: one rounding, so host and v_pk_fma_f32 agree bit for bit). Hosts without
// FMA3 run the default clone, whose std::fma is libm's correctly rounded one: the same results.
__attribute__((target_clones("fma", "default"))) std::vector<float> sharpen(const std::vector<float>& img, int w,
                                                                            int h, float gain, float sigma,
                                                                            int mask) {
  float g[64];
  gaussian_taps(sigma, mask, g);
  const int R = mask / 2;
  std::vector<float> tmp(img.size()), out(img.size());
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float acc = 0.0f;
      for (int i = -R; i <= R; ++i) {
        acc = std::fma(g[i + R], img[(size_t)clampi(y + i, 0, h - 1) * w + x], acc);
      }
      tmp[(size_t)y * w + x] = acc;
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float acc = 0.0f;
      for (int j = -R; j <= R; ++j) {
        acc = std::fma(g[j + R], tmp[(size_t)y * w + clampi(x + j, 0, w - 1)], acc);
      }
      const float c = img[(size_t)y * w + x];
      out[(size_t)y * w + x] = sharpen_combine(c, acc, gain);
    }
  return out;
}

std::vector<float> sharpen_direct(const std::vector<float>& img, int w, int h, float gain, float sigma, int mask) {
  const int R = mask / 2;
  std::vector<double> m2((size_t)mask * mask);
  double sum = 0;
  for (int i = -R; i <= R; ++i)
    for (int j = -R; j <= R; ++j) {
      double v = std::exp(-(double)(i * i + j * j) / (2.0 * sigma * sigma));
      m2[(size_t)(i + R) * mask + (j + R)] = v;
      sum += v;
    }
  std::vector<float> m2f(m2.size());
  for (size_t i = 0; i < m2.size(); ++i) m2f[i] = (float)(m2[i] / sum);
  std::vector<float> out(img.size());
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      float acc = 0.f;
      for (int i = -R; i <= R; ++i)
        for (int j = -R; j <= R; ++j)
          acc += m2f[(size_t)(i + R) * mask + (j + R)] *
                 img[(size_t)clampi(y + i, 0, h - 1) * w + clampi(x + j, 0, w - 1)];
      const float c = img[(size_t)y * w + x];
      out[(size_t)y * w + x] = c + gain * (c - acc);
    }
  return out;
}

std::vector<uint8_t> band(const std::vector<float>& s, float lo, float hi) {
  std::vector<uint8_t> b(s.size());
  for (size_t i = 0; i < s.size(); ++i) b[i] = in_band(s[i], lo, hi) ? 1 : 0;
  return b;
}

std::vector<uint8_t> region_grow(const std::vector<uint8_t>& bnd, int w, int h, const std::vector<Seed>& seeds,
                                 int connectivity) {
  std::vector<uint8_t> reg(bnd.size(), 0);
  std::deque<int> q;
  for (const Seed& s : seeds) {
    if (s.x < 0 || s.y < 0 || s.x >= w || s.y >= h) continue;
    const int i = s.y * w + s.x;
    if (bnd[i] && !reg[i]) {
      reg[i] = 1;
      q.push_back(i);
    }
  }
  while (!q.empty()) {
    const int i = q.front();
    q.pop_front();
    const int x = i % w, y = i / w;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dx && !dy) continue;
        if (connectivity == 4 && dx && dy) continue;
        const int nx = x + dx, ny = y + dy;
        if (nx < 0 || ny < 0 || nx >= w || ny >= h) continue;
        const int j = ny * w + nx;
        if (bnd[j] && !reg[j]) {
          reg[j] = 1;
          q.push_back(j);
        }
      }
  }
  return reg;
}

static std::vector<uint8_t> morph(const std::vector<uint8_t>& m, int w, int h, int size, bool dil, bool disc) {
  const int r = size / 2;
  std::vector<uint8_t> out(m.size());
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      bool any = false, all = true;
      for (int dy = -r; dy <= r; ++dy)
        for (int dx = -r; dx <= r; ++dx) {
          if (disc && dx * dx + dy * dy > r * r) continue;
          const int nx = x + dx, ny = y + dy;
          if (nx < 0 || ny < 0 || nx >= w || ny >= h) continue;
          const bool v = m[(size_t)ny * w + nx] != 0;
          any |= v;
          all &= v;
        }
      out[(size_t)y * w + x] = (dil ? any : all) ? 1 : 0;
    }
  return out;
}

std::vector<uint8_t> dilate(const std::vector<uint8_t>& m, int w, int h, int size, bool disc) {
  return morph(m, w, h, size, true, disc);
}
std::vector<uint8_t> erode(const std::vector<uint8_t>& m, int w, int h, int size, bool disc) {
  return morph(m, w, h, size, false, disc);
}

std::vector<uint8_t> border(const std::vector<uint8_t>& m, int w, int h, int radius) {
  if (radius <= 0) return std::vector<uint8_t>(m.size(), 0);
  std::vector<uint8_t> e = erode(m, w, h, 2 * radius + 1), b(m.size());
  for (size_t i = 0; i < m.size(); ++i) b[i] = (m[i] && !e[i]) ? 1 : 0;
  return b;
}

std::vector<uint8_t> region_grow3d(const std::vector<uint8_t>& bnd, int w, int h, int d, const std::vector<Seed>& seeds,
                                   int connectivity) {
  std::vector<uint8_t> reg(bnd.size(), 0);
  std::deque<size_t> q;
  const size_t plane = (size_t)w * h;
  for (const Seed& s : seeds) {
    if (s.x < 0 || s.y < 0 || s.z < 0 || s.x >= w || s.y >= h || s.z >= d) continue;
    const size_t i = (size_t)s.z * plane + (size_t)s.y * w + s.x;
    if (bnd[i] && !reg[i]) {
      reg[i] = 1;
      q.push_back(i);
    }
  }
  while (!q.empty()) {
    const size_t i = q.front();
    q.pop_front();
    const int z = (int)(i / plane), y = (int)((i % plane) / w), x = (int)(i % w);
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int nz = std::abs(dx) + std::abs(dy) + std::abs(dz);
          if (nz == 0 || (connectivity == 6 && nz != 1)) continue;
          const int X = x + dx, Y = y + dy, Z = z + dz;
          if (X < 0 || Y < 0 || Z < 0 || X >= w || Y >= h || Z >= d) continue;
          const size_t j = (size_t)Z * plane + (size_t)Y * w + X;
          if (bnd[j] && !reg[j]) {
            reg[j] = 1;
            q.push_back(j);
          }
        }
  }
  return reg;
}

std::vector<uint8_t> dilate3d(const std::vector<uint8_t>& m, int w, int h, int d, int size, bool ball) {
  const int r = size / 2;
  const size_t plane = (size_t)w * h;
  if (ball) {  // direct definition: OR over the offsets with dx² + dy² + dz² ≤ r²
    std::vector<uint8_t> out(m.size(), 0);
    for (int z = 0; z < d; ++z)
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
          uint8_t v = 0;
          for (int dz = -r; dz <= r && !v; ++dz)
            for (int dy = -r; dy <= r && !v; ++dy)
              for (int dx = -r; dx <= r && !v; ++dx) {
                if (dx * dx + dy * dy + dz * dz > r * r) continue;
                const int X = x + dx, Y = y + dy, Z = z + dz;
                if (X < 0 || Y < 0 || Z < 0 || X >= w || Y >= h || Z >= d) continue;
                v = m[(size_t)Z * plane + (size_t)Y * w + X];
              }
          out[(size_t)z * plane + (size_t)y * w + x] = v ? 1 : 0;
        }
    return out;
  }
  // Separable max over x, then y, then z (exact for a cube SE with out-of-volume ignored).
  std::vector<uint8_t> a(m.size()), b(m.size());
  for (int z = 0; z < d; ++z)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        uint8_t v = 0;
        for (int k = std::max(0, x - r); k <= std::min(w - 1, x + r); ++k) v |= m[z * plane + (size_t)y * w + k];
        a[z * plane + (size_t)y * w + x] = v;
      }
  for (int z = 0; z < d; ++z)
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        uint8_t v = 0;
        for (int k = std::max(0, y - r); k <= std::min(h - 1, y + r); ++k) v |= a[z * plane + (size_t)k * w + x];
        b[z * plane + (size_t)y * w + x] = v;
      }
  for (int z = 0; z < d; ++z)
    for (size_t p = 0; p < plane; ++p) {
      uint8_t v = 0;
      for (int k = std::max(0, z - r); k <= std::min(d - 1, z + r); ++k) v |= b[(size_t)k * plane + p];
      a[(size_t)z * plane + p] = v;
    }
  return a;
}

std::vector<uint8_t> render_gray(const std::vector<float>& v, const RenderGeom& g, float lo, float hi, bool nearest) {
  std::vector<uint8_t> out((size_t)g.out_w * g.out_h, 0);
  const float inv = window_inv(lo, hi);
  if (nearest) {
    for (int u = 0; u < g.out_h; ++u) {
      const float sy = render_src_coord(u, g.oy, g.invy);
      if (!(sy >= 0.0f && sy < (float)g.src_h)) continue;
      const int y = clampi((int)std::floor(sy), 0, g.src_h - 1);
      for (int t = 0; t < g.out_w; ++t) {
        const float sx = render_src_coord(t, g.ox, g.invx);
        if (!(sx >= 0.0f && sx < (float)g.src_w)) continue;
        const int x = clampi((int)std::floor(sx), 0, g.src_w - 1);
        out[(size_t)u * g.out_w + t] = gray_u8(v[(size_t)y * g.src_w + x], lo, inv);
      }
    }
    return out;
  }
  for (int u = 0; u < g.out_h; ++u) {
    const float sy = render_src_coord(u, g.oy, g.invy);
    if (!(sy >= 0.0f && sy < (float)g.src_h)) continue;
    const float fy = sy - 0.5f;
    const float y0f = std::floor(fy);
    const float wy = fy - y0f;
    const int y0 = clampi((int)y0f, 0, g.src_h - 1), y1 = clampi((int)y0f + 1, 0, g.src_h - 1);
    for (int t = 0; t < g.out_w; ++t) {
      const float sx = render_src_coord(t, g.ox, g.invx);
      if (!(sx >= 0.0f && sx < (float)g.src_w)) continue;
      const float fx = sx - 0.5f;
      const float x0f = std::floor(fx);
      const float wx = fx - x0f;
      const int x0 = clampi((int)x0f, 0, g.src_w - 1), x1 = clampi((int)x0f + 1, 0, g.src_w - 1);
      const float val = bilerp(v[(size_t)y0 * g.src_w + x0], v[(size_t)y0 * g.src_w + x1], v[(size_t)y1 * g.src_w + x0],
                               v[(size_t)y1 * g.src_w + x1], wx, wy);
      out[(size_t)u * g.out_w + t] = gray_u8(val, lo, inv);
    }
  }
  return out;
}

std::vector<uint8_t> render_labels(const std::vector<uint8_t>& label, const std::vector<uint8_t>& bm, const RenderGeom& g,
                                   uint8_t fill, uint8_t border_value) {
  std::vector<uint8_t> out((size_t)g.out_w * g.out_h, 0);
  for (int u = 0; u < g.out_h; ++u) {
    const float sy = render_src_coord(u, g.oy, g.invy);
    if (!(sy >= 0.0f && sy < (float)g.src_h)) continue;
    const int y = clampi((int)std::floor(sy), 0, g.src_h - 1);
    for (int t = 0; t < g.out_w; ++t) {
      const float sx = render_src_coord(t, g.ox, g.invx);
      if (!(sx >= 0.0f && sx < (float)g.src_w)) continue;
      const int x = clampi((int)std::floor(sx), 0, g.src_w - 1);
      const size_t i = (size_t)y * g.src_w + x;
      out[(size_t)u * g.out_w + t] = bm[i] ? border_value : (label[i] ? fill : 0);
    }
  }
  return out;
}

SliceResult run(const SliceInput& s, const PipelineParams& p, bool with_erosion) {
  SliceResult r;
  r.clipped = norm_clip(s, p);
  r.median = median(r.clipped, s.w, s.h, p.median_window);
  r.sharpened = sharpen(r.median, s.w, s.h, p.sharpen_gain, p.sharpen_sigma, p.sharpen_mask);
  r.band = band(r.sharpened, p.srg_min, p.srg_max);
  r.region = region_grow(r.band, s.w, s.h, reference_seeds(s.w, s.h), p.srg_connectivity);
  const bool disc = p.se_shape == kSeDisc;
  r.dilated = dilate(r.region, s.w, s.h, p.dilation_size, disc);
  if (with_erosion) r.eroded = erode(r.region, s.w, s.h, p.erosion_size, disc);
  std::vector<float> v = rescaled(s, p);
  auto mm = std::minmax_element(v.begin(), v.end());
  r.window_lo = *mm.first;
  r.window_hi = *mm.second;
  return r;
}

SliceJpegs export_jpegs(const SliceInput& s, const SliceResult& r, const PipelineParams& p, const RenderParams& rp) {
  RenderGeom g = make_render_geom(s.w, s.h, s.spacing_x, s.spacing_y, rp.out_width, rp.out_height);
  SliceJpegs j;
  std::vector<uint8_t> c0 = render_gray(rescaled(s, p), g, r.window_lo, r.window_hi, rp.filter == kFilterNearest);
  j.original = jpeg::encode_gray(c0.data(), g.out_w, g.out_h, g.out_w, rp.jpeg_quality, (jpeg::Sampling)rp.jpeg_sampling);
  std::vector<uint8_t> bm = border(r.dilated, s.w, s.h, rp.border_radius);
  std::vector<uint8_t> c1 =
      render_labels(r.dilated, bm, g, opacity_u8(rp.label_opacity), opacity_u8(rp.border_opacity));
  j.processed = jpeg::encode_gray(c1.data(), g.out_w, g.out_h, g.out_w, rp.jpeg_quality, (jpeg::Sampling)rp.jpeg_sampling);
  return j;
}

StageImages test_pipeline_images(const SliceInput& in, const PipelineParams& p, const RenderParams& rp,
                                 SliceResult* stages) {
  StageImages out;
  SliceResult r = run(in, p, true);
  const RenderGeom g = make_render_geom(in.w, in.h, in.spacing_x, in.spacing_y, rp.out_width, rp.out_height);
  const uint8_t fill = opacity_u8(rp.label_opacity), bv = opacity_u8(rp.border_opacity);
  auto mm = std::minmax_element(r.sharpened.begin(), r.sharpened.end());
  auto& c = out.canvases;
  const bool nearest = rp.filter == kFilterNearest;
  c.push_back(render_gray(rescaled(in, p), g, r.window_lo, r.window_hi, nearest));
  c.push_back(render_gray(r.sharpened, g, *mm.first, *mm.second, nearest));
  c.push_back(render_labels(r.region, border(r.region, in.w, in.h, rp.border_radius), g, fill, bv));
  c.push_back(render_labels(r.eroded, border(r.eroded, in.w, in.h, rp.border_radius), g, fill, bv));
  c.push_back(render_labels(r.dilated, border(r.dilated, in.w, in.h, rp.border_radius), g, fill, bv));
  for (auto& cv : c) out.jpegs.push_back(jpeg::encode_gray(cv.data(), rp.out_width, rp.out_height, rp.out_width,
                                                            rp.jpeg_quality, (jpeg::Sampling)rp.jpeg_sampling));
  if (stages) *stages = std::move(r);
  return out;
}

}  // namespace nm03::golden
