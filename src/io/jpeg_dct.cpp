// Sequential DCT JPEG, Huffman coding, one component (nm03/jpeg_dct.h), from ITU T.81: markers
// (Annex B), sequential Huffman decoding (F.2.2), and the IJG library's integer "islow" inverse DCT
// (the LL&M algorithm as jidctint.c computes it, with jdmaster.c's range-limit table) so that 8-bit
// output is byte-identical to libjpeg's. This software is based in part on the work of the
// Independent JPEG Group.
#include "nm03/jpeg_dct.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "jpeg_entropy.h"
#include "nm03/common.h"
#include "nm03/jpeg_common.h"

namespace nm03::jpegdct {

using namespace jpeg_entropy;

namespace {

// islow constants (CONST_BITS = 13): FIX(x) = round(x · 2^13).
constexpr int kConstBits = 13;
constexpr int64_t F0_298631336 = 2446, F0_390180644 = 3196, F0_541196100 = 4433, F0_765366865 = 6270,
                  F0_899976223 = 7373, F1_175875602 = 9633, F1_501321110 = 12299, F1_847759065 = 15137,
                  F1_961570560 = 16069, F2_053119869 = 16819, F2_562915447 = 20995, F3_072711026 = 25172;

inline int64_t descale(int64_t x, int n) { return (x + (int64_t(1) << (n - 1))) >> n; }

// The post-IDCT range limit of jdmaster.c (prepare_range_limit_table), indexed by the centred
// value & RANGE_MASK: a clamp to [0, MAXJSAMPLE] for values within ±2·(MAXJSAMPLE + 1).
struct RangeLimit {
  int maxj, center, mask;
  std::vector<uint16_t> post;  // post[v & mask] = output sample of centred value v
  explicit RangeLimit(int precision) : maxj((1 << precision) - 1), center(1 << (precision - 1)), mask(4 * (1 << precision) - 1) {
    const int n = maxj + 1;
    post.assign((size_t)4 * n, 0);
    for (int i = 0; i < n - center; ++i) post[(size_t)i] = (uint16_t)(center + i);
    for (int i = n - center; i < 2 * n; ++i) post[(size_t)i] = (uint16_t)maxj;
    for (int i = 2 * n; i < 4 * n - center; ++i) post[(size_t)i] = 0;
    for (int i = 4 * n - center; i < 4 * n; ++i) post[(size_t)i] = (uint16_t)(i - (4 * n - center));
  }
};

// jidctint.c jpeg_idct_islow: dequantise + 2-D inverse DCT of one block into out (stride `ostride`).
void idct_islow(const int32_t* coef, const uint16_t* q, int pass1_bits, const RangeLimit& rl, uint16_t* out,
                size_t ostride) {
  int64_t ws[64];
  for (int c = 0; c < 8; ++c) {  // pass 1: columns
    const int32_t* in = coef + c;
    const uint16_t* qc = q + c;
    if (!in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56]) {
      const int64_t dc = (int64_t)in[0] * qc[0] * (int64_t(1) << pass1_bits);
      for (int k = 0; k < 8; ++k) ws[c + 8 * k] = dc;
      continue;
    }
    int64_t z2 = (int64_t)in[16] * qc[16], z3 = (int64_t)in[48] * qc[48];
    int64_t z1 = (z2 + z3) * F0_541196100;
    int64_t tmp2 = z1 + z3 * -F1_847759065;
    int64_t tmp3 = z1 + z2 * F0_765366865;
    z2 = (int64_t)in[0] * qc[0];
    z3 = (int64_t)in[32] * qc[32];
    int64_t tmp0 = (z2 + z3) * (int64_t(1) << kConstBits);
    int64_t tmp1 = (z2 - z3) * (int64_t(1) << kConstBits);
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = (int64_t)in[56] * qc[56];
    tmp1 = (int64_t)in[40] * qc[40];
    tmp2 = (int64_t)in[24] * qc[24];
    tmp3 = (int64_t)in[8] * qc[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1_175875602;
    tmp0 *= F0_298631336;
    tmp1 *= F2_053119869;
    tmp2 *= F3_072711026;
    tmp3 *= F1_501321110;
    z1 *= -F0_899976223;
    z2 *= -F2_562915447;
    z3 *= -F1_961570560;
    z4 *= -F0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    const int sh = kConstBits - pass1_bits;
    ws[c + 0] = descale(tmp10 + tmp3, sh);
    ws[c + 56] = descale(tmp10 - tmp3, sh);
    ws[c + 8] = descale(tmp11 + tmp2, sh);
    ws[c + 48] = descale(tmp11 - tmp2, sh);
    ws[c + 16] = descale(tmp12 + tmp1, sh);
    ws[c + 40] = descale(tmp12 - tmp1, sh);
    ws[c + 24] = descale(tmp13 + tmp0, sh);
    ws[c + 32] = descale(tmp13 - tmp0, sh);
  }
  const int sh2 = kConstBits + pass1_bits + 3;
  for (int r = 0; r < 8; ++r) {  // pass 2: rows
    const int64_t* w = ws + 8 * r;
    uint16_t* o = out + (size_t)r * ostride;
    if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
      const uint16_t v = rl.post[(size_t)(descale(w[0], pass1_bits + 3) & rl.mask)];
      for (int k = 0; k < 8; ++k) o[k] = v;
      continue;
    }
    int64_t z2 = w[2], z3 = w[6];
    int64_t z1 = (z2 + z3) * F0_541196100;
    int64_t tmp2 = z1 + z3 * -F1_847759065;
    int64_t tmp3 = z1 + z2 * F0_765366865;
    int64_t tmp0 = (w[0] + w[4]) * (int64_t(1) << kConstBits);
    int64_t tmp1 = (w[0] - w[4]) * (int64_t(1) << kConstBits);
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
    tmp0 = w[7];
    tmp1 = w[5];
    tmp2 = w[3];
    tmp3 = w[1];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * F1_175875602;
    tmp0 *= F0_298631336;
    tmp1 *= F2_053119869;
    tmp2 *= F3_072711026;
    tmp3 *= F1_501321110;
    z1 *= -F0_899976223;
    z2 *= -F2_562915447;
    z3 *= -F1_961570560;
    z4 *= -F0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    auto put = [&](int k, int64_t v) { o[k] = rl.post[(size_t)(descale(v, sh2) & rl.mask)]; };
    put(0, tmp10 + tmp3);
    put(7, tmp10 - tmp3);
    put(1, tmp11 + tmp2);
    put(6, tmp11 - tmp2);
    put(2, tmp12 + tmp1);
    put(5, tmp12 - tmp1);
    put(3, tmp13 + tmp0);
    put(4, tmp13 - tmp0);
  }
}

inline int32_t extend(uint32_t v, int s) {
  return s == 0 ? 0 : (v < (1u << (s - 1)) ? (int32_t)v - (int32_t)(1u << s) + 1 : (int32_t)v);
}

}  // namespace

Info decode(const uint8_t* d, size_t n, std::vector<uint16_t>& out, int expect_rows, int expect_cols) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) throw SliceError("JPEG: missing SOI marker");
  size_t pos = 2;
  Info info;
  Table dc[4], ac[4];
  uint16_t qt[4][64];
  bool qdef[4] = {false, false, false, false};
  bool have_sof = false;
  int comp_id = -1, tq = 0;
  for (;;) {
    while (pos < n && d[pos] != 0xFF) ++pos;
    while (pos + 1 < n && d[pos + 1] == 0xFF) ++pos;
    if (pos + 1 >= n) throw SliceError("JPEG: no scan before the end of the data");
    const uint8_t m = d[pos + 1];
    pos += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;
    if (m == 0xD9) throw SliceError("JPEG: EOI before any scan");
    if (pos + 2 > n) throw SliceError("Truncated JPEG marker segment");
    const size_t len = be16(d + pos);
    if (len < 2 || pos + len > n) throw SliceError("Truncated JPEG marker segment");
    const uint8_t* s = d + pos + 2;
    const size_t sl = len - 2;
    if (m == 0xC0 || m == 0xC1) {  // SOF0 baseline / SOF1 extended sequential, Huffman
      if (sl < 6) throw SliceError("JPEG: short SOF");
      info.sof = m - 0xC0;
      info.precision = s[0];
      info.rows = be16(s + 1);
      info.cols = be16(s + 3);
      const int nf = s[5];
      if (info.precision != 8 && info.precision != 12) throw SliceError("JPEG: sample precision must be 8 or 12");
      if (m == 0xC0 && info.precision != 8) throw SliceError("JPEG: baseline with 12-bit samples");
      if (info.rows == 0 || info.cols == 0) throw SliceError("JPEG: zero image size (DNL not supported)");
      if (nf != 1) throw SliceError("JPEG with " + std::to_string(nf) + " components (monochrome supported)");
      if ((expect_rows > 0 && info.rows != expect_rows) || (expect_cols > 0 && info.cols != expect_cols))
        throw SliceError("JPEG frame is " + std::to_string(info.cols) + "x" + std::to_string(info.rows) + ", expected " +
                         std::to_string(expect_cols) + "x" + std::to_string(expect_rows));
      if (sl < 9) throw SliceError("JPEG: short SOF");
      comp_id = s[6];
      tq = s[8];
      if (tq > 3) throw SliceError("JPEG: bad quantisation table id");
      have_sof = true;
    } else if (m == 0xC3) {
      throw SliceError("JPEG: lossless process (decoded by the lossless codec, not here)");
    } else if ((m >= 0xC0 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      throw SliceError("Unsupported JPEG process (SOF" + std::to_string(m - 0xC0) + "): sequential Huffman DCT only");
    } else if (m == 0xCC) {
      throw SliceError("Unsupported JPEG process: arithmetic coding");
    } else if (m == 0xDB) {  // DQT
      size_t q = 0;
      while (q < sl) {
        const int pq = s[q] >> 4, id = s[q] & 15;
        const size_t need = 1 + (pq ? 128 : 64);
        if (id > 3 || pq > 1 || q + need > sl) throw SliceError("JPEG: malformed DQT");
        for (int k = 0; k < 64; ++k)
          qt[id][jpeg::kNatural[k]] = pq ? be16(s + q + 1 + 2 * k) : s[q + 1 + k];
        qdef[id] = true;
        q += need;
      }
    } else if (m == 0xC4) {  // DHT
      size_t q = 0;
      while (q < sl) {
        const int tc = s[q] >> 4, th = s[q] & 15;
        if (tc > 1 || th > 3 || q + 17 > sl) throw SliceError("JPEG: malformed DHT");
        Table t;
        int total = 0;
        for (int l = 1; l <= 16; ++l) total += (t.bits[l] = s[q + l]);
        if (total > 256 || q + 17 + (size_t)total > sl) throw SliceError("JPEG: malformed DHT");
        std::memcpy(t.vals, s + q + 17, (size_t)total);
        t.nvals = total;
        t.build();
        t.defined = true;
        (tc == 0 ? dc : ac)[th] = t;
        q += 17 + (size_t)total;
      }
    } else if (m == 0xDD) {
      if (sl < 2) throw SliceError("JPEG: short DRI");
      info.restart_interval = be16(s);
    } else if (m == 0xDA) {  // SOS
      if (!have_sof) throw SliceError("JPEG: scan before SOF");
      if (sl < 6 || s[0] != 1) throw SliceError("JPEG: scan must have one component");
      if (s[1] != comp_id) throw SliceError("JPEG: scan component not in the frame");
      const int td = s[2] >> 4, ta = s[2] & 15;
      if (s[3] != 0 || s[4] != 63 || s[5] != 0) throw SliceError("JPEG: not a sequential scan");
      if (td > 3 || ta > 3 || !dc[td].defined || !ac[ta].defined) throw SliceError("JPEG: scan uses an undefined Huffman table");
      if (!qdef[tq]) throw SliceError("JPEG: undefined quantisation table");
      const int bw = (info.cols + 7) / 8, bh = (info.rows + 7) / 8;
      const size_t nblocks = (size_t)bw * bh;
      const size_t avail = n - (pos + len);
      if (nblocks > avail * 4 + 64) throw SliceError("Truncated JPEG data");  // ≥ 2 bits (DC, EOB) per block
      out.assign((size_t)info.rows * info.cols, 0);
      const int pass1 = info.precision == 8 ? 2 : 1;
      const RangeLimit rl(info.precision);
      const int max_cat = info.precision == 8 ? 11 : 15;
      BitReader br(d, n, pos + len);
      int32_t pred = 0;
      int32_t coef[64];
      uint16_t blk[64];
      int rst = 0;
      for (size_t b = 0; b < nblocks; ++b) {
        if (info.restart_interval && b > 0 && b % (size_t)info.restart_interval == 0) {
          br.restart(rst++ & 7);
          pred = 0;
        }
        std::memset(coef, 0, sizeof(coef));
        const int cs = decode_symbol(dc[td], br);
        if (cs > max_cat) throw SliceError("Corrupt JPEG: DC category out of range");
        pred = (int32_t)((uint32_t)pred + (uint32_t)extend(br.get(cs), cs));  // wraps on corrupt data (no UB)
        coef[0] = pred;
        for (int k = 1; k < 64; ++k) {
          const int rs = decode_symbol(ac[ta], br);
          const int r = rs >> 4, sz = rs & 15;
          if (sz == 0) {
            if (r != 15) break;  // EOB
            k += 15;             // ZRL
            continue;
          }
          k += r;
          if (k > 63) throw SliceError("Corrupt JPEG: AC run past the block");
          coef[jpeg::kNatural[k]] = extend(br.get(sz), sz);
        }
        idct_islow(coef, qt[tq], pass1, rl, blk, 8);
        const int bx = (int)(b % (size_t)bw), by = (int)(b / (size_t)bw);
        const int x0 = bx * 8, y0 = by * 8;
        const int cw = std::min(8, info.cols - x0), ch = std::min(8, info.rows - y0);
        for (int y = 0; y < ch; ++y) std::memcpy(out.data() + (size_t)(y0 + y) * info.cols + x0, blk + 8 * y, (size_t)cw * 2);
      }
      br.finish();
      return info;
    }
    pos += len;
  }
}

std::vector<uint8_t> encode(const uint16_t* px, int rows, int cols, int precision, int quality, int restart_blocks) {
  if (rows < 1 || cols < 1 || rows > 65535 || cols > 65535) throw SliceError("JPEG: bad image size");
  if (precision != 8 && precision != 12) throw SliceError("JPEG: precision must be 8 or 12");
  if (restart_blocks < 0 || restart_blocks > 65535) throw SliceError("JPEG: bad restart interval");
  uint16_t q[64];  // natural order
  jpeg::quality_table(jpeg::kStdLuma, quality, q);
  const int bw = (cols + 7) / 8, bh = (rows + 7) / 8;
  const size_t nblocks = (size_t)bw * bh;
  const int center = 1 << (precision - 1), maxv = (1 << precision) - 1;
  // Pass 1: quantised coefficients (floating-point FDCT; edge blocks replicate the last row/column).
  std::vector<int32_t> coefs(nblocks * 64);
  double cosv[8][8];
  for (int x = 0; x < 8; ++x)
    for (int u = 0; u < 8; ++u) cosv[x][u] = std::cos((2 * x + 1) * u * M_PI / 16.0);
  for (size_t b = 0; b < nblocks; ++b) {
    const int x0 = (int)(b % (size_t)bw) * 8, y0 = (int)(b / (size_t)bw) * 8;
    double f[8][8];
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        const int yy = std::min(rows - 1, y0 + y), xx = std::min(cols - 1, x0 + x);
        f[y][x] = (double)std::min<int>(px[(size_t)yy * cols + xx], maxv) - center;
      }
    for (int v = 0; v < 8; ++v)
      for (int u = 0; u < 8; ++u) {
        double acc = 0;
        for (int y = 0; y < 8; ++y)
          for (int x = 0; x < 8; ++x) acc += f[y][x] * cosv[x][u] * cosv[y][v];
        const double cu = u ? 1.0 : M_SQRT1_2, cv = v ? 1.0 : M_SQRT1_2;
        coefs[b * 64 + (size_t)v * 8 + u] = (int32_t)std::lround(0.25 * cu * cv * acc / q[v * 8 + u]);
      }
  }
  // Pass 2: symbol statistics → optimal tables (K.2).
  uint64_t fdc[256] = {0}, fac[256] = {0};
  auto cat = [](int32_t v) { return v ? 32 - __builtin_clz((uint32_t)(v < 0 ? -v : v)) : 0; };
  auto scan = [&](auto&& dc_sym, auto&& ac_sym) {
    int32_t pred = 0;
    for (size_t b = 0; b < nblocks; ++b) {
      if (restart_blocks && b > 0 && b % (size_t)restart_blocks == 0) pred = 0;
      const int32_t* c = coefs.data() + b * 64;
      dc_sym(b, c[0] - pred);
      pred = c[0];
      int run = 0;
      for (int k = 1; k < 64; ++k) {
        const int32_t v = c[jpeg::kNatural[k]];
        if (!v) {
          ++run;
          continue;
        }
        while (run > 15) {
          ac_sym(0xF0, 0);
          run -= 16;
        }
        ac_sym((run << 4) | cat(v), v);
        run = 0;
      }
      if (run) ac_sym(0x00, 0);
    }
  };
  scan([&](size_t, int32_t d) { ++fdc[cat(d)]; }, [&](int rs, int32_t) { ++fac[rs]; });
  Table tdc, tac;
  optimal_table(fdc, tdc);
  optimal_table(fac, tac);
  std::vector<uint8_t> o = {0xFF, 0xD8};
  auto seg = [&](uint8_t m, const std::vector<uint8_t>& body) {
    o.push_back(0xFF);
    o.push_back(m);
    o.push_back((uint8_t)((body.size() + 2) >> 8));
    o.push_back((uint8_t)(body.size() + 2));
    o.insert(o.end(), body.begin(), body.end());
  };
  {
    std::vector<uint8_t> dqt = {0x00};
    for (int k = 0; k < 64; ++k) dqt.push_back((uint8_t)q[jpeg::kNatural[k]]);
    seg(0xDB, dqt);
  }
  seg(precision == 8 ? 0xC0 : 0xC1,
      {(uint8_t)precision, (uint8_t)(rows >> 8), (uint8_t)rows, (uint8_t)(cols >> 8), (uint8_t)cols, 1, 1, 0x11, 0});
  for (int tc = 0; tc < 2; ++tc) {
    const Table& t = tc ? tac : tdc;
    std::vector<uint8_t> dht = {(uint8_t)(tc << 4)};
    for (int l = 1; l <= 16; ++l) dht.push_back(t.bits[l]);
    dht.insert(dht.end(), t.vals, t.vals + t.nvals);
    seg(0xC4, dht);
  }
  if (restart_blocks) seg(0xDD, {(uint8_t)(restart_blocks >> 8), (uint8_t)restart_blocks});
  seg(0xDA, {1, 1, 0x00, 0, 63, 0});
  BitWriter bw_(o);
  size_t last_rst_block = 0;
  int rst = 0;
  scan(
      [&](size_t b, int32_t d) {
        if (restart_blocks && b > 0 && b % (size_t)restart_blocks == 0 && b != last_rst_block) {
          bw_.flush_ones();
          o.push_back(0xFF);
          o.push_back((uint8_t)(0xD0 + (rst++ & 7)));
          last_rst_block = b;
        }
        const int c = cat(d);
        bw_.put(tdc.code_of[c], tdc.size_of[c]);
        if (c) bw_.put((uint32_t)(d < 0 ? d - 1 : d) & ((1u << c) - 1), c);
      },
      [&](int rs, int32_t v) {
        bw_.put(tac.code_of[rs], tac.size_of[rs]);
        const int c = rs & 15;
        if (c) bw_.put((uint32_t)(v < 0 ? v - 1 : v) & ((1u << c) - 1), c);
      });
  bw_.flush_ones();
  o.push_back(0xFF);
  o.push_back(0xD9);
  return o;
}

}  // namespace nm03::jpegdct
