// Lossless JPEG, process 14 (nm03/jpeg_lossless.h), from ITU T.81: markers (Annex B), Huffman
// table specification and canonical codes (Annex C), decoding procedure (F.2.2.3), lossless
// predictors and modulo-2^16 differences (Annex H), optimal table generation (Annex K.2).
#include "nm03/jpeg_lossless.h"

#include <algorithm>
#include <cstring>
#include <string>

#include "jpeg_entropy.h"
#include "nm03/common.h"

namespace nm03::jpegll {

using namespace jpeg_entropy;

namespace {

// Prediction (H.1.2.1): first line of the image or of a restart interval — 2^(P−Pt−1) for its first
// sample, then Ra; first sample of any other line — Rb; otherwise selection value sv.
inline int32_t predict(int sv, bool first_line, int x, const uint16_t* cur, const uint16_t* prev, int32_t p0) {
  if (first_line) return x == 0 ? p0 : cur[x - 1];
  if (x == 0) return prev[0];
  const int32_t ra = cur[x - 1], rb = prev[x], rc = prev[x - 1];
  switch (sv) {
    case 1: return ra;
    case 2: return rb;
    case 3: return rc;
    case 4: return ra + rb - rc;
    case 5: return ra + ((rb - rc) >> 1);
    case 6: return rb + ((ra - rc) >> 1);
    default: return (ra + rb) >> 1;
  }
}


}  // namespace

Info decode(const uint8_t* d, size_t n, std::vector<uint16_t>& out, int expect_rows, int expect_cols) {
  if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) throw SliceError("Lossless JPEG: missing SOI marker");
  size_t pos = 2;
  Info info;
  Table tables[4];
  bool have_sof = false;
  int comp_id = -1;
  for (;;) {
    while (pos < n && d[pos] != 0xFF) ++pos;  // tolerate garbage between segments
    while (pos + 1 < n && d[pos + 1] == 0xFF) ++pos;
    if (pos + 1 >= n) throw SliceError("Lossless JPEG: no scan before the end of the data");
    const uint8_t m = d[pos + 1];
    pos += 2;
    if (m == 0xD8 || m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // no length
    if (m == 0xD9) throw SliceError("Lossless JPEG: EOI before any scan");
    if (pos + 2 > n) throw SliceError("Truncated lossless JPEG marker segment");
    const size_t len = be16(d + pos);
    if (len < 2 || pos + len > n) throw SliceError("Truncated lossless JPEG marker segment");
    const uint8_t* s = d + pos + 2;
    const size_t sl = len - 2;
    if (m == 0xC3) {  // SOF3: lossless, Huffman
      if (sl < 6) throw SliceError("Lossless JPEG: short SOF3");
      info.precision = s[0];
      info.rows = be16(s + 1);
      info.cols = be16(s + 3);
      const int nf = s[5];
      if (info.precision < 2 || info.precision > 16) throw SliceError("Lossless JPEG: precision out of range");
      if (info.rows == 0) throw SliceError("Lossless JPEG: height given by DNL is not supported");
      if (info.cols == 0) throw SliceError("Lossless JPEG: zero width");
      if (nf != 1) throw SliceError("Lossless JPEG with " + std::to_string(nf) + " components (one is supported)");
      if ((expect_rows > 0 && info.rows != expect_rows) || (expect_cols > 0 && info.cols != expect_cols))
        throw SliceError("JPEG frame is " + std::to_string(info.cols) + "x" + std::to_string(info.rows) + ", expected " +
                         std::to_string(expect_cols) + "x" + std::to_string(expect_rows));
      if (sl < 9) throw SliceError("Lossless JPEG: short SOF3");
      comp_id = s[6];
      if (s[7] != 0x11) throw SliceError("Lossless JPEG: subsampled component");
      have_sof = true;
    } else if ((m >= 0xC0 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      throw SliceError("Unsupported JPEG process (SOF" + std::to_string(m - 0xC0) + "): only lossless SOF3 is decoded");
    } else if (m == 0xC4) {  // DHT
      size_t q = 0;
      while (q < sl) {
        const int tc = s[q] >> 4, th = s[q] & 15;
        if (th > 3 || q + 17 > sl) throw SliceError("Lossless JPEG: malformed DHT");
        Table t;
        int total = 0;
        for (int l = 1; l <= 16; ++l) total += (t.bits[l] = s[q + l]);
        if (total > 256 || q + 17 + (size_t)total > sl) throw SliceError("Lossless JPEG: malformed DHT");
        std::memcpy(t.vals, s + q + 17, (size_t)total);
        t.nvals = total;
        for (int i = 0; i < total; ++i)
          if (t.vals[i] > 16 && tc == 0) throw SliceError("Lossless JPEG: difference category above 16");
        if (tc == 0) {
          t.build();
          t.defined = true;
          tables[th] = t;
        }
        q += 17 + (size_t)total;
      }
    } else if (m == 0xDD) {  // DRI
      if (sl < 2) throw SliceError("Lossless JPEG: short DRI");
      info.restart_interval = be16(s);
    } else if (m == 0xCC) {
      throw SliceError("Unsupported JPEG process: arithmetic coding");
    } else if (m == 0xDA) {  // SOS
      if (!have_sof) throw SliceError("Lossless JPEG: scan before SOF3");
      if (sl < 6 || s[0] != 1) throw SliceError("Lossless JPEG: scan must have one component");
      if (s[1] != comp_id) throw SliceError("Lossless JPEG: scan component not in the frame");
      const int td = s[2] >> 4;
      const int ss = s[3], ah_al = s[5];
      info.predictor = ss;
      info.point_transform = ah_al & 15;
      if (ss < 1 || ss > 7) throw SliceError("Lossless JPEG: selection value " + std::to_string(ss) + " (1..7 supported)");
      if (td > 3 || !tables[td].defined) throw SliceError("Lossless JPEG: scan uses an undefined Huffman table");
      if (info.point_transform >= info.precision) throw SliceError("Lossless JPEG: point transform ≥ precision");
      if (info.restart_interval && info.restart_interval % info.cols)
        throw SliceError("Lossless JPEG: restart interval of " + std::to_string(info.restart_interval) +
                         " samples does not span whole rows (unsupported)");
      const size_t npx = (size_t)info.rows * info.cols;
      // Every sample takes at least one bit: a stream shorter than that is truncated (checked before
      // allocating the image).
      const size_t avail = n - (pos + len);
      if (npx > avail * 8 + 64) throw SliceError("Truncated lossless JPEG data");
      out.assign(npx, 0);
      const Table& t = tables[td];
      const int pt = info.point_transform;
      const int32_t p0 = 1 << (info.precision - pt - 1);
      const int rows_per_interval = info.restart_interval ? info.restart_interval / info.cols : info.rows;
      BitReader br(d, n, pos + len);
      std::vector<uint16_t> line[2] = {std::vector<uint16_t>((size_t)info.cols), std::vector<uint16_t>((size_t)info.cols)};
      int rst = 0;
      for (int y = 0; y < info.rows; ++y) {
        const bool first_line = y % rows_per_interval == 0;
        if (first_line && y > 0) br.restart(rst++ & 7);
        uint16_t* cur = line[y & 1].data();
        const uint16_t* prev = line[(y + 1) & 1].data();
        uint16_t* o = out.data() + (size_t)y * info.cols;
        for (int x = 0; x < info.cols; ++x) {
          const int cat = decode_symbol(t, br);
          int32_t diff;
          if (cat == 0)
            diff = 0;
          else if (cat == 16)
            diff = 32768;
          else {
            const int32_t v = (int32_t)br.get(cat);
            diff = v < (1 << (cat - 1)) ? v - (1 << cat) + 1 : v;
          }
          const uint16_t r = (uint16_t)((predict(ss, first_line, x, cur, prev, p0) + diff) & 0xFFFF);
          cur[x] = r;
          o[x] = (uint16_t)(r << pt);
        }
      }
      br.finish();
      return info;
    }
    pos += len;
  }
}

std::vector<uint8_t> encode(const uint16_t* px, int rows, int cols, int precision, int predictor, int pt, int restart_rows) {
  if (rows < 1 || cols < 1 || rows > 65535 || cols > 65535) throw SliceError("lossless JPEG: bad image size");
  if (precision < 2 || precision > 16) throw SliceError("lossless JPEG: precision must be 2..16");
  if (predictor < 1 || predictor > 7) throw SliceError("lossless JPEG: predictor must be 1..7");
  if (pt < 0 || pt >= precision) throw SliceError("lossless JPEG: bad point transform");
  if (restart_rows < 0 || (int64_t)restart_rows * cols > 65535) throw SliceError("lossless JPEG: restart interval too long");
  const uint32_t mask = precision == 16 ? 0xFFFFu : (1u << precision) - 1;
  const int32_t p0 = 1 << (precision - pt - 1);
  const int rpi = restart_rows > 0 ? restart_rows : rows;
  // Pass 1: difference categories (and the differences) in scan order.
  std::vector<uint8_t> cats((size_t)rows * cols);
  std::vector<int32_t> diffs((size_t)rows * cols);
  std::vector<uint16_t> line[2] = {std::vector<uint16_t>((size_t)cols), std::vector<uint16_t>((size_t)cols)};
  uint64_t freq[256] = {0};
  for (int y = 0; y < rows; ++y) {
    const bool first_line = y % rpi == 0;
    uint16_t* cur = line[y & 1].data();
    const uint16_t* prev = line[(y + 1) & 1].data();
    for (int x = 0; x < cols; ++x) {
      const uint16_t v = (uint16_t)((px[(size_t)y * cols + x] & mask) >> pt);
      cur[x] = v;
      const uint32_t d16 = (uint32_t)(v - predict(predictor, first_line, x, cur, prev, p0)) & 0xFFFFu;
      int cat;
      int32_t d = 0;
      if (d16 == 0x8000u) {
        cat = 16;
      } else {
        d = d16 >= 0x8000u ? (int32_t)d16 - 0x10000 : (int32_t)d16;
        const uint32_t a = (uint32_t)(d < 0 ? -d : d);
        cat = a ? 32 - __builtin_clz(a) : 0;
      }
      cats[(size_t)y * cols + x] = (uint8_t)cat;
      diffs[(size_t)y * cols + x] = d;
      ++freq[cat];
    }
  }
  Table t;
  optimal_table(freq, t);
  std::vector<uint8_t> o = {0xFF, 0xD8};
  auto seg = [&](uint8_t m, const std::vector<uint8_t>& body) {
    o.push_back(0xFF);
    o.push_back(m);
    o.push_back((uint8_t)((body.size() + 2) >> 8));
    o.push_back((uint8_t)(body.size() + 2));
    o.insert(o.end(), body.begin(), body.end());
  };
  seg(0xC3, {(uint8_t)precision, (uint8_t)(rows >> 8), (uint8_t)rows, (uint8_t)(cols >> 8), (uint8_t)cols, 1, 1, 0x11, 0});
  {
    std::vector<uint8_t> dht = {0x00};
    for (int l = 1; l <= 16; ++l) dht.push_back(t.bits[l]);
    dht.insert(dht.end(), t.vals, t.vals + t.nvals);
    seg(0xC4, dht);
  }
  if (restart_rows > 0 && restart_rows < rows) {
    const int ri = restart_rows * cols;
    seg(0xDD, {(uint8_t)(ri >> 8), (uint8_t)ri});
  }
  seg(0xDA, {1, 1, 0x00, (uint8_t)predictor, 0, (uint8_t)pt});
  BitWriter bw(o);
  int rst = 0;
  for (int y = 0; y < rows; ++y) {
    if (y > 0 && y % rpi == 0) {
      bw.flush_ones();
      o.push_back(0xFF);
      o.push_back((uint8_t)(0xD0 + (rst++ & 7)));
    }
    for (int x = 0; x < cols; ++x) {
      const int cat = cats[(size_t)y * cols + x];
      bw.put(t.code_of[cat], t.size_of[cat]);
      if (cat && cat < 16) {
        const int32_t d = diffs[(size_t)y * cols + x];
        bw.put((uint32_t)(d < 0 ? d - 1 : d) & ((1u << cat) - 1), cat);
      }
    }
  }
  bw.flush_ones();
  o.push_back(0xFF);
  o.push_back(0xD9);
  return o;
}

}  // namespace nm03::jpegll
