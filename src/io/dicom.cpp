// DICOM Part-10 reader/writer. Replaces DCMTK behind FAST's DICOMFileImporter
// (reference call sites: test_pipeline.cpp:33-42, main_sequential.cpp:175-177,
// main_parallel.cpp:78-80). Only what a 2D monochrome slice import needs is interpreted; every
// other element is skipped structurally (including undefined-length sequences).
#include "nm03/dicom.h"
#include "nm03/jpeg_dct.h"
#include "nm03/jpeg_lossless.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>

namespace nm03::dicom {
namespace {

constexpr uint32_t kUndefined = 0xFFFFFFFFu;

struct Cursor {
  const uint8_t* d;
  size_t n;
  size_t pos;
  bool big;  // big-endian element encoding

  bool has(size_t k) const { return pos + k <= n; }
  void need(size_t k) const {
    if (!has(k)) throw SliceError("Truncated DICOM data");
  }
  uint16_t u16() {
    need(2);
    uint16_t v = big ? (uint16_t)((d[pos] << 8) | d[pos + 1]) : (uint16_t)(d[pos] | (d[pos + 1] << 8));
    pos += 2;
    return v;
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    if (big)
      v = ((uint32_t)d[pos] << 24) | ((uint32_t)d[pos + 1] << 16) | ((uint32_t)d[pos + 2] << 8) | d[pos + 3];
    else
      v = (uint32_t)d[pos] | ((uint32_t)d[pos + 1] << 8) | ((uint32_t)d[pos + 2] << 16) | ((uint32_t)d[pos + 3] << 24);
    pos += 4;
    return v;
  }
};

bool long_length_vr(const char* vr) {
  static const char* kLong[] = {"OB", "OD", "OF", "OL", "OV", "OW", "SQ", "SV", "UC", "UN", "UR", "UT", "UV"};
  for (const char* v : kLong)
    if (vr[0] == v[0] && vr[1] == v[1]) return true;
  return false;
}

struct Elem {
  uint16_t group, elem;
  char vr[3];
  uint32_t len;
  size_t value_pos;
};

// Reads one element header; explicit==false → implicit VR.
Elem read_elem(Cursor& c, bool explicit_vr) {
  Elem e{};
  e.group = c.u16();
  e.elem = c.u16();
  e.vr[0] = e.vr[1] = e.vr[2] = 0;
  if (e.group == 0xFFFE) {  // item / delimiters never carry a VR
    e.len = c.u32();
  } else if (explicit_vr) {
    c.need(2);
    e.vr[0] = (char)c.d[c.pos];
    e.vr[1] = (char)c.d[c.pos + 1];
    c.pos += 2;
    if (long_length_vr(e.vr)) {
      c.need(2);
      c.pos += 2;
      e.len = c.u32();
    } else {
      e.len = c.u16();
    }
  } else {
    e.len = c.u32();
  }
  e.value_pos = c.pos;
  return e;
}

void skip_sequence(Cursor& c, bool explicit_vr, int depth);

// Skip a dataset nested in an undefined-length item until the item delimiter.
void skip_item_dataset(Cursor& c, bool explicit_vr, int depth) {
  while (c.has(8)) {
    Elem e = read_elem(c, explicit_vr);
    if (e.group == 0xFFFE && e.elem == 0xE00D) return;  // item delimitation
    if (e.len == kUndefined) {
      skip_sequence(c, explicit_vr, depth + 1);
    } else {
      c.need(e.len);
      c.pos += e.len;
    }
  }
  throw SliceError("Unterminated DICOM item");
}

void skip_sequence(Cursor& c, bool explicit_vr, int depth) {
  if (depth > 64) throw SliceError("DICOM sequence nesting too deep");
  while (c.has(8)) {
    Elem e = read_elem(c, explicit_vr);
    if (e.group == 0xFFFE && e.elem == 0xE0DD) return;  // sequence delimitation
    if (e.group == 0xFFFE && e.elem == 0xE000) {
      if (e.len == kUndefined)
        skip_item_dataset(c, explicit_vr, depth);
      else {
        c.need(e.len);
        c.pos += e.len;
      }
      continue;
    }
    throw SliceError("Malformed DICOM sequence");
  }
  throw SliceError("Unterminated DICOM sequence");
}

std::string str_value(const Cursor& c, const Elem& e) {
  std::string s((const char*)c.d + e.value_pos, e.len);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\0')) s.pop_back();
  size_t b = 0;
  while (b < s.size() && s[b] == ' ') ++b;
  return s.substr(b);
}

std::vector<double> ds_values(const std::string& s) {
  std::vector<double> out;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('\\', i);
    if (j == std::string::npos) j = s.size();
    std::string part = s.substr(i, j - i);
    if (!part.empty()) out.push_back(std::strtod(part.c_str(), nullptr));
    i = j + 1;
  }
  return out;
}

uint16_t us_value(const Cursor& c, const Elem& e) {
  if (e.len < 2) throw SliceError("Bad US element");
  const uint8_t* p = c.d + e.value_pos;
  return c.big ? (uint16_t)((p[0] << 8) | p[1]) : (uint16_t)(p[0] | (p[1] << 8));
}

// Largest inflated dataset accepted (DICOM element lengths are 32-bit; a 2 GiB dataset is far
// beyond any slice or series file): a small crafted stream cannot make the reader allocate more.
constexpr size_t kMaxInflated = size_t(1) << 31;

// Raw deflate stream (RFC 1951, no zlib header: PS3.5 A.5) → bytes.
std::vector<uint8_t> inflate_raw(const uint8_t* src, size_t n) {
  if (n > 0xFFFFFFFFu) throw SliceError("Deflated DICOM dataset too large");
  z_stream z{};
  if (inflateInit2(&z, -MAX_WBITS) != Z_OK) throw SliceError("zlib inflateInit failed");
  std::vector<uint8_t> out(std::max<size_t>(n * 4, 1 << 16));
  z.next_in = const_cast<Bytef*>(src);
  z.avail_in = (uInt)n;
  size_t have = 0;
  int r = Z_OK;
  while (r != Z_STREAM_END) {
    if (have == out.size()) {
      if (out.size() >= kMaxInflated) {
        inflateEnd(&z);
        throw SliceError("Deflated DICOM dataset inflates beyond 2 GiB");
      }
      out.resize(std::min(out.size() * 2, kMaxInflated));
    }
    z.next_out = out.data() + have;
    z.avail_out = (uInt)(out.size() - have);
    r = inflate(&z, Z_NO_FLUSH);
    have = out.size() - z.avail_out;
    if (r == Z_STREAM_END) break;
    if (r != Z_OK) {
      inflateEnd(&z);
      throw SliceError("Corrupt deflated DICOM dataset");
    }
    if (z.avail_in == 0 && z.avail_out != 0) {  // input used up without the stream's end
      inflateEnd(&z);
      throw SliceError("Truncated deflated DICOM dataset");
    }
  }
  inflateEnd(&z);
  out.resize(have);
  return out;
}

// One RLE segment (PS3.5 G.3.1, PackBits) → exactly `n` bytes at dst with stride `stride`.
void unpackbits(const uint8_t* p, size_t len, uint8_t* dst, size_t n, size_t stride) {
  size_t i = 0, o = 0;
  while (o < n) {
    if (i >= len) throw SliceError("Truncated RLE segment");
    const int8_t c = (int8_t)p[i++];
    if (c >= 0) {
      const size_t k = (size_t)c + 1;
      if (i + k > len || o + k > n) throw SliceError("Corrupt RLE literal run");
      for (size_t j = 0; j < k; ++j) dst[(o + j) * stride] = p[i + j];
      i += k;
      o += k;
    } else if (c != -128) {
      const size_t k = (size_t)(1 - c);
      if (i >= len || o + k > n) throw SliceError("Corrupt RLE replicate run");
      const uint8_t v = p[i++];
      for (size_t j = 0; j < k; ++j) dst[(o + j) * stride] = v;
      o += k;
    }
  }
}

// One RLE fragment (64-byte header of segment offsets, then the segments) → one frame of native
// little-endian samples: segment 0 holds the most significant bytes (PS3.5 G.2).
void decode_rle_frame(const uint8_t* f, size_t len, int rows, int cols, int bytes_per_sample, uint8_t* out) {
  if (len < 64) throw SliceError("Truncated RLE header");
  auto le32 = [&](size_t o) { return (uint32_t)f[o] | ((uint32_t)f[o + 1] << 8) | ((uint32_t)f[o + 2] << 16) | ((uint32_t)f[o + 3] << 24); };
  const uint32_t nseg = le32(0);
  if ((int)nseg != bytes_per_sample) throw SliceError("RLE segment count " + std::to_string(nseg) + " does not match BitsAllocated");
  const size_t n = (size_t)rows * cols;
  for (uint32_t k = 0; k < nseg; ++k) {
    const size_t a = le32(4 + 4 * k), b = k + 1 < nseg ? le32(8 + 4 * k) : len;
    if (a < 64 || a > b || b > len) throw SliceError("Bad RLE segment offset");
    // segment k = byte (nseg - 1 - k) of every little-endian sample
    unpackbits(f + a, b - a, out + (nseg - 1 - k), n, (size_t)bytes_per_sample);
  }
}

// JPEG frames (PS3.5 A.4; lossless or sequential DCT by the transfer syntax): one frame's fragments concatenated (a single-frame image may
// span several fragments; a multi-frame one has one fragment per frame), decoded and stored as
// native little-endian samples. The codec's precision must fit BitsAllocated; signed data is
// sign-extended from BitsStored like the native encodings written by this repo (the codec carries the
// stored bit patterns).
void decode_jpeg_lossless_frames(Header& h, const uint8_t* d, const std::vector<std::pair<size_t, size_t>>& frags, int frames) {
  if (frags.empty()) throw SliceError("JPEG pixel data without fragments");
  if (frames > 1 && (int)frags.size() != frames)
    throw SliceError("JPEG pixel data has " + std::to_string(frags.size()) + " fragments for " + std::to_string(frames) +
                     " frames (one fragment per frame is supported for multi-frame images)");
  const size_t fpix = (size_t)h.rows * h.cols, fb = h.frame_bytes();
  size_t total = 0;
  for (const auto& f : frags) total += f.second;
  if (fpix * frames > total * 8 + 64 * (size_t)frames)  // ≥ 1 bit per sample
    throw SliceError("JPEG fragment too short for a " + std::to_string(h.rows) + "x" + std::to_string(h.cols) + " frame");
  auto dec = std::make_shared<std::vector<uint8_t>>(fb * frames);
  std::vector<uint8_t> joined;
  std::vector<uint16_t> px;
  for (int f = 0; f < frames; ++f) {
    const uint8_t* src;
    size_t len;
    if (frames == 1 && frags.size() > 1) {
      joined.clear();
      for (const auto& fr : frags) joined.insert(joined.end(), d + fr.first, d + fr.first + fr.second);
      src = joined.data();
      len = joined.size();
    } else {
      src = d + frags[f].first;
      len = frags[f].second;
    }
    int rows = 0, cols = 0, precision = 0;
    if (h.syntax == Syntax::kJpegLossless) {
      const jpegll::Info info = jpegll::decode(src, len, px, h.rows, h.cols);
      rows = info.rows, cols = info.cols, precision = info.precision;
    } else {
      const jpegdct::Info info = jpegdct::decode(src, len, px, h.rows, h.cols);
      if (h.syntax == Syntax::kJpegBaseline && info.precision != 8)
        throw SliceError("JPEG Baseline transfer syntax with " + std::to_string(info.precision) + "-bit samples");
      rows = info.rows, cols = info.cols, precision = info.precision;
    }
    if (rows != h.rows || cols != h.cols)
      throw SliceError("JPEG frame is " + std::to_string(cols) + "x" + std::to_string(rows) + ", the dataset says " +
                       std::to_string(h.cols) + "x" + std::to_string(h.rows));
    if (precision > h.bits_allocated)
      throw SliceError("JPEG precision " + std::to_string(precision) + " exceeds BitsAllocated " +
                       std::to_string(h.bits_allocated));
    uint8_t* o = dec->data() + f * fb;
    const int bs = h.bits_stored > 0 ? h.bits_stored : h.bits_allocated;
    const bool sext = h.pixel_rep == 1 && bs < 16 && h.bits_allocated == 16;
    for (size_t i = 0; i < fpix; ++i) {
      uint16_t v = px[i];
      if (h.bits_allocated == 8) {
        o[i] = (uint8_t)v;
        continue;
      }
      if (sext && (v >> (bs - 1) & 1)) v = (uint16_t)(v | (uint16_t)(0xFFFFu << bs));
      o[2 * i] = (uint8_t)v;
      o[2 * i + 1] = (uint8_t)(v >> 8);
    }
  }
  h.decoded = dec;
  h.pixel_offset = 0;
  h.pixel_length = dec->size();
}

}  // namespace

const char* syntax_name(Syntax s) {
  switch (s) {
    case Syntax::kImplicitLE: return "implicit";
    case Syntax::kExplicitLE: return "explicit";
    case Syntax::kExplicitBE: return "big";
    case Syntax::kDeflatedLE: return "deflated";
    case Syntax::kRleLossless: return "rle";
    case Syntax::kJpegLossless: return "jpeg-lossless";
    case Syntax::kJpegBaseline: return "jpeg-baseline";
    case Syntax::kJpegExtended: return "jpeg-extended";
  }
  return "?";
}

Header parse(const uint8_t* data, size_t size) { return parse_prefix(data, size, size); }

Header parse_prefix(const uint8_t* data, size_t avail, size_t size) {
  Header h;
  const size_t full = size;
  size = avail;
  Cursor c{data, size, 0, false};
  bool explicit_vr = true;
  if (size >= 132 && std::memcmp(data + 128, "DICM", 4) == 0) {
    c.pos = 132;
    // File meta information: always Explicit VR Little Endian.
    while (c.has(8)) {
      size_t save = c.pos;
      uint16_t g = c.u16();
      c.pos = save;
      if (g != 0x0002) break;
      Elem e = read_elem(c, true);
      if (e.len == kUndefined) throw SliceError("Undefined length in file meta group");
      c.need(e.len);
      if (e.elem == 0x0010) h.transfer_syntax = str_value(c, e);
      c.pos += e.len;
    }
  } else {
    // No preamble: assume an Implicit VR LE dataset (legacy ACR-NEMA style files).
    h.transfer_syntax = "1.2.840.10008.1.2";
    if (size < 8) throw SliceError("Not a DICOM file");
  }
  const std::string& ts = h.transfer_syntax;
  std::shared_ptr<std::vector<uint8_t>> inflated;
  if (ts == "1.2.840.10008.1.2") {
    h.syntax = Syntax::kImplicitLE;
    explicit_vr = false;
  } else if (ts == "1.2.840.10008.1.2.1" || ts.empty()) {
    h.syntax = Syntax::kExplicitLE;
  } else if (ts == "1.2.840.10008.1.2.2") {
    h.syntax = Syntax::kExplicitBE;
    c.big = true;
  } else if (ts == "1.2.840.10008.1.2.1.99") {
    // Deflated Explicit VR LE: everything after the meta group is one raw deflate stream.
    h.syntax = Syntax::kDeflatedLE;
    if (avail < full) throw SliceError("Truncated DICOM data");  // callers retry with the whole file
    inflated = std::make_shared<std::vector<uint8_t>>(inflate_raw(data + c.pos, size - c.pos));
    c = Cursor{inflated->data(), inflated->size(), 0, false};
  } else if (ts == "1.2.840.10008.1.2.5") {
    h.syntax = Syntax::kRleLossless;
  } else if (ts == "1.2.840.10008.1.2.4.70" || ts == "1.2.840.10008.1.2.4.57") {
    h.syntax = Syntax::kJpegLossless;  // lossless JPEG, process 14 (SV1 / any selection value)
  } else if (ts == "1.2.840.10008.1.2.4.50") {
    h.syntax = Syntax::kJpegBaseline;  // lossy 8-bit sequential DCT, process 1
  } else if (ts == "1.2.840.10008.1.2.4.51") {
    h.syntax = Syntax::kJpegExtended;  // lossy 8/12-bit sequential DCT, processes 2 & 4
  } else if (ts.rfind("1.2.840.10008.1.2.4.", 0) == 0) {
    throw SliceError("Unsupported compressed DICOM transfer syntax (JPEG family): " + ts);
  } else {
    throw SliceError("Unsupported DICOM transfer syntax: " + ts);
  }

  bool have_pixels = false;
  while (c.has(8)) {
    Elem e = read_elem(c, explicit_vr);
    if (e.group == 0x7FE0 && e.elem == 0x0010) {
      if (e.len == kUndefined) {
        const bool jpeg = h.syntax == Syntax::kJpegLossless || h.syntax == Syntax::kJpegBaseline ||
                          h.syntax == Syntax::kJpegExtended;
        if (h.syntax != Syntax::kRleLossless && !jpeg)
          throw SliceError("Encapsulated (compressed) pixel data in a native transfer syntax");
        if (avail < full) throw SliceError("Truncated DICOM data");  // callers retry with the whole file
        // Basic Offset Table item, then one fragment per frame (PS3.5 A.4, G.2), then the
        // sequence delimiter.
        std::vector<std::pair<size_t, size_t>> frags;
        bool bot = true;
        for (;;) {
          Elem it = read_elem(c, true);
          if (it.group == 0xFFFE && it.elem == 0xE0DD) break;
          if (it.group != 0xFFFE || it.elem != 0xE000 || it.len == kUndefined) throw SliceError("Malformed encapsulated pixel data");
          c.need(it.len);
          if (!bot) frags.push_back({it.value_pos, it.len});
          bot = false;
          c.pos += it.len;
        }
        if (h.rows <= 0 || h.cols <= 0 || (h.bits_allocated != 8 && h.bits_allocated != 16))
          throw SliceError(std::string(jpeg ? "JPEG" : "RLE") + " image without Rows/Columns/BitsAllocated before its pixel data");
        const int frames = std::max(1, h.frames);
        if (jpeg) {
          decode_jpeg_lossless_frames(h, c.d, frags, frames);
          have_pixels = true;
          break;
        }
        if ((int)frags.size() != frames)
          throw SliceError("RLE pixel data has " + std::to_string(frags.size()) + " fragments for " + std::to_string(frames) +
                           " frame(s) (one fragment per frame is supported)");
        const size_t fb = h.frame_bytes();
        // PackBits expands at most 64× (a 2-byte replicate run → 128 bytes): a fragment too short
        // for its frame is corrupt, found before the frame buffers are allocated.
        for (int f = 0; f < frames; ++f)
          if (fb > 64 * frags[f].second) throw SliceError("RLE fragment too short for a " + std::to_string(h.rows) + "x" +
                                                           std::to_string(h.cols) + " frame");
        auto dec = std::make_shared<std::vector<uint8_t>>(fb * frames);
        for (int f = 0; f < frames; ++f)
          decode_rle_frame(c.d + frags[f].first, frags[f].second, h.rows, h.cols, h.bits_allocated / 8, dec->data() + f * fb);
        h.decoded = dec;
        h.pixel_offset = 0;
        h.pixel_length = dec->size();
        have_pixels = true;
        break;
      }
      if (h.syntax == Syntax::kRleLossless || h.syntax == Syntax::kJpegLossless || h.syntax == Syntax::kJpegBaseline ||
          h.syntax == Syntax::kJpegExtended)
        throw SliceError(std::string(h.syntax == Syntax::kRleLossless ? "RLE Lossless" : "JPEG") +
                         " transfer syntax with native (not encapsulated) pixel data");
      h.pixel_offset = e.value_pos;
      h.pixel_length = e.len;
      have_pixels = true;
      break;
    }
    if (e.len == kUndefined) {
      skip_sequence(c, explicit_vr, 0);
      continue;
    }
    c.need(e.len);
    if (explicit_vr && e.vr[0] == 'S' && e.vr[1] == 'Q') {
      c.pos += e.len;
      continue;
    }
    const uint32_t tag = ((uint32_t)e.group << 16) | e.elem;
    switch (tag) {
      case 0x00080018: h.sop_instance_uid = str_value(c, e); break;
      case 0x00080060: h.modality = str_value(c, e); break;
      case 0x00100020: h.patient_id = str_value(c, e); break;
      case 0x0020000E: h.series_uid = str_value(c, e); break;
      case 0x00200013: h.instance_number = std::atoi(str_value(c, e).c_str()); break;
      case 0x00200032: {
        auto v = ds_values(str_value(c, e));
        if (v.size() >= 3) {
          h.has_position = true;
          h.position[0] = v[0];
          h.position[1] = v[1];
          h.position[2] = v[2];
        }
        break;
      }
      case 0x00201041: {
        auto v = ds_values(str_value(c, e));
        if (!v.empty()) h.slice_location = v[0];
        break;
      }
      case 0x00280002: h.samples = us_value(c, e); break;
      case 0x00280004: h.photometric = str_value(c, e); break;
      case 0x00280008: h.frames = std::atoi(str_value(c, e).c_str()); break;
      case 0x00280010: h.rows = us_value(c, e); break;
      case 0x00280011: h.cols = us_value(c, e); break;
      case 0x00280030: {
        auto v = ds_values(str_value(c, e));  // row spacing \ column spacing
        if (v.size() >= 2) {
          h.spacing_y = (float)v[0];
          h.spacing_x = (float)v[1];
        }
        break;
      }
      case 0x00280100: h.bits_allocated = us_value(c, e); break;
      case 0x00280101: h.bits_stored = us_value(c, e); break;
      case 0x00280102: h.high_bit = us_value(c, e); break;
      case 0x00280103: h.pixel_rep = us_value(c, e); break;
      case 0x00281052: {
        auto v = ds_values(str_value(c, e));
        if (!v.empty()) {
          h.intercept = (float)v[0];
          h.has_rescale = true;
        }
        break;
      }
      case 0x00281053: {
        auto v = ds_values(str_value(c, e));
        if (!v.empty()) {
          h.slope = (float)v[0];
          h.has_rescale = true;
        }
        break;
      }
      default: break;
    }
    c.pos += e.len;
  }
  if (!have_pixels) throw SliceError("No pixel data element in DICOM file");
  if (h.rows <= 0 || h.cols <= 0) throw SliceError("DICOM image has no Rows/Columns");
  if (h.samples != 1) throw SliceError("Only single-sample (monochrome) DICOM images are supported");
  if (h.frames < 1) h.frames = 1;
  if (inflated) h.decoded = inflated;
  if (!h.photometric.empty() && h.photometric != "MONOCHROME1" && h.photometric != "MONOCHROME2")
    throw SliceError("Unsupported PhotometricInterpretation: " + h.photometric);
  h.invert = h.photometric == "MONOCHROME1";
  if (h.bits_allocated == 16) {
    h.type = h.pixel_rep ? kI16 : kU16;
  } else if (h.bits_allocated == 8) {
    h.type = kU8;
  } else {
    throw SliceError("Unsupported BitsAllocated: " + std::to_string(h.bits_allocated));
  }
  if (h.bits_stored <= 0 || h.bits_stored > h.bits_allocated) h.bits_stored = h.bits_allocated;
  // Every frame must be present (a multi-frame file's last frame is checked, not only its first).
  const size_t need = h.frame_bytes() * (size_t)h.frames;
  const size_t limit = h.decoded ? h.decoded->size() : full;
  if (h.pixel_length < need || h.pixel_offset + need > limit)
    throw SliceError(h.frames > 1 ? "DICOM pixel data shorter than NumberOfFrames*Rows*Columns"
                                  : "DICOM pixel data shorter than Rows*Columns");
  if (!(h.slope == h.slope) || h.slope == 0.f) h.slope = 1.f;
  return h;
}

void invert_samples(uint16_t* px, size_t n, int bits) {
  const uint16_t mask = (uint16_t)(bits >= 16 ? 0xFFFFu : ((1u << bits) - 1u));
  for (size_t i = 0; i < n; ++i) px[i] = (uint16_t)(~px[i] & mask);
}

int select_frame(const Header& h, int policy) {
  if (h.frames <= 1) return 0;  // a single-frame file is its own slice under every policy
  if (policy < 0) {
    if (h.frames > 1)
      throw SliceError("Multi-frame DICOM (" + std::to_string(h.frames) +
                       " frames): the 2D pipeline imports single-frame slices (select one with --frame K)");
    return 0;
  }
  if (policy >= h.frames)
    throw SliceError("Frame " + std::to_string(policy) + " requested from a DICOM file with " + std::to_string(h.frames) +
                     " frame(s)");
  return policy;
}

void copy_pixels16(const Header& h, const uint8_t* data, size_t size, uint16_t* dst, int frame) {
  if (frame < 0 || frame >= h.frames) throw SliceError("DICOM frame " + std::to_string(frame) + " out of range");
  const size_t n = (size_t)h.rows * h.cols;
  const size_t off = h.pixel_offset + (size_t)frame * h.frame_bytes();
  const size_t limit = h.decoded ? h.decoded->size() : size;
  if (off + n * (h.bits_allocated / 8) > limit) throw SliceError("Truncated pixel data");
  const uint8_t* src = h.pixel_base(data) + off;
  if (h.bits_allocated == 8) {
    for (size_t i = 0; i < n; ++i) dst[i] = src[i];
  } else if (!h.native_le()) {
    for (size_t i = 0; i < n; ++i) dst[i] = (uint16_t)((src[2 * i] << 8) | src[2 * i + 1]);
  } else {
    std::memcpy(dst, src, n * 2);
  }
  if (h.invert) invert_samples(dst, n, h.bits_stored);
}

size_t read_file_into(const std::string& path, std::vector<uint8_t>& buf) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) throw SliceError("Cannot open file: " + path + " (" + std::strerror(errno) + ")");
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    throw SliceError("Cannot stat file: " + path);
  }
  size_t n = (size_t)st.st_size;
  if (buf.size() < n) buf.resize(n);
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::read(fd, buf.data() + got, n - got);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {
      ::close(fd);
      throw SliceError("Read error on file: " + path);
    }
    got += (size_t)r;
  }
  ::close(fd);
  return n;
}

// ------------------------------------------------------------------------------------------------
// SliceFile: header from a 16 KiB prefix, pixels read straight into the caller's buffer.
// ------------------------------------------------------------------------------------------------
SliceFile::SliceFile(const std::string& path, ReadMode mode, size_t prefix)
    : SliceFile(AT_FDCWD, path.c_str(), path, mode, prefix) {}

SliceFile::SliceFile(int dirfd, const char* name, const std::string& path, ReadMode mode, size_t prefix)
    : path_(path), mode_(mode), prefix_(prefix < 1024 ? 1024 : prefix) {
  fd_ = ::openat(dirfd, name, O_RDONLY | O_CLOEXEC);
  if (fd_ < 0) throw SliceError("Cannot open file: " + path + " (" + std::strerror(errno) + ")");
  if (mode_ == ReadMode::kStaged) return;  // size from the whole-file read (header): no fstat
  stat_size();
}

void SliceFile::stat_size() {
  struct stat st;
  if (fstat(fd_, &st) != 0) {
    ::close(fd_);
    fd_ = -1;
    throw SliceError("Cannot stat file: " + path_);
  }
  size_ = (size_t)st.st_size;
  size_known_ = true;
}

SliceFile::~SliceFile() {
  if (map_ && own_map_) ::munmap(const_cast<uint8_t*>(map_), size_);
  if (fd_ >= 0) ::close(fd_);
}

void SliceFile::pread_all(void* dst, size_t n, size_t off) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = ::pread(fd_, (uint8_t*)dst + got, n - got, (off_t)(off + got));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) throw SliceError("Read error on file: " + path_);
    got += (size_t)r;
  }
}

const Header& SliceFile::header(std::vector<uint8_t>& buf) {
  buf_ = &buf;
  if (mode_ == ReadMode::kStaged && !size_known_) {
    // One read of up to the buffer's size (≥ 256 KiB): a short read of a regular file is its end
    // (pool threads block signals, so no read is cut short by one); a full buffer may mean more,
    // then the size comes from fstat.
    if (buf.size() < (256u << 10)) buf.resize(256u << 10);
    size_t got = 0;
    for (;;) {
      const ssize_t r = ::pread(fd_, buf.data() + got, buf.size() - got, (off_t)got);
      if (r < 0 && errno == EINTR) continue;
      if (r < 0) throw SliceError("Read error on file: " + path_);
      got += (size_t)r;
      if (got < buf.size() || r == 0) break;
      stat_size();
      if (size_ <= got) break;
      buf.resize(size_);
    }
    size_ = got;
    size_known_ = true;
    have_ = size_;
    try {
      h_ = parse(buf.data(), size_);
    } catch (const SliceError&) {
      // A short read is normally the end of the file, but a read can also come back short
      // without reaching it (a signal on a thread that does not block them, NFS/FUSE): before
      // reporting a truncated file, check the size and finish the read.
      stat_size();
      if (size_ <= got) throw;
      if (buf.size() < size_) buf.resize(size_);
      pread_all(buf.data() + got, size_ - got, got);
      have_ = size_;
      h_ = parse(buf.data(), size_);
    }
    whole_ = true;
    return h_;
  }
  if (mode_ == ReadMode::kMapped && size_ > 0) {
    const bool fixed = map_at_ && size_ <= map_cap_;
    void* m = ::mmap(fixed ? map_at_ : nullptr, size_, PROT_READ, MAP_PRIVATE | MAP_POPULATE | (fixed ? MAP_FIXED : 0),
                     fd_, 0);
    if (m == MAP_FAILED) throw SliceError("Cannot map file: " + path_);
    own_map_ = !fixed;
    map_ = static_cast<const uint8_t*>(m);
    have_ = size_;
    h_ = parse(map_, size_);
    whole_ = true;
    return h_;
  }
  const size_t pre = mode_ == ReadMode::kStaged ? size_ : std::min(size_, prefix_);
  if (buf.size() < pre) buf.resize(pre);
  pread_all(buf.data(), pre, 0);
  buf_ = &buf;
  have_ = pre;
  if (pre < size_) {
    try {
      h_ = parse_prefix(buf.data(), pre, size_);
      whole_ = false;
      // Direct reads only for raw little-endian 16-bit samples; everything else is converted.
      if (h_.bits_allocated == 16 && h_.syntax != Syntax::kExplicitBE && !h_.decoded) return h_;
    } catch (const SliceError&) {
      // header longer than the prefix (or malformed): parse the whole file below
    }
  }
  if (buf.size() < size_) buf.resize(size_);
  if (pre < size_) pread_all(buf.data() + pre, size_ - pre, pre);
  have_ = size_;
  h_ = parse(buf.data(), size_);
  whole_ = true;
  return h_;
}

void SliceFile::pixels16(uint16_t* dst, int frame) {
  if (frame < 0 || frame >= h_.frames) throw SliceError("DICOM frame " + std::to_string(frame) + " out of range");
  const size_t n = (size_t)h_.rows * h_.cols * 2;
  const size_t off = h_.pixel_offset + (size_t)frame * h_.frame_bytes();
  if (whole_) {
    const bool raw16 = h_.bits_allocated == 16 && h_.native_le() && !h_.invert;
    if (raw16 && mode_ != ReadMode::kDirect) {
      const size_t limit = h_.decoded ? h_.decoded->size() : size_;
      if (off + n > limit) throw SliceError("Truncated pixel data");
      stream_copy(dst, h_.pixel_base(data()) + off, n);
    } else {
      copy_pixels16(h_, data(), size_, dst, frame);
    }
    return;
  }
  // Pixel bytes that came with the header read are taken from it; the rest is read into dst.
  size_t k = off < have_ ? std::min(n, have_ - off) : 0;
  if (k) std::memcpy(dst, buf_->data() + off, k);
  if (k < n) pread_all(reinterpret_cast<uint8_t*>(dst) + k, n - k, off + k);
  if (h_.invert) invert_samples(dst, n / 2, h_.bits_stored);
}

const uint16_t* SliceFile::staged_samples(int frame) const {
  if (!whole_ || mode_ == ReadMode::kDirect || !buf_) return nullptr;
  if (h_.bits_allocated != 16 || !h_.native_le() || h_.invert) return nullptr;
  if (frame < 0 || frame >= h_.frames) return nullptr;
  const size_t n = (size_t)h_.rows * h_.cols * 2;
  const size_t off = h_.pixel_offset + (size_t)frame * h_.frame_bytes();
  const size_t limit = h_.decoded ? h_.decoded->size() : size_;
  if (off + n > limit || (off & 1)) return nullptr;
  return reinterpret_cast<const uint16_t*>(h_.pixel_base(data()) + off);
}

void stream_copy(void* dst, const void* src, size_t n) {
  stream_copy_unfenced(dst, src, n);
  _mm_sfence();  // streaming stores are weakly ordered: complete them before the upload is queued
}

void stream_copy_unfenced(void* dst, const void* src, size_t n) {
  auto* d = static_cast<uint8_t*>(dst);
  const auto* s = static_cast<const uint8_t*>(src);
  size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (head > n) head = n;
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  for (; n >= 64; n -= 64, d += 64, s += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 32));
    const __m128i e = _mm_loadu_si128(reinterpret_cast<const __m128i*>(s + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(d), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(d + 48), e);
  }
  std::memcpy(d, s, n);
}

std::vector<uint8_t> read_file(const std::string& path) {
  std::vector<uint8_t> b;
  size_t n = read_file_into(path, b);
  b.resize(n);
  return b;
}

// ------------------------------------------------------------------------------------------------
// Writer
// ------------------------------------------------------------------------------------------------
namespace {

struct Out {
  std::vector<uint8_t> b;
  bool big = false;
  void u16(uint16_t v) {
    if (big) {
      b.push_back((uint8_t)(v >> 8));
      b.push_back((uint8_t)v);
    } else {
      b.push_back((uint8_t)v);
      b.push_back((uint8_t)(v >> 8));
    }
  }
  void u32(uint32_t v) {
    if (big) {
      for (int s = 24; s >= 0; s -= 8) b.push_back((uint8_t)(v >> s));
    } else {
      for (int s = 0; s < 32; s += 8) b.push_back((uint8_t)(v >> s));
    }
  }
  void raw(const void* p, size_t n) {
    const uint8_t* q = (const uint8_t*)p;
    b.insert(b.end(), q, q + n);
  }
  void elem(uint16_t g, uint16_t e, const char* vr, const void* val, uint32_t len, bool explicit_vr) {
    u16(g);
    u16(e);
    if (explicit_vr) {
      b.push_back((uint8_t)vr[0]);
      b.push_back((uint8_t)vr[1]);
      if (long_length_vr(vr)) {
        u16(0);
        u32(len);
      } else {
        u16((uint16_t)len);
      }
    } else {
      u32(len);
    }
    raw(val, len);
  }
  void str(uint16_t g, uint16_t e, const char* vr, std::string s, bool explicit_vr) {
    if (s.size() & 1) s.push_back(vr[0] == 'U' && vr[1] == 'I' ? '\0' : ' ');
    elem(g, e, vr, s.data(), (uint32_t)s.size(), explicit_vr);
  }
  void us(uint16_t g, uint16_t e, uint16_t v, bool explicit_vr) {
    uint8_t t[2];
    if (big) {
      t[0] = (uint8_t)(v >> 8);
      t[1] = (uint8_t)v;
    } else {
      t[0] = (uint8_t)v;
      t[1] = (uint8_t)(v >> 8);
    }
    elem(g, e, "US", t, 2, explicit_vr);
  }
};

std::string fmt_ds(double v) {
  char buf[32];
  std::snprintf(buf, sizeof(buf), "%.6g", v);
  return buf;
}

}  // namespace

namespace {

// PackBits (PS3.5 G.3.1) of n bytes read at stride `stride`: replicate runs of ≥ 3 equal bytes,
// literal runs otherwise, each at most 128 long.
void packbits(const uint8_t* src, size_t n, size_t stride, std::vector<uint8_t>& out) {
  auto at = [&](size_t i) { return src[i * stride]; };
  size_t i = 0;
  while (i < n) {
    size_t r = 1;
    while (i + r < n && r < 128 && at(i + r) == at(i)) ++r;
    if (r >= 3) {
      out.push_back((uint8_t)(int8_t)(1 - (int)r));
      out.push_back(at(i));
      i += r;
      continue;
    }
    size_t l = 0;  // literal run up to the next run of ≥ 3
    while (i + l < n && l < 128) {
      if (i + l + 2 < n && at(i + l) == at(i + l + 1) && at(i + l) == at(i + l + 2)) break;
      ++l;
    }
    out.push_back((uint8_t)(l - 1));
    for (size_t j = 0; j < l; ++j) out.push_back(at(i + j));
    i += l;
  }
  if (out.size() & 1) out.push_back(0x80);  // segments are padded to even length (no-op code)
}

std::vector<uint8_t> deflate_raw(const uint8_t* src, size_t n) {
  z_stream z{};
  if (deflateInit2(&z, Z_DEFAULT_COMPRESSION, Z_DEFLATED, -MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    throw std::runtime_error("zlib deflateInit failed");
  std::vector<uint8_t> out(deflateBound(&z, (uLong)n) + 16);
  z.next_in = const_cast<Bytef*>(src);
  z.avail_in = (uInt)n;
  z.next_out = out.data();
  z.avail_out = (uInt)out.size();
  const int r = deflate(&z, Z_FINISH);
  deflateEnd(&z);
  if (r != Z_STREAM_END) throw std::runtime_error("zlib deflate failed");
  out.resize(z.total_out);
  return out;
}

}  // namespace

std::vector<uint8_t> write(const WriteSpec& s) {
  const char* ts = s.syntax == Syntax::kImplicitLE   ? "1.2.840.10008.1.2"
                   : s.syntax == Syntax::kExplicitLE ? "1.2.840.10008.1.2.1"
                   : s.syntax == Syntax::kExplicitBE ? "1.2.840.10008.1.2.2"
                   : s.syntax == Syntax::kDeflatedLE ? "1.2.840.10008.1.2.1.99"
                   : s.syntax == Syntax::kJpegLossless
                       ? (s.jpeg_predictor == 1 ? "1.2.840.10008.1.2.4.70" : "1.2.840.10008.1.2.4.57")
                   : s.syntax == Syntax::kJpegBaseline ? "1.2.840.10008.1.2.4.50"
                   : s.syntax == Syntax::kJpegExtended ? "1.2.840.10008.1.2.4.51"
                                                       : "1.2.840.10008.1.2.5";
  const bool dct = s.syntax == Syntax::kJpegBaseline || s.syntax == Syntax::kJpegExtended;
  const bool encapsulated = s.syntax == Syntax::kRleLossless || s.syntax == Syntax::kJpegLossless || dct;
  if ((s.syntax == Syntax::kDeflatedLE || encapsulated) && !s.preamble)
    throw std::runtime_error("deflated / RLE / JPEG files need the file meta group (preamble)");
  const char* sop_class = "1.2.840.10008.5.1.4.1.1.4";  // MR Image Storage
  Out out;
  if (s.preamble) {
    out.b.assign(128, 0);
    out.raw("DICM", 4);
    Out meta;
    uint8_t ver[2] = {0, 1};
    meta.elem(0x0002, 0x0001, "OB", ver, 2, true);
    meta.str(0x0002, 0x0002, "UI", sop_class, true);
    meta.str(0x0002, 0x0003, "UI", s.sop_uid, true);
    meta.str(0x0002, 0x0010, "UI", ts, true);
    meta.str(0x0002, 0x0012, "UI", "1.2.826.0.1.3680043.10.999", true);
    meta.str(0x0002, 0x0013, "SH", "NM03_MI355X", true);
    uint8_t gl[4] = {(uint8_t)meta.b.size(), (uint8_t)(meta.b.size() >> 8), (uint8_t)(meta.b.size() >> 16),
                     (uint8_t)(meta.b.size() >> 24)};
    out.elem(0x0002, 0x0000, "UL", gl, 4, true);
    out.raw(meta.b.data(), meta.b.size());
  }
  const size_t meta_end = out.b.size();
  const bool ex = s.syntax != Syntax::kImplicitLE;
  out.big = s.syntax == Syntax::kExplicitBE;
  const int frames = std::max(1, s.frames);
  out.str(0x0008, 0x0008, "CS", "ORIGINAL\\PRIMARY", ex);
  out.str(0x0008, 0x0016, "UI", sop_class, ex);
  out.str(0x0008, 0x0018, "UI", s.sop_uid, ex);
  out.str(0x0008, 0x0060, "CS", s.modality, ex);
  out.str(0x0010, 0x0010, "PN", "SYNTHETIC^" + s.patient_id, ex);
  out.str(0x0010, 0x0020, "LO", s.patient_id, ex);
  out.str(0x0018, 0x0050, "DS", fmt_ds(s.slice_thickness), ex);
  out.str(0x0020, 0x000D, "UI", s.study_uid, ex);
  out.str(0x0020, 0x000E, "UI", s.series_uid, ex);
  out.str(0x0020, 0x0013, "IS", std::to_string(s.instance_number), ex);
  out.str(0x0020, 0x0032, "DS",
          fmt_ds(s.position[0]) + "\\" + fmt_ds(s.position[1]) + "\\" + fmt_ds(s.position[2]), ex);
  out.str(0x0020, 0x0037, "DS", "1\\0\\0\\0\\1\\0", ex);
  out.str(0x0020, 0x1041, "DS", fmt_ds(s.position[2]), ex);
  out.us(0x0028, 0x0002, 1, ex);
  out.str(0x0028, 0x0004, "CS", s.photometric, ex);
  if (frames > 1) out.str(0x0028, 0x0008, "IS", std::to_string(frames), ex);
  out.us(0x0028, 0x0010, (uint16_t)s.rows, ex);
  out.us(0x0028, 0x0011, (uint16_t)s.cols, ex);
  out.str(0x0028, 0x0030, "DS", fmt_ds(s.spacing_y) + "\\" + fmt_ds(s.spacing_x), ex);
  const int ba = s.type == kU8 ? 8 : 16;
  out.us(0x0028, 0x0100, (uint16_t)ba, ex);
  int bs = s.bits_stored > 0 && s.bits_stored <= ba ? s.bits_stored : ba;
  out.us(0x0028, 0x0101, (uint16_t)bs, ex);
  out.us(0x0028, 0x0102, (uint16_t)(bs - 1), ex);
  out.us(0x0028, 0x0103, s.type == kI16 ? 1 : 0, ex);
  if (s.write_rescale) {
    out.str(0x0028, 0x1052, "DS", fmt_ds(s.intercept), ex);
    out.str(0x0028, 0x1053, "DS", fmt_ds(s.slope), ex);
  }
  const size_t n = (size_t)s.rows * s.cols * frames;
  const size_t bps = ba / 8;
  // Native little-endian samples (big-endian for kExplicitBE) of every frame.
  std::vector<uint8_t> px(ba == 8 ? (n + (n & 1)) : n * 2, 0);
  if (ba == 8) {
    for (size_t i = 0; i < n; ++i) px[i] = s.pixels ? (uint8_t)s.pixels[i] : 0;
  } else {
    for (size_t i = 0; i < n; ++i) {
      uint16_t v = s.pixels ? s.pixels[i] : 0;
      if (out.big) {
        px[2 * i] = (uint8_t)(v >> 8);
        px[2 * i + 1] = (uint8_t)v;
      } else {
        px[2 * i] = (uint8_t)v;
        px[2 * i + 1] = (uint8_t)(v >> 8);
      }
    }
  }
  if (encapsulated) {
    // Encapsulated: (7FE0,0010) OB of undefined length, an empty Basic Offset Table item, one
    // fragment per frame (JPEG: optionally several), the sequence delimiter.
    const size_t fpix = (size_t)s.rows * s.cols;
    out.u16(0x7FE0);
    out.u16(0x0010);
    out.raw("OB", 2);
    out.u16(0);
    out.u32(0xFFFFFFFFu);
    auto item = [&](uint16_t e, const std::vector<uint8_t>& v) {
      out.u16(0xFFFE);
      out.u16(e);
      out.u32((uint32_t)v.size());
      out.raw(v.data(), v.size());
    };
    item(0xE000, {});
    for (int f = 0; (s.syntax == Syntax::kJpegLossless || dct) && f < frames; ++f) {
      std::vector<uint16_t> fr(fpix);
      for (size_t i = 0; i < fpix; ++i) fr[i] = s.pixels ? s.pixels[f * fpix + i] : 0;
      std::vector<uint8_t> j;
      if (dct) {
        const int prec = s.syntax == Syntax::kJpegBaseline || bs <= 8 ? 8 : 12;
        const uint16_t mx = (uint16_t)((1u << prec) - 1), m = (uint16_t)((1u << bs) - 1);
        for (auto& v : fr) v = std::min<uint16_t>((uint16_t)(v & m), mx);
        j = jpegdct::encode(fr.data(), s.rows, s.cols, prec, s.jpeg_quality, s.jpeg_restart_rows * ((s.cols + 7) / 8));
      } else {
        j = jpegll::encode(fr.data(), s.rows, s.cols, std::max(2, bs), s.jpeg_predictor, 0, s.jpeg_restart_rows);
      }
      if (j.size() & 1) j.push_back(0);  // even item length (a trailing pad byte after EOI)
      const int nf = frames == 1 ? std::max(1, s.jpeg_fragments) : 1;
      const size_t step = (j.size() / nf + 1) & ~(size_t)1;
      for (size_t o = 0; o < j.size(); o += step)
        item(0xE000, std::vector<uint8_t>(j.begin() + (long)o, j.begin() + (long)std::min(j.size(), o + step)));
    }
    for (int f = 0; s.syntax == Syntax::kRleLossless && f < frames; ++f) {
      std::vector<uint8_t> frag(64, 0), segs;
      std::vector<uint32_t> offs;
      for (size_t k = 0; k < bps; ++k) {
        offs.push_back((uint32_t)(64 + segs.size()));
        // segment k: byte (bps - 1 - k) of each little-endian sample (MSB first)
        packbits(px.data() + f * fpix * bps + (bps - 1 - k), fpix, bps, segs);
      }
      auto put = [&](size_t o, uint32_t v) {
        for (int b = 0; b < 4; ++b) frag[o + b] = (uint8_t)(v >> (8 * b));
      };
      put(0, (uint32_t)bps);
      for (size_t k = 0; k < bps; ++k) put(4 + 4 * k, offs[k]);
      frag.insert(frag.end(), segs.begin(), segs.end());
      item(0xE000, frag);
    }
    out.u16(0xFFFE);
    out.u16(0xE0DD);
    out.u32(0);
  } else {
    out.elem(0x7FE0, 0x0010, ba == 8 ? "OB" : "OW", px.data(), (uint32_t)px.size(), ex);
  }
  if (s.syntax == Syntax::kDeflatedLE) {
    std::vector<uint8_t> z = deflate_raw(out.b.data() + meta_end, out.b.size() - meta_end);
    if (z.size() & 1) z.push_back(0);  // even length
    out.b.resize(meta_end);
    out.b.insert(out.b.end(), z.begin(), z.end());
  }
  return out.b;
}

void write_file(const std::string& path, const WriteSpec& spec) {
  std::vector<uint8_t> b = write(spec);
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) throw std::runtime_error("Cannot create " + path);
  f.write((const char*)b.data(), (std::streamsize)b.size());
  if (!f) throw std::runtime_error("Write failed: " + path);
}

}  // namespace nm03::dicom
