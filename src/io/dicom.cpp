// DICOM Part-10 reader/writer. Replaces DCMTK behind FAST's DICOMFileImporter
// (reference call sites: test_pipeline.cpp:33-42, main_sequential.cpp:175-177,
// main_parallel.cpp:78-80). Only what a 2D monochrome slice import needs is interpreted; every
// other element is skipped structurally (including undefined-length sequences).
#include "nm03/dicom.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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

}  // namespace

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
  if (ts == "1.2.840.10008.1.2") {
    h.syntax = Syntax::kImplicitLE;
    explicit_vr = false;
  } else if (ts == "1.2.840.10008.1.2.1" || ts.empty()) {
    h.syntax = Syntax::kExplicitLE;
  } else if (ts == "1.2.840.10008.1.2.2") {
    h.syntax = Syntax::kExplicitBE;
    c.big = true;
  } else {
    throw SliceError("Unsupported DICOM transfer syntax: " + ts);
  }

  bool have_pixels = false;
  while (c.has(8)) {
    Elem e = read_elem(c, explicit_vr);
    if (e.group == 0x7FE0 && e.elem == 0x0010) {
      if (e.len == kUndefined) throw SliceError("Encapsulated (compressed) pixel data is not supported");
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
  if (h.bits_allocated == 16) {
    h.type = h.pixel_rep ? kI16 : kU16;
  } else if (h.bits_allocated == 8) {
    h.type = kU8;
  } else {
    throw SliceError("Unsupported BitsAllocated: " + std::to_string(h.bits_allocated));
  }
  if (h.bits_stored <= 0 || h.bits_stored > h.bits_allocated) h.bits_stored = h.bits_allocated;
  const size_t need = (size_t)h.rows * h.cols * (h.bits_allocated / 8);
  if (h.pixel_length < need || h.pixel_offset + need > full)
    throw SliceError("DICOM pixel data shorter than Rows*Columns");
  if (!(h.slope == h.slope) || h.slope == 0.f) h.slope = 1.f;
  return h;
}

void copy_pixels16(const Header& h, const uint8_t* data, size_t size, uint16_t* dst) {
  const size_t n = (size_t)h.rows * h.cols;
  const uint8_t* src = data + h.pixel_offset;
  if (h.pixel_offset + n * (h.bits_allocated / 8) > size) throw SliceError("Truncated pixel data");
  if (h.bits_allocated == 8) {
    for (size_t i = 0; i < n; ++i) dst[i] = src[i];
  } else if (h.syntax == Syntax::kExplicitBE) {
    for (size_t i = 0; i < n; ++i) dst[i] = (uint16_t)((src[2 * i] << 8) | src[2 * i + 1]);
  } else {
    std::memcpy(dst, src, n * 2);
  }
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
      if (h_.bits_allocated == 16 && h_.syntax != Syntax::kExplicitBE) return h_;
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

void SliceFile::pixels16(uint16_t* dst) {
  if (whole_) {
    const bool raw16 = h_.bits_allocated == 16 && h_.syntax != Syntax::kExplicitBE;
    const size_t n = (size_t)h_.rows * h_.cols * 2;
    if (raw16 && mode_ != ReadMode::kDirect) {
      if (h_.pixel_offset + n > size_) throw SliceError("Truncated pixel data");
      stream_copy(dst, data() + h_.pixel_offset, n);
    } else {
      copy_pixels16(h_, data(), size_, dst);
    }
    return;
  }
  // Pixel bytes that came with the header read are taken from it; the rest is read into dst.
  const size_t n = (size_t)h_.rows * h_.cols * 2;
  size_t k = h_.pixel_offset < have_ ? std::min(n, have_ - h_.pixel_offset) : 0;
  if (k) std::memcpy(dst, buf_->data() + h_.pixel_offset, k);
  if (k < n) pread_all(reinterpret_cast<uint8_t*>(dst) + k, n - k, h_.pixel_offset + k);
}

const uint16_t* SliceFile::staged_samples() const {
  if (!whole_ || mode_ == ReadMode::kDirect || !buf_) return nullptr;
  if (h_.bits_allocated != 16 || h_.syntax == Syntax::kExplicitBE) return nullptr;
  const size_t n = (size_t)h_.rows * h_.cols * 2;
  if (h_.pixel_offset + n > size_ || (h_.pixel_offset & 1)) return nullptr;
  return reinterpret_cast<const uint16_t*>(data() + h_.pixel_offset);
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

std::vector<uint8_t> write(const WriteSpec& s) {
  const char* ts = s.syntax == Syntax::kImplicitLE   ? "1.2.840.10008.1.2"
                   : s.syntax == Syntax::kExplicitLE ? "1.2.840.10008.1.2.1"
                                                     : "1.2.840.10008.1.2.2";
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
  const bool ex = s.syntax != Syntax::kImplicitLE;
  out.big = s.syntax == Syntax::kExplicitBE;
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
  out.str(0x0028, 0x0004, "CS", "MONOCHROME2", ex);
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
  const size_t n = (size_t)s.rows * s.cols;
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
  out.elem(0x7FE0, 0x0010, ba == 8 ? "OB" : "OW", px.data(), (uint32_t)px.size(), ex);
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
