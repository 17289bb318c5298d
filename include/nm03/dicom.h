// nm03/dicom.h — self-contained DICOM Part-10 reader/writer (replaces FAST's DCMTK-based
// DICOMFileImporter with setLoadSeries(false): test_pipeline.cpp:33-42, main_sequential.cpp:175-177).
//
// Supported: Part-10 files (preamble + "DICM") and bare datasets; Implicit VR LE, Explicit VR LE,
// Explicit VR BE, Deflated Explicit VR LE (1.2.840.10008.1.2.1.99, zlib), RLE Lossless
// (1.2.840.10008.1.2.5, encapsulated PackBits segments) and lossless JPEG — JPEG Lossless First-Order
// Prediction (1.2.840.10008.1.2.4.70) and JPEG Lossless Process 14 (1.2.840.10008.1.2.4.57), decoded
// on the host (nm03/jpeg_lossless.h), and lossy JPEG Baseline (1.2.840.10008.1.2.4.50) and Extended
// (1.2.840.10008.1.2.4.51, 12-bit) with the IJG islow inverse DCT (nm03/jpeg_dct.h); 8/16-bit
// monochrome, signed/unsigned,
// BitsStored masking, modality rescale, PixelSpacing, undefined-length sequences, MONOCHROME1
// (inverted at import, see Header::invert), multi-frame files (frame selection, see copy_pixels16).
// The other JPEG-family encapsulated syntaxes (progressive JPEG, JPEG-LS, JPEG 2000, ...)
// are rejected with a SliceError: the slice is skipped and counted like a fast::Exception in the
// reference. DCMTK behind FAST would decode them; that part of parity is unpinned (no DCMTK here).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "nm03/common.h"

namespace nm03::dicom {

enum class Syntax : uint8_t {
  kImplicitLE,
  kExplicitLE,
  kExplicitBE,
  kDeflatedLE,
  kRleLossless,
  kJpegLossless,   // 1.2.840.10008.1.2.4.70 / .4.57 (nm03/jpeg_lossless.h)
  kJpegBaseline,   // 1.2.840.10008.1.2.4.50: 8-bit sequential DCT (nm03/jpeg_dct.h)
  kJpegExtended,   // 1.2.840.10008.1.2.4.51: 8/12-bit sequential DCT
};

// Name of a transfer syntax as used in messages and by the Python bindings.
const char* syntax_name(Syntax s);

struct Header {
  int rows = 0, cols = 0, frames = 1;
  int bits_allocated = 0, bits_stored = 0, high_bit = 0, pixel_rep = 0, samples = 1;
  PixelType type = kU16;
  bool has_rescale = false;
  float slope = 1.f, intercept = 0.f;
  float spacing_x = 1.f, spacing_y = 1.f;  // column spacing, row spacing (mm)
  int instance_number = 0;
  bool has_position = false;
  double position[3] = {0, 0, 0};
  double slice_location = 0;
  std::string photometric, transfer_syntax, sop_instance_uid, series_uid, patient_id, modality;
  Syntax syntax = Syntax::kExplicitLE;
  size_t pixel_offset = 0;  // byte offset of (7FE0,0010) value in the buffer (in *decoded when set)
  size_t pixel_length = 0;  // byte length of the value field
  // PhotometricInterpretation MONOCHROME1 (minimum = white). The importer inverts such samples
  // within the stored bits (v → ~v & (2^BitsStored − 1), i.e. 2^B − 1 − v for unsigned data, −1 − v
  // for signed) so every stage sees MONOCHROME2 semantics (bright = high), the presentation DCMTK
  // hands to a viewer. With the reference's fixed-range IntensityNormalization (0..10000) this is a
  // documented choice, not a pinned FAST behaviour.
  bool invert = false;
  // Deflated, RLE and lossless JPEG files: the decoded bytes (inflated dataset, or every frame's
  // samples as native little-endian words/bytes); pixel_offset and pixel_length then refer to this buffer.
  std::shared_ptr<const std::vector<uint8_t>> decoded;
  size_t frame_bytes() const { return (size_t)rows * cols * (bits_allocated / 8); }
  // Samples are little-endian words (or bytes) at pixel_offset of pixel_base().
  bool native_le() const { return decoded || syntax != Syntax::kExplicitBE; }
  const uint8_t* pixel_base(const uint8_t* file) const { return decoded ? decoded->data() : file; }
};

// Parse a whole file image held in memory. Throws SliceError on malformed/unsupported input.
Header parse(const uint8_t* data, size_t size);

// Parse from a prefix `avail` bytes long of a `size`-byte file: succeeds when every element up to
// the pixel data lies in the prefix (throws SliceError "Truncated" otherwise).
Header parse_prefix(const uint8_t* data, size_t avail, size_t size);

// Frame `frame` (0-based) as 16-bit words in `dst` (rows*cols uint16): 8-bit data is widened,
// big-endian data byte-swapped, RLE/deflated data taken from Header::decoded, MONOCHROME1 inverted.
// Throws SliceError when the frame does not exist.
void copy_pixels16(const Header& h, const uint8_t* data, size_t size, uint16_t* dst, int frame = 0);

// Which frame of a file the 2D pipeline imports: `policy` < 0 rejects multi-frame files with a
// SliceError naming the frame count (a slice pipeline is handed a stack, and silently taking one of
// its frames would hide that); policy ≥ 0 selects that frame (an error if the file has fewer).
// Single-frame files always yield frame 0.
int select_frame(const Header& h, int policy);

// Inverts `n` samples within `bits` stored bits in place (MONOCHROME1 → MONOCHROME2).
void invert_samples(uint16_t* px, size_t n, int bits);

// Read a file completely (throws SliceError if it cannot be read).
std::vector<uint8_t> read_file(const std::string& path);
// Read into a caller-provided growable buffer (avoids reallocations in loader threads).
size_t read_file_into(const std::string& path, std::vector<uint8_t>& buf);

// A slice file opened for loading: the header is parsed from a 16 KiB prefix and, for
// little-endian 16-bit data, the pixels are read with one pread straight into the destination
// (the engine's pinned upload blob) — no intermediate whole-file buffer and no extra copy.
// How SliceFile moves a slice from the page cache into the caller's (pinned) buffer:
//   kDirect — parse a `prefix`-byte header read, then pread the pixels straight into dst (pixel
//             bytes already in the prefix are copied from it);
//   kStaged — one pread of the whole file into the caller's scratch buffer (cache-resident), then
//             non-temporal stores into dst: no read-for-ownership of the destination lines, which
//             the copy engine reads next anyway.
//   kMapped — the file is mapped (MAP_POPULATE) and parsed / packed / copied straight from the
//             page-cache pages: no copy into a scratch buffer, at the price of a mapping and an
//             unmap (TLB shootdown) per file. Otherwise behaves like kStaged.
enum class ReadMode { kDirect, kStaged, kMapped };

class SliceFile {
 public:
  explicit SliceFile(const std::string& path, ReadMode mode = ReadMode::kDirect, size_t prefix = 16384);
  // `name` relative to the directory fd `dirfd` (openat: no path walk from the root per file);
  // `path` is only used in messages.
  SliceFile(int dirfd, const char* name, const std::string& path, ReadMode mode = ReadMode::kDirect,
            size_t prefix = 16384);
  ~SliceFile();
  SliceFile(const SliceFile&) = delete;
  SliceFile& operator=(const SliceFile&) = delete;
  // File size; for kStaged known only after header() (the whole-file read replaces the fstat).
  size_t size() const { return size_; }
  // kMapped only: map the file at `addr` (MAP_FIXED inside a caller-reserved region of `cap`
  // bytes) instead of a fresh address, and leave it mapped: the caller unmaps the whole region in
  // one call (one TLB shootdown for a batch of files instead of one per file). Files larger than
  // `cap` get an ordinary mapping.
  void map_at(void* addr, size_t cap) {
    map_at_ = addr;
    map_cap_ = cap;
  }
  // Parses the header (`buf` is scratch space owned by the caller and must outlive pixels16).
  const Header& header(std::vector<uint8_t>& buf);
  // Frame `frame` as 16-bit words into dst (rows*cols elements), MONOCHROME1 inverted.
  void pixels16(uint16_t* dst, int frame = 0);
  // True when pixels16 reads straight from the file (prefix parse, LE 16-bit data).
  bool direct() const { return !whole_; }
  // Staged reads of little-endian 16-bit data (including decoded RLE/deflated files): frame
  // `frame`'s samples inside the caller's scratch buffer or the decoded buffer (valid until reused),
  // else nullptr — also for MONOCHROME1, whose samples must go through pixels16's inversion.
  const uint16_t* staged_samples(int frame = 0) const;

 private:
  void pread_all(void* dst, size_t n, size_t off);
  void stat_size();
  bool size_known_ = false;
  const uint8_t* data() const { return map_ ? map_ : buf_->data(); }
  std::string path_;
  const uint8_t* map_ = nullptr;  // kMapped: the whole file
  bool own_map_ = true;           // false: mapped at map_at_, the caller unmaps
  void* map_at_ = nullptr;
  size_t map_cap_ = 0;
  int fd_ = -1;
  size_t size_ = 0;
  ReadMode mode_ = ReadMode::kDirect;
  size_t prefix_ = 16384;
  size_t have_ = 0;  // bytes of the file at the start of *buf_
  Header h_;
  bool whole_ = true;
  std::vector<uint8_t>* buf_ = nullptr;
};

// memcpy with non-temporal (streaming) stores for the 16-byte-aligned body of dst.
void stream_copy(void* dst, const void* src, size_t n);
// The same without the closing store fence: for a sequence of copies fenced once by the caller
// (a fence per small copy drains the write-combining buffers every time).
void stream_copy_unfenced(void* dst, const void* src, size_t n);

struct WriteSpec {
  int rows = 256, cols = 256;
  PixelType type = kU16;
  int bits_stored = 16;
  const uint16_t* pixels = nullptr;  // rows*cols 16-bit samples (8-bit type: low bytes used)
  bool write_rescale = false;
  float slope = 1.f, intercept = 0.f;
  float spacing_x = 1.f, spacing_y = 1.f;
  double slice_thickness = 1.0;
  int instance_number = 1;
  double position[3] = {0, 0, 0};
  std::string patient_id = "PGBM-000";
  std::string study_uid = "1.2.826.0.1.3680043.10.1", series_uid = "1.2.826.0.1.3680043.10.2",
              sop_uid = "1.2.826.0.1.3680043.10.3";
  std::string modality = "MR";
  std::string photometric = "MONOCHROME2";
  int frames = 1;  // pixels holds frames*rows*cols samples; NumberOfFrames written when > 1
  // kDeflatedLE: the dataset after the meta group is raw-deflated (zlib); kRleLossless: one
  // PackBits-coded fragment per frame (MSB segment, then LSB segment for 16-bit data);
  // kJpegLossless: one lossless JPEG per frame (precision = BitsStored), selection value
  // `jpeg_predictor` (1: transfer syntax .4.70, else .4.57), restart markers every
  // `jpeg_restart_rows` rows (0: none), each frame split into `jpeg_fragments` fragments.
  // kJpegBaseline / kJpegExtended: one lossy DCT JPEG per frame (8-bit / 12-bit samples, the stored
  // bits clamped to the precision) at `jpeg_quality`, restart markers every `jpeg_restart_rows` block
  // rows (0: none).
  Syntax syntax = Syntax::kExplicitLE;
  int jpeg_predictor = 1, jpeg_restart_rows = 0, jpeg_fragments = 1, jpeg_quality = 90;
  bool preamble = true;  // write 128-byte preamble + "DICM" + file meta group (required by kDeflatedLE/kRleLossless)
};

std::vector<uint8_t> write(const WriteSpec& spec);
void write_file(const std::string& path, const WriteSpec& spec);

}  // namespace nm03::dicom
