// nm03/dicom.h — self-contained DICOM Part-10 reader/writer (replaces FAST's DCMTK-based
// DICOMFileImporter with setLoadSeries(false): test_pipeline.cpp:33-42, main_sequential.cpp:175-177).
//
// Supported: Part-10 files (preamble + "DICM") and bare datasets; Implicit VR LE, Explicit VR LE,
// Explicit VR BE; 8/16-bit monochrome, signed/unsigned, BitsStored masking, modality rescale,
// PixelSpacing, undefined-length sequences. Compressed/encapsulated pixel data and deflate are
// rejected with a SliceError (the slice is skipped like a fast::Exception in the reference).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "nm03/common.h"

namespace nm03::dicom {

enum class Syntax : uint8_t { kImplicitLE, kExplicitLE, kExplicitBE };

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
  size_t pixel_offset = 0;  // byte offset of (7FE0,0010) value in the buffer
  size_t pixel_length = 0;  // byte length of the value field
};

// Parse a whole file image held in memory. Throws SliceError on malformed/unsupported input.
Header parse(const uint8_t* data, size_t size);

// Parse from a prefix `avail` bytes long of a `size`-byte file: succeeds when every element up to
// the pixel data lies in the prefix (throws SliceError "Truncated" otherwise).
Header parse_prefix(const uint8_t* data, size_t avail, size_t size);

// Copy the first frame's pixels to `dst` as 16-bit words (8-bit data is widened, big-endian data
// is byte-swapped). dst must hold rows*cols uint16.
void copy_pixels16(const Header& h, const uint8_t* data, size_t size, uint16_t* dst);

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
  // First frame as 16-bit words into dst (rows*cols elements).
  void pixels16(uint16_t* dst);
  // True when pixels16 reads straight from the file (prefix parse, LE 16-bit data).
  bool direct() const { return !whole_; }
  // Staged reads of little-endian 16-bit data: the first frame's samples inside the caller's
  // scratch buffer (valid until it is reused), else nullptr.
  const uint16_t* staged_samples() const;

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
  Syntax syntax = Syntax::kExplicitLE;
  bool preamble = true;  // write 128-byte preamble + "DICM" + file meta group
};

std::vector<uint8_t> write(const WriteSpec& spec);
void write_file(const std::string& path, const WriteSpec& spec);

}  // namespace nm03::dicom
