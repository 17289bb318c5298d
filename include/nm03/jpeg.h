// nm03/jpeg.h — host side of the JPEG exporter (replaces FAST ImageFileExporter → Qt → libjpeg,
// main_sequential.cpp:61-73). Produces baseline JFIF, 3 components (Y=gray, Cb=Cr=128), 4:2:0,
// quality-scaled Annex K tables, standard Huffman tables, byte-compatible with libjpeg(-turbo).
//
// The GPU encoder (k4_jpeg.hip) produces the entropy-coded segment; the host prepends
// `make_header` and appends EOI. `encode_gray420` is the single-threaded golden encoder.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "nm03/jpeg_common.h"

namespace nm03::jpeg {

struct Tables {
  int quality = 75;
  uint16_t qluma[64];    // natural order
  uint16_t qchroma[64];  // natural order
  int32_t div_luma[64];  // islow divisors 8·Q, natural order
  int32_t div_chroma[64];
};

Tables make_tables(int quality);

// SOI, APP0(JFIF 1.01), DQT×2, SOF0, DHT×4, SOS for a w×h image with 2x2/1x1/1x1 sampling.
std::vector<uint8_t> make_header(int width, int height, const Tables& t);

// Golden single-thread encode of an 8-bit gray plane as YCbCr 4:2:0 (complete file bytes).
std::vector<uint8_t> encode_gray420(const uint8_t* gray, int width, int height, int stride, int quality);

// Entropy-coded segment only (stuffed, padded with 1-bits), no markers. Used for tests against
// the GPU encoder.
std::vector<uint8_t> encode_scan_gray420(const uint8_t* gray, int width, int height, int stride,
                                         const Tables& t);

// Write header + scan + EOI to a file (single writev-style write).
void write_jpeg_file(const std::string& path, const std::vector<uint8_t>& header, const uint8_t* scan,
                     size_t scan_len);
// Same, `name` relative to the directory fd `dirfd` (openat: no path walk per file); `dir` only
// names the file in error messages. `creating`: the directory's creation hint (0 unknown, 1 the
// directory is being filled — create with O_EXCL directly, 2 its files exist — open without O_CREAT
// first); a missing file sets it to 1.
void write_jpeg_at(int dirfd, const std::string& dir, const std::string& name, const std::vector<uint8_t>& header,
                   const uint8_t* scan, size_t scan_len,
                   std::atomic<uint8_t>* creating = nullptr);

}  // namespace nm03::jpeg
