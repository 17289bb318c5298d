// nm03/jpeg.h — host side of the JPEG exporter (replaces FAST ImageFileExporter → Qt → libjpeg,
// main_sequential.cpp:61-73). Produces baseline JFIF, 3 components (Y=gray, Cb=Cr=128), 4:2:0 by
// default (4:4:4 and a one-component gray file on request: jpeg::Sampling), quality-scaled Annex K
// tables, standard Huffman tables, byte-compatible with libjpeg(-turbo).
//
// The GPU encoder (k4_jpeg.hip) produces the entropy-coded segment; the host prepends
// `make_header` and appends EOI. `encode_gray` is the single-threaded golden encoder.
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

// SOI, APP0(JFIF 1.01), DQT, SOF0, DHT, SOS for a w×h image: YCbCr with 2x2/1x1/1x1 (4:2:0) or
// 1x1/1x1/1x1 (4:4:4) sampling — DQT×2, DHT×4 — or one gray component — DQT×1, DHT×2.
std::vector<uint8_t> make_header(int width, int height, const Tables& t, Sampling s = kSampling420);

// Golden single-thread encode of an 8-bit gray plane (complete file bytes): YCbCr 4:2:0 by
// default (Y = gray, Cb = Cr = 128), or 4:4:4, or a one-component gray file.
std::vector<uint8_t> encode_gray(const uint8_t* gray, int width, int height, int stride, int quality,
                                 Sampling s = kSampling420);

// Entropy-coded segment only (stuffed, padded with 1-bits), no markers. Used for tests against
// the GPU encoder and as the engine's fallback for an image the GPU encoder gives up on.
std::vector<uint8_t> encode_scan_gray(const uint8_t* gray, int width, int height, int stride, const Tables& t,
                                      Sampling s = kSampling420);

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
