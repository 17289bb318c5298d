// nm03/jpeg_dct.h — sequential DCT JPEG with Huffman coding (ITU T.81 processes 1, 2 and 4: SOF0 /
// SOF1, 8- and 12-bit samples) for one-component (monochrome) images: the codec behind the DICOM
// transfer syntaxes JPEG Baseline (1.2.840.10008.1.2.4.50) and JPEG Extended (1.2.840.10008.1.2.4.51).
//
// FAST imports through DCMTK (main_sequential.cpp:175-177), whose dcmjpeg codecs decode these
// syntaxes with the IJG library's integer "islow" inverse DCT [F]; SURVEY §2.2 O1. The decoder here
// uses the same islow arithmetic (LL&M, CONST_BITS 13, PASS1_BITS 2 for 8-bit / 1 for 12-bit data,
// IJG's range-limit table), so 8-bit images decode to the bytes libjpeg(-turbo) produces — checked
// against Pillow in tests/test_jpeg_dct.py. Parity with DCMTK itself is unpinned (not in the image).
// This software is based in part on the work of the Independent JPEG Group.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace nm03::jpegdct {

struct Info {
  int precision = 0;  // 8 or 12
  int rows = 0, cols = 0;
  int sof = 0;        // 0 (baseline) or 1 (extended)
  int restart_interval = 0;  // blocks (MCUs) per restart interval, 0: none
};

// Decodes one sequential Huffman-coded DCT JPEG with a single component into rows × cols samples
// (0 .. 2^P − 1). Throws SliceError on malformed input, on other processes (progressive,
// lossless — see jpeg_lossless.h — hierarchical, arithmetic coding) and on several components.
// `expect_rows` / `expect_cols` > 0: the frame must have that size, checked at the SOF before any
// allocation (a DICOM caller knows it: a corrupt SOF cannot make it allocate gigabytes).
Info decode(const uint8_t* data, size_t len, std::vector<uint16_t>& out, int expect_rows = 0, int expect_cols = 0);

// Encodes rows × cols samples of `precision` bits (8: baseline SOF0, 12: extended SOF1) at IJG
// `quality` (the Annex K luminance table scaled like jcparam.c), floating-point forward DCT, optimal
// Huffman tables, a restart marker every `restart_blocks` blocks (0: none). For writer round trips.
std::vector<uint8_t> encode(const uint16_t* px, int rows, int cols, int precision, int quality = 90,
                            int restart_blocks = 0);

}  // namespace nm03::jpegdct
