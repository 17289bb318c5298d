// nm03/jpeg_lossless.h — lossless JPEG (ITU T.81 Annex H, process 14: SOF3, Huffman coding,
// predictors 1–7, point transform) for one-component images: the codec behind the DICOM transfer
// syntaxes JPEG Lossless First-Order Prediction (1.2.840.10008.1.2.4.70, selection value 1) and
// JPEG Lossless Process 14 (1.2.840.10008.1.2.4.57, any selection value).
//
// FAST imports DICOM through DCMTK (main_sequential.cpp:175-177), whose dcmjpeg codecs decode these
// syntaxes [F]; SURVEY §2.2 O1. Written from the standard; parity with DCMTK is unpinned (neither
// DCMTK nor pydicom is in the image and the reference ships no fixtures): the tests check the
// decoder against this encoder, against an independent Python encoder of the same standard, and the
// engine's outputs against the plain encoding of the same samples.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace nm03::jpegll {

struct Info {
  int precision = 0;        // P, 2..16 bits
  int rows = 0, cols = 0;
  int predictor = 0;        // selection value Ss, 1..7
  int point_transform = 0;  // Al
  int restart_interval = 0; // samples per restart interval (0: none)
};

// Decodes one lossless JPEG image (SOI … EOI) into rows × cols samples (each < 2^P, shifted left by
// the point transform). Throws SliceError on malformed input, other JPEG processes (baseline,
// progressive, arithmetic coding, hierarchical), several components, restart intervals that do not
// span whole rows, or a stream shorter than its image.
// `expect_rows` / `expect_cols` > 0: the frame must have that size (checked at the SOF, before any
// allocation).
Info decode(const uint8_t* data, size_t len, std::vector<uint16_t>& out, int expect_rows = 0, int expect_cols = 0);

// Encodes rows × cols samples (only the low `precision` bits are used) with selection value
// `predictor` (1..7), point transform `pt` and a restart marker every `restart_rows` rows (0: none);
// Huffman table optimised for the image (T.81 Annex K.2).
std::vector<uint8_t> encode(const uint16_t* px, int rows, int cols, int precision, int predictor = 1, int pt = 0,
                            int restart_rows = 0);

}  // namespace nm03::jpegll
