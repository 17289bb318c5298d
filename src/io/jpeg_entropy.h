// Baseline entropy coding shared by the JPEG codecs of the DICOM importer (ITU T.81): Huffman
// tables (Annex C) with canonical decoding (F.2.2.3) and optimal generation (Annex K.2), and the
// entropy-coded segment's bit reader / writer with 0xFF00 stuffing and restart-marker handling.
// Used by jpeg_lossless.cpp (process 14) and jpeg_dct.cpp (processes 1, 2, 4).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "nm03/common.h"

namespace nm03::jpeg_entropy {

// One Huffman table: DC class (difference categories: 0..11 DCT, 0..16 lossless) or AC class.
struct Table {
  bool defined = false;
  uint8_t bits[17] = {0};  // bits[l]: codes of length l
  uint8_t vals[256] = {0};
  int nvals = 0;
  int32_t mincode[17] = {0}, maxcode[18] = {0}, valptr[17] = {0};
  uint16_t lut[1 << 9] = {0};  // codes ≤ 9 bits: (length << 8) | value, indexed by the next 9 bits
  // encoder side
  uint16_t code_of[256] = {0};
  uint8_t size_of[256] = {0};

  void build() {
    // C.2: sizes and canonical codes in the order of vals.
    int k = 0, code = 0;
    std::memset(lut, 0, sizeof(lut));
    std::memset(size_of, 0, sizeof(size_of));
    for (int l = 1; l <= 16; ++l) {
      if (bits[l]) {
        valptr[l] = k;
        mincode[l] = code;
        for (int i = 0; i < bits[l]; ++i, ++k, ++code) {
          if (code >= (1 << l)) throw SliceError("Corrupt lossless JPEG: Huffman table over-subscribed");
          const uint8_t v = vals[k];
          code_of[v] = (uint16_t)code;
          size_of[v] = (uint8_t)l;
          if (l <= 9)
            for (int e = code << (9 - l); e < (code + 1) << (9 - l); ++e) lut[e] = (uint16_t)((l << 8) | v);
        }
        maxcode[l] = code - 1;
      } else {
        maxcode[l] = -1;
      }
      code <<= 1;
    }
    maxcode[17] = 0x7FFFFFFF;
  }
};

// Entropy-coded segment reader: MSB-first bits, 0xFF00 stuffing removed; a marker stops the input
// (zero bits are supplied past it), and consumed() > real_bits() means the scan ran past its data.
class BitReader {
 public:
  BitReader(const uint8_t* d, size_t n, size_t pos) : d_(d), n_(n), pos_(pos) {}
  uint32_t peek(int k) {
    if (cnt_ < k) fill();
    return (uint32_t)(acc_ >> (64 - k));
  }
  void skip(int k) {
    acc_ <<= k;
    cnt_ -= k;
    consumed_ += (uint64_t)k;
  }
  uint32_t get(int k) {
    if (k == 0) return 0;
    const uint32_t v = peek(k);
    skip(k);
    return v;
  }
  // Restart marker m (0..7) expected next: buffered bits (the padding of the last byte) are dropped.
  void restart(int m) {
    if (consumed_ > real_) throw SliceError("Truncated lossless JPEG data");
    acc_ = 0;
    cnt_ = 0;
    consumed_ = real_ = 0;
    while (pos_ + 1 < n_ && d_[pos_] == 0xFF && d_[pos_ + 1] == 0xFF) ++pos_;  // fill bytes
    if (pos_ + 1 >= n_ || d_[pos_] != 0xFF || d_[pos_ + 1] != 0xD0 + m)
      throw SliceError("Lossless JPEG: missing restart marker RST" + std::to_string(m));
    pos_ += 2;
  }
  void finish() const {
    if (consumed_ > real_) throw SliceError("Truncated lossless JPEG data");
  }

 private:
  void fill() {
    while (cnt_ <= 56) {
      uint8_t b = 0;
      if (pos_ < n_) {
        b = d_[pos_];
        if (b == 0xFF) {
          if (pos_ + 1 < n_ && d_[pos_ + 1] == 0x00) {
            pos_ += 2;
            real_ += 8;
          } else {
            b = 0;  // a marker: stay before it
          }
        } else {
          ++pos_;
          real_ += 8;
        }
      }
      acc_ |= (uint64_t)b << (56 - cnt_);
      cnt_ += 8;
    }
  }
  const uint8_t* d_;
  size_t n_, pos_;
  uint64_t acc_ = 0;
  int cnt_ = 0;
  uint64_t consumed_ = 0, real_ = 0;
};

// One Huffman-coded symbol (F.2.2.3 DECODE, with a 9-bit lookup for short codes).
inline int decode_symbol(const Table& t, BitReader& br) {
  const uint16_t e = t.lut[br.peek(9)];
  if (e) {
    br.skip(e >> 8);
    return e & 0xFF;
  }
  const uint32_t look = br.peek(16);
  for (int l = 10; l <= 16; ++l) {
    const int32_t c = (int32_t)(look >> (16 - l));
    if (c <= t.maxcode[l]) {
      br.skip(l);
      const int idx = t.valptr[l] + c - t.mincode[l];
      if (idx < 0 || idx >= t.nvals) break;
      return t.vals[idx];
    }
  }
  throw SliceError("Corrupt lossless JPEG: bad Huffman code");
}


// T.81 K.2: code lengths from frequencies (≤ 16 bits, no all-ones code), symbols 0..255.
inline void optimal_table(const uint64_t* freq_in, Table& t) {
  uint64_t freq[257];
  int codesize[257], others[257];
  for (int i = 0; i < 256; ++i) freq[i] = freq_in[i];
  freq[256] = 1;  // reserved: no code of all ones
  for (int i = 0; i < 257; ++i) {
    codesize[i] = 0;
    others[i] = -1;
  }
  for (;;) {
    int v1 = -1, v2 = -1;
    for (int i = 0; i < 257; ++i)
      if (freq[i] && (v1 < 0 || freq[i] <= freq[v1])) v1 = i;
    for (int i = 0; i < 257; ++i)
      if (freq[i] && i != v1 && (v2 < 0 || freq[i] <= freq[v2])) v2 = i;
    if (v2 < 0) break;
    freq[v1] += freq[v2];
    freq[v2] = 0;
    ++codesize[v1];
    while (others[v1] >= 0) {
      v1 = others[v1];
      ++codesize[v1];
    }
    others[v1] = v2;
    ++codesize[v2];
    while (others[v2] >= 0) {
      v2 = others[v2];
      ++codesize[v2];
    }
  }
  int bits[64] = {0};
  for (int i = 0; i < 257; ++i)
    if (codesize[i]) ++bits[codesize[i]];
  for (int i = 63; i > 16; --i)  // K.3: limit to 16 bits
    while (bits[i] > 0) {
      int j = i - 2;
      while (bits[j] == 0) --j;
      bits[i] -= 2;
      bits[i - 1] += 1;
      bits[j + 1] += 2;
      bits[j] -= 1;
    }
  int i = 16;
  while (bits[i] == 0) --i;
  bits[i] -= 1;  // the reserved symbol's code
  int k = 0;
  for (int l = 1; l <= 16; ++l) t.bits[l] = (uint8_t)bits[l];
  for (int l = 1; l <= 63; ++l)
    for (int v = 0; v < 256; ++v)
      if (codesize[v] == l) t.vals[k++] = (uint8_t)v;
  t.nvals = k;
  t.build();
  t.defined = true;
}

class BitWriter {
 public:
  explicit BitWriter(std::vector<uint8_t>& o) : o_(o) {}
  void put(uint32_t v, int k) {
    for (int b = k - 1; b >= 0; --b) {
      acc_ = (uint8_t)((acc_ << 1) | ((v >> b) & 1));
      if (++cnt_ == 8) emit();
    }
  }
  void flush_ones() {  // pad the last byte with 1 bits
    while (cnt_) {
      acc_ = (uint8_t)((acc_ << 1) | 1);
      if (++cnt_ == 8) emit();
    }
  }

 private:
  void emit() {
    o_.push_back(acc_);
    if (acc_ == 0xFF) o_.push_back(0x00);
    acc_ = 0;
    cnt_ = 0;
  }
  std::vector<uint8_t>& o_;
  uint8_t acc_ = 0;
  int cnt_ = 0;
};


inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

}  // namespace nm03::jpeg_entropy
