// Host JPEG pieces: marker writer and the golden CPU encoder. The GPU path in
// src/kernels/k4_jpeg.hip must produce the same entropy-coded bytes as encode_scan_gray.
#include "nm03/jpeg.h"

#include <fcntl.h>

#include <atomic>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace nm03::jpeg {

Tables make_tables(int quality) {
  Tables t;
  t.quality = quality;
  quality_table(kStdLuma, quality, t.qluma);
  quality_table(kStdChroma, quality, t.qchroma);
  for (int i = 0; i < 64; ++i) {
    t.div_luma[i] = (int32_t)t.qluma[i] * 8;
    t.div_chroma[i] = (int32_t)t.qchroma[i] * 8;
  }
  return t;
}

namespace {

void put16(std::vector<uint8_t>& b, int v) {
  b.push_back((uint8_t)(v >> 8));
  b.push_back((uint8_t)v);
}

void put_dqt(std::vector<uint8_t>& b, int id, const uint16_t* q) {
  b.push_back(0xFF);
  b.push_back(0xDB);
  put16(b, 2 + 1 + 64);
  b.push_back((uint8_t)id);
  for (int k = 0; k < 64; ++k) b.push_back((uint8_t)q[kNatural[k]]);
}

void put_dht(std::vector<uint8_t>& b, int cls_id, const uint8_t* bits, const uint8_t* vals) {
  int n = 0;
  for (int i = 0; i < 16; ++i) n += bits[i];
  b.push_back(0xFF);
  b.push_back(0xC4);
  put16(b, 2 + 1 + 16 + n);
  b.push_back((uint8_t)cls_id);
  for (int i = 0; i < 16; ++i) b.push_back(bits[i]);
  for (int i = 0; i < n; ++i) b.push_back(vals[i]);
}

// MSB-first bit writer with 0xFF byte stuffing (libjpeg emit_bits / flush_bits semantics).
struct BitWriter {
  std::vector<uint8_t>& out;
  uint64_t acc = 0;
  int n = 0;
  explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
  void put(uint32_t code, int len) {
    if (len == 0) return;
    acc = (acc << len) | (code & ((1u << len) - 1u));
    n += len;
    while (n >= 8) {
      uint8_t byte = (uint8_t)(acc >> (n - 8));
      out.push_back(byte);
      if (byte == 0xFF) out.push_back(0x00);
      n -= 8;
    }
  }
  void flush() {
    if (n > 0) put(0x7F, 8 - n);  // pad the last byte with 1-bits (libjpeg flush_bits)
    acc = 0;
    n = 0;
  }
};

void encode_block(BitWriter& w, const int16_t* zz, int& last_dc, const HuffEnc& dc, const HuffEnc& ac) {
  int diff = zz[0] - last_dc;
  last_dc = zz[0];
  int nb = mag_bits(diff);
  w.put(dc.e[nb] & 0xFFFF, (int)(dc.e[nb] >> 16));
  if (nb) w.put((uint32_t)(diff < 0 ? diff - 1 : diff), nb);
  int run = 0;
  for (int k = 1; k < 64; ++k) {
    int v = zz[k];
    if (v == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      w.put(ac.e[0xF0] & 0xFFFF, (int)(ac.e[0xF0] >> 16));
      run -= 16;
    }
    int n = mag_bits(v);
    uint32_t sym = ac.e[(run << 4) + n];
    w.put(sym & 0xFFFF, (int)(sym >> 16));
    w.put((uint32_t)(v < 0 ? v - 1 : v), n);
    run = 0;
  }
  if (run > 0) w.put(ac.e[0] & 0xFFFF, (int)(ac.e[0] >> 16));
}

}  // namespace

std::vector<uint8_t> make_header(int width, int height, const Tables& t, Sampling s) {
  const bool gray = s == kSamplingGray;
  const int nc = gray ? 1 : 3;
  std::vector<uint8_t> b;
  b.reserve(700);
  b.push_back(0xFF);
  b.push_back(0xD8);  // SOI
  // APP0 JFIF 1.01, no units, 1:1 density, no thumbnail (libjpeg defaults).
  const uint8_t app0[] = {0xFF, 0xE0, 0x00, 0x10, 'J', 'F', 'I', 'F', 0x00, 0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
  b.insert(b.end(), app0, app0 + sizeof(app0));
  // libjpeg writes the tables the frame's components use: DQT before SOF0, DHT (per scan
  // component: DC then AC, each table once) before SOS.
  put_dqt(b, 0, t.qluma);
  if (!gray) put_dqt(b, 1, t.qchroma);
  // SOF0
  b.push_back(0xFF);
  b.push_back(0xC0);
  put16(b, 8 + 3 * nc);
  b.push_back(8);
  put16(b, height);
  put16(b, width);
  b.push_back((uint8_t)nc);
  const uint8_t comps[9] = {1, (uint8_t)(s == kSampling420 ? 0x22 : 0x11), 0, 2, 0x11, 1, 3, 0x11, 1};
  b.insert(b.end(), comps, comps + 3 * nc);
  put_dht(b, 0x00, kDcLumaBits, kDcLumaVals);
  put_dht(b, 0x10, kAcLumaBits, kAcLumaVals);
  if (!gray) {
    put_dht(b, 0x01, kDcChromaBits, kDcChromaVals);
    put_dht(b, 0x11, kAcChromaBits, kAcChromaVals);
  }
  // SOS
  b.push_back(0xFF);
  b.push_back(0xDA);
  put16(b, 6 + 2 * nc);
  b.push_back((uint8_t)nc);
  const uint8_t sos[6] = {1, 0x00, 2, 0x11, 3, 0x11};
  b.insert(b.end(), sos, sos + 2 * nc);
  b.push_back(0);
  b.push_back(63);
  b.push_back(0);
  return b;
}

namespace {

// Luma block (bx, by) of the gray plane, edge-replicated past the image (libjpeg's
// expand_right_edge and bottom-row replication), transformed and quantised into zig-zag order.
void luma_block(const uint8_t* gray, int width, int height, int stride, int bx, int by, const Tables& t, int16_t* zz) {
  int32_t blk[64];
  for (int r = 0; r < 8; ++r) {
    const int y = by * 8 + r < height ? by * 8 + r : height - 1;
    for (int c = 0; c < 8; ++c) {
      const int x = bx * 8 + c < width ? bx * 8 + c : width - 1;
      blk[r * 8 + c] = (int32_t)gray[(size_t)y * stride + x] - 128;
    }
  }
  fdct_islow(blk);
  for (int k = 0; k < 64; ++k) zz[k] = quantize(blk[kNatural[k]], t.div_luma[kNatural[k]]);
}

}  // namespace

std::vector<uint8_t> encode_scan_gray(const uint8_t* gray, int width, int height, int stride, const Tables& t,
                                      Sampling s) {
  std::vector<uint8_t> out;
  out.reserve((size_t)width * height / 8);
  BitWriter w(out);
  const int bw = (width + 7) / 8, bh = (height + 7) / 8;
  int last_dc_y = 0, last_dc_cb = 0, last_dc_cr = 0;
  int16_t zz[64];
  int16_t zero_zz[64] = {0};
  if (s != kSampling420) {
    // One luma block per MCU in raster order (a one-component scan is never interleaved; 4:4:4
    // interleaves the Y, Cb and Cr blocks of each 8×8 MCU). No padding blocks.
    for (int by = 0; by < bh; ++by)
      for (int bx = 0; bx < bw; ++bx) {
        luma_block(gray, width, height, stride, bx, by, t, zz);
        encode_block(w, zz, last_dc_y, kHuffDcLuma, kHuffAcLuma);
        if (s == kSampling444) {
          encode_block(w, zero_zz, last_dc_cb, kHuffDcChroma, kHuffAcChroma);
          encode_block(w, zero_zz, last_dc_cr, kHuffDcChroma, kHuffAcChroma);
        }
      }
    w.flush();
    return out;
  }
  // 4:2:0: libjpeg pads each component to whole blocks by edge replication and fills MCU padding
  // with dummy blocks whose DC repeats the previous block (jccoefct.c compress_data).
  const int mcux = (width + 15) / 16, mcuy = (height + 15) / 16;
  for (int my = 0; my < mcuy; ++my) {
    for (int mx = 0; mx < mcux; ++mx) {
      for (int sub = 0; sub < 4; ++sub) {
        const int by = my * 2 + (sub >> 1), bx = mx * 2 + (sub & 1);
        if (by < bh && bx < bw) {
          luma_block(gray, width, height, stride, bx, by, t, zz);
        } else {
          // Dummy block: zero AC, DC = previous block's DC in this MCU row of the component.
          std::memset(zz, 0, sizeof(zz));
          zz[0] = (int16_t)last_dc_y;
        }
        encode_block(w, zz, last_dc_y, kHuffDcLuma, kHuffAcLuma);
      }
      // Cb, Cr: constant 128 → all-zero blocks.
      encode_block(w, zero_zz, last_dc_cb, kHuffDcChroma, kHuffAcChroma);
      encode_block(w, zero_zz, last_dc_cr, kHuffDcChroma, kHuffAcChroma);
    }
  }
  w.flush();
  return out;
}

std::vector<uint8_t> encode_gray(const uint8_t* gray, int width, int height, int stride, int quality, Sampling s) {
  Tables t = make_tables(quality);
  std::vector<uint8_t> f = make_header(width, height, t, s);
  std::vector<uint8_t> sc = encode_scan_gray(gray, width, height, stride, t, s);
  f.insert(f.end(), sc.begin(), sc.end());
  f.push_back(0xFF);
  f.push_back(0xD9);
  return f;
}

void write_jpeg_file(const std::string& path, const std::vector<uint8_t>& header, const uint8_t* scan, size_t scan_len) {
  write_jpeg_at(AT_FDCWD, "", path, header, scan, scan_len);
}

void write_jpeg_at(int dirfd, const std::string& dir, const std::string& name, const std::vector<uint8_t>& header,
                   const uint8_t* scan, size_t scan_len, std::atomic<uint8_t>* creating) {
  auto path = [&] { return dir.empty() ? name : dir + "/" + name; };
  // Overwrite in place instead of O_TRUNC: re-exporting a cohort rewrites files of (nearly) the
  // same size, and truncate + reallocate costs 4-12x more than pwrite on ext4/overlayfs. The old
  // tail is cut only when the previous file was longer, so the bytes on disk are identical.
  // O_CREAT makes open() take the directory's inode lock exclusively (kernels before 6.12 even
  // when the file exists), which serialises every writer of a patient directory: with a
  // per-directory hint, existing files are opened without it first, and once a directory is seen
  // to be empty (a fresh or wiped output tree) its files are created directly.
  // A file this call creates (O_EXCL) is empty, so its size needs no fstat afterwards.
  int fd = -1;
  bool fresh = false;
  if (creating && creating->load(std::memory_order_relaxed) != 1) {
    fd = ::openat(dirfd, name.c_str(), O_WRONLY | O_CLOEXEC);
    if (fd < 0 && errno == ENOENT) creating->store(1, std::memory_order_relaxed);
  }
  if (fd < 0 && creating) {
    fd = ::openat(dirfd, name.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0644);
    fresh = fd >= 0;
  }
  if (fd < 0) fd = ::openat(dirfd, name.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("Cannot create " + path() + ": " + std::strerror(errno));
  static const uint8_t eoi[2] = {0xFF, 0xD9};
  struct iovec iov[3] = {{(void*)header.data(), header.size()}, {(void*)scan, scan_len}, {(void*)eoi, 2}};
  const size_t total = header.size() + scan_len + 2;
  size_t done = 0;
  int idx = 0;
  while (done < total) {
    ssize_t w = ::pwritev(fd, iov + idx, 3 - idx, (off_t)done);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) {
      ::close(fd);
      throw std::runtime_error("Write failed: " + path());
    }
    done += (size_t)w;
    size_t adv = (size_t)w;
    while (idx < 3 && adv >= iov[idx].iov_len) {
      adv -= iov[idx].iov_len;
      ++idx;
    }
    if (idx < 3) {
      iov[idx].iov_base = (uint8_t*)iov[idx].iov_base + adv;
      iov[idx].iov_len -= adv;
    }
  }
  // The previous file's size by lseek(SEEK_END) (an fstat copies a whole struct stat: 1.3% of the
  // pool's CPU in the round-6 profile).
  const off_t end = fresh ? 0 : ::lseek(fd, 0, SEEK_END);
  if (end > (off_t)total && ftruncate(fd, (off_t)total) != 0) {
    ::close(fd);
    throw std::runtime_error("Truncate failed: " + path());
  }
  ::close(fd);
}

}  // namespace nm03::jpeg
