// Native unit tests of the host runtime (SURVEY §4.2 tier T0/T1, registered with CTest and run by
// tests/test_native_unit.py): cohort naming rules, DICOM round trips through every loader path,
// streaming copies, the JPEG container, golden operators against brute-force definitions, the
// host thread pool, loopback collectives and the wire format, NUMA cpulists and the CLI defaults.
// Host code only — no GPU is touched, so this runs in CPU-only CI.
//
//   build/bin/nm03_unit_tests [filter]      (exit status = number of failed checks)
#include <dirent.h>
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <queue>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "nm03/app.h"
#include "nm03/cohort.h"
#include "nm03/comm.h"
#include "nm03/dicom.h"
#include "nm03/engine.h"
#include "nm03/golden.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg.h"
#include "nm03/jpeg_common.h"
#include "nm03/numa.h"
#include "nm03/pack12.h"
#include "nm03/params.h"
#include "nm03/thread_pool.h"

namespace {

int g_failed = 0, g_checks = 0;
const char* g_test = "";

#define CHECK(cond)                                                                         \
  do {                                                                                      \
    ++g_checks;                                                                             \
    if (!(cond)) {                                                                          \
      ++g_failed;                                                                           \
      std::fprintf(stderr, "FAIL [%s] %s:%d: %s\n", g_test, __FILE__, __LINE__, #cond);     \
    }                                                                                       \
  } while (0)

struct Test {
  const char* name;
  std::function<void()> fn;
};
std::vector<Test>& registry() {
  static std::vector<Test> r;
  return r;
}
struct Reg {
  Reg(const char* n, std::function<void()> f) { registry().push_back({n, std::move(f)}); }
};
#define TEST(name)                      \
  static void name();                   \
  static Reg reg_##name(#name, name);   \
  static void name()

std::string tmpdir() {
  static std::string d = [] {
    char t[] = "/tmp/nm03_unit_XXXXXX";
    const char* p = mkdtemp(t);
    return std::string(p ? p : "/tmp");
  }();
  return d;
}

// ---- cohort naming (main_sequential.cpp:18-30, 93-168) ------------------------------------------
TEST(extract_file_number_rules) {
  using nm03::cohort::extract_file_number;
  CHECK(extract_file_number("1-14.dcm") == 14);
  CHECK(extract_file_number("1-01.dcm") == 1);
  CHECK(extract_file_number("a-b-7.dcm") == 7);
  CHECK(extract_file_number("junk.dcm") == 1000);  // no '-': parse failure → 1000
  CHECK(extract_file_number("1-.dcm") == 1000);
  CHECK(extract_file_number("1-x2.dcm") == 1000);
}

TEST(path_helpers) {
  using namespace nm03::cohort;
  CHECK(with_slash("a/b") == "a/b/");
  CHECK(with_slash("a/b/") == "a/b/");
  CHECK(stem("/x/y/1-14.dcm") == "1-14");
  CHECK(filename("/x/y/1-14.dcm") == "1-14.dcm");
  CHECK(cohort_dir("/d/").find("Brain-Tumor-Progression/T1-Post-Combined-P001-P020") != std::string::npos);
}

TEST(patient_discovery_sorted_and_filtered) {
  using namespace nm03::cohort;
  const std::string root = tmpdir() + "/cohort/";
  for (const char* p : {"PGBM-010", "PGBM-002", "OTHER-1", "PGBM-001"}) make_dirs(root + p + "/series-b");
  make_dirs(root + "PGBM-001/series-a");
  for (int k : {10, 2, 1}) {
    nm03::dicom::WriteSpec ws;
    std::vector<uint16_t> px(16, 7);
    ws.rows = ws.cols = 4;
    ws.pixels = px.data();
    nm03::dicom::write_file(root + "PGBM-001/series-a/1-" + std::to_string(k) + ".dcm", ws);
  }
  const auto ids = find_patient_dirs(root);
  CHECK(ids.size() == 3);
  CHECK(ids.size() == 3 && ids[0] == "PGBM-001" && ids[1] == "PGBM-002" && ids[2] == "PGBM-010");
  const Series s = list_patient_series(root, "PGBM-001");  // sorted series dirs: "series-a" first
  CHECK(s.series_dir.find("series-a") != std::string::npos);
  CHECK(s.files.size() == 3);
  CHECK(s.files.size() == 3 && stem(s.files[0]) == "1-1" && stem(s.files[1]) == "1-2" && stem(s.files[2]) == "1-10");
}

// ---- DICOM ---------------------------------------------------------------------------------------
std::vector<uint16_t> ramp(int n, uint32_t mul) {
  std::vector<uint16_t> v(n);
  for (int i = 0; i < n; ++i) v[i] = (uint16_t)(i * mul + 13);
  return v;
}

TEST(dicom_round_trip_all_syntaxes) {
  using namespace nm03::dicom;
  for (Syntax sx : {Syntax::kExplicitLE, Syntax::kImplicitLE, Syntax::kExplicitBE}) {
    const int rows = 33, cols = 47;
    auto px = ramp(rows * cols, 977);
    WriteSpec ws;
    ws.rows = rows;
    ws.cols = cols;
    ws.pixels = px.data();
    ws.syntax = sx;
    ws.write_rescale = true;
    ws.slope = 2.f;
    ws.intercept = -5.f;
    ws.spacing_x = 0.75f;
    const auto bytes = write(ws);
    const Header h = parse(bytes.data(), bytes.size());
    CHECK(h.rows == rows && h.cols == cols && h.syntax == sx);
    CHECK(h.slope == 2.f && h.intercept == -5.f && h.spacing_x == 0.75f);
    std::vector<uint16_t> got(rows * cols);
    copy_pixels16(h, bytes.data(), bytes.size(), got.data());
    CHECK(got == px);
  }
}

TEST(slice_file_modes_agree) {
  using namespace nm03::dicom;
  const int rows = 128, cols = 160;  // 40 KiB of pixels: larger than the 16 KiB prefix
  auto px = ramp(rows * cols, 31337);
  WriteSpec ws;
  ws.rows = rows;
  ws.cols = cols;
  ws.pixels = px.data();
  const std::string path = tmpdir() + "/slice.dcm";
  write_file(path, ws);
  struct Mode {
    ReadMode m;
    size_t prefix;
  };
  for (Mode md : {Mode{ReadMode::kDirect, 16384}, Mode{ReadMode::kDirect, 1024}, Mode{ReadMode::kStaged, 0},
                  Mode{ReadMode::kMapped, 0}}) {
    SliceFile f(path, md.m, md.prefix);
    std::vector<uint8_t> scratch;
    const Header& h = f.header(scratch);
    CHECK(h.rows == rows && h.cols == cols);
    std::vector<uint16_t> buf(rows * cols + 3, 0xABCD);
    f.pixels16(buf.data() + 3);  // misaligned destination
    CHECK(std::equal(px.begin(), px.end(), buf.begin() + 3));
    CHECK(buf[0] == 0xABCD && buf[2] == 0xABCD);
    CHECK(f.direct() == (md.m == ReadMode::kDirect));
    if (md.m != ReadMode::kDirect) {  // staged / mapped expose the samples in place
      const uint16_t* sm = f.staged_samples();
      CHECK(sm != nullptr && std::equal(px.begin(), px.end(), sm));
    }
  }
}

TEST(slice_file_staged_sizes) {
  // Staged reads take the file size from the whole-file read (no fstat): files below, at and above
  // the 256 KiB first read, with a caller buffer that starts empty, small and already large.
  using namespace nm03::dicom;
  for (int rows : {64, 360, 512}) {  // 8 KiB, ≈253 KiB (just below 256 KiB with the header), 512 KiB
    const int cols = rows == 360 ? 360 : rows;
    auto px = ramp(rows * cols, 4242 + rows);
    WriteSpec ws;
    ws.rows = rows;
    ws.cols = cols;
    ws.pixels = px.data();
    const std::string path = tmpdir() + "/staged_" + std::to_string(rows) + ".dcm";
    write_file(path, ws);
    for (size_t start : {(size_t)0, (size_t)1000, (size_t)(1u << 20)}) {
      std::vector<uint8_t> scratch(start);
      SliceFile f(path, ReadMode::kStaged, 0);
      const Header& h = f.header(scratch);
      CHECK(h.rows == rows && h.cols == cols);
      CHECK(f.size() > (size_t)rows * cols * 2);
      const uint16_t* sm = f.staged_samples();
      CHECK(sm != nullptr && std::equal(px.begin(), px.end(), sm));
    }
  }
}

TEST(duplicate_device_detection) {
  using nm03::RankDevice;
  auto mk = [](const char* bus) {
    RankDevice d;
    d.bus_id = bus;
    return d;
  };
  CHECK(nm03::duplicate_device({mk("0000:0d:00.0"), mk("0000:26:00.0"), mk("0000:f1:00.0")}).empty());
  const std::string m = nm03::duplicate_device({mk("0000:0d:00.0"), mk("0000:26:00.0"), mk("0000:0d:00.0")});
  CHECK(m.find("ranks 0 and 2") != std::string::npos && m.find("0000:0d:00.0") != std::string::npos);
  CHECK(nm03::duplicate_device({mk(""), mk("")}).empty());  // no GPU: nothing to compare
  const std::string j = nm03::rank_devices_json({mk("0000:0d:00.0"), mk("0000:26:00.0")});
  CHECK(j.find("\"bus_id\": [\"0000:0d:00.0\", \"0000:26:00.0\"]") != std::string::npos ||
        j.find("\"bus_id\":[\"0000:0d:00.0\",\"0000:26:00.0\"]") != std::string::npos);
}

TEST(stream_copy_edges) {
  std::vector<uint8_t> src(5000), dst(5100);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (uint8_t)(i * 7 + 1);
  for (size_t off : {0u, 1u, 7u, 15u, 16u, 33u})
    for (size_t n : {0u, 1u, 15u, 63u, 64u, 65u, 1000u, 4999u}) {
      std::fill(dst.begin(), dst.end(), 0);
      nm03::dicom::stream_copy(dst.data() + off, src.data() + 1, n);
      CHECK(std::equal(src.begin() + 1, src.begin() + 1 + n, dst.begin() + off));
      CHECK(dst[off + n] == 0 && (off == 0 || dst[off - 1] == 0));
    }
}

TEST(dicom_rejects_garbage) {
  const std::string junk = "DICM-but-not-really";
  bool threw = false;
  try {
    (void)nm03::dicom::parse(reinterpret_cast<const uint8_t*>(junk.data()), junk.size());
  } catch (const std::exception&) {
    threw = true;
  }
  CHECK(threw);
}

// Mutation fuzz of the reader (tests/test_dicom_fuzz.py does the same through Python): here it runs
// inside tools/sanitize_check.sh's ASan / UBSan builds, which also catch reads past a buffer that
// would not crash. Every syntax and a multi-frame file as seeds; flips, 0xFF runs, truncations,
// small integers over 4-byte fields; deterministic xorshift.
TEST(dicom_mutation_fuzz) {
  using namespace nm03::dicom;
  std::vector<std::vector<uint8_t>> seeds;
  auto px = ramp(3 * 12 * 16, 4093);
  for (auto& v : px) v &= 0x0FFF;
  for (Syntax sx : {Syntax::kExplicitLE, Syntax::kImplicitLE, Syntax::kExplicitBE, Syntax::kDeflatedLE,
                    Syntax::kRleLossless, Syntax::kJpegLossless, Syntax::kJpegExtended})
    for (int frames : {1, 3}) {
      WriteSpec ws;
      ws.rows = 12;
      ws.cols = 16;
      ws.bits_stored = 12;
      ws.frames = frames;
      ws.pixels = px.data();
      ws.syntax = sx;
      seeds.push_back(write(ws));
      if (sx == Syntax::kJpegLossless && frames == 1) {  // restart markers, predictor 7, split fragments
        ws.jpeg_restart_rows = 3;
        ws.jpeg_predictor = 7;
        ws.jpeg_fragments = 2;
        seeds.push_back(write(ws));
      }
    }
  uint64_t r = 0x9E3779B97F4A7C15ull;
  auto rnd = [&](uint64_t n) {
    r ^= r << 13, r ^= r >> 7, r ^= r << 17;
    return n ? r % n : 0;
  };
  int parsed = 0, rejected = 0;
  for (const auto& s : seeds)
    for (int it = 0; it < 1500; ++it) {
      std::vector<uint8_t> b = s;
      switch (rnd(4)) {
        case 0:
          for (int k = 0, n = 1 + (int)rnd(7); k < n; ++k) b[rnd(b.size())] = (uint8_t)rnd(256);
          break;
        case 1: {
          const size_t i = rnd(b.size() - 4);
          for (size_t k = 0, n = 2 + rnd(3); k < n; ++k) b[i + k] = 0xFF;
          break;
        }
        case 2:
          b.resize(rnd(b.size()));
          break;
        default: {
          const size_t i = rnd(b.size() - 4);
          const uint32_t v = (uint32_t)rnd(1u << 20);
          std::memcpy(&b[i], &v, 4);
        }
      }
      try {
        const Header h = parse(b.data(), b.size());
        ++parsed;
        const int frames = std::max(1, h.frames);
        if ((size_t)h.rows * h.cols * frames > ((size_t)1 << 22)) continue;
        std::vector<uint16_t> out((size_t)h.rows * h.cols);
        for (int f = 0; f < frames; ++f) {
          try {
            copy_pixels16(h, b.data(), b.size(), out.data(), f);
          } catch (const std::exception&) {
          }
        }
      } catch (const std::exception&) {
        ++rejected;
      }
    }
  CHECK(parsed > 100 && rejected > 100);
}

TEST(pack12_round_trip_and_declines) {
  using namespace nm03::pack12;
  if (!available()) return;  // no AVX2: the engine ships 16-bit samples
  std::mt19937 rng(12);
  for (size_t n : {16u, 48u, 65536u}) {
    std::vector<uint16_t> px(n);
    for (auto& v : px) v = (uint16_t)(rng() & 0xFFF);
    px[0] = 0xFFF;
    std::vector<uint8_t> packed(n / 2 * 3 + 32, 0xEE);
    CHECK(pack(px.data(), n, packed.data()) == n / 2 * 3);
    std::vector<uint16_t> back(n);
    unpack(packed.data(), n, back.data());
    CHECK(back == px);
    // byte layout: pair k = s[2k] | s[2k+1] << 12, little endian at byte 3k
    const uint32_t v0 = packed[0] | (packed[1] << 8) | (packed[2] << 16);
    CHECK(v0 == ((uint32_t)px[0] | ((uint32_t)px[1] << 12)));
    px[n - 1] = 0x1000;  // one 13-bit sample: shipped unpacked
    CHECK(pack(px.data(), n, packed.data()) == 0);
  }
  std::vector<uint16_t> odd(24, 5);
  std::vector<uint8_t> out(64);
  CHECK(pack(odd.data(), odd.size(), out.data()) == 0);  // n % 16 != 0
  CHECK(!fits12(odd.data(), odd.size()));
}

TEST(pack12_stream_exact_bytes) {
  // pack_stream (the engine's path into pinned memory): same bytes as pack(), at unaligned
  // destinations, across bounce-chunk boundaries, and not one byte past n * 3 / 2.
  using namespace nm03::pack12;
  if (!available()) return;
  std::mt19937 rng(3);
  for (size_t n : {16u, 2048u, 2064u, 65536u, 262144u}) {
    std::vector<uint16_t> px(n);
    for (auto& v : px) v = (uint16_t)(rng() & 0xFFF);
    CHECK(fits12(px.data(), n));
    std::vector<uint8_t> ref(n / 2 * 3 + 32);
    CHECK(pack(px.data(), n, ref.data()) == n / 2 * 3);
    for (size_t mis : {0u, 1u, 8u, 13u}) {
      std::vector<uint8_t> dst(n / 2 * 3 + 64, 0xAB);
      pack_stream(px.data(), n, dst.data() + mis);
      CHECK(std::equal(ref.begin(), ref.begin() + n / 2 * 3, dst.begin() + mis));
      for (size_t k = 0; k < mis; ++k) CHECK(dst[k] == 0xAB);
      for (size_t k = mis + n / 2 * 3; k < dst.size(); ++k) CHECK(dst[k] == 0xAB);
      std::vector<uint8_t> dc(n / 2 * 3 + 64, 0xAB);  // the checked single-pass form
      CHECK(pack_stream_checked(px.data(), n, dc.data() + mis));
      CHECK(std::equal(dst.begin(), dst.end(), dc.begin()));
    }
    std::vector<uint8_t> dc(n / 2 * 3 + 64);
    for (size_t at : {(size_t)0, n / 2, n - 1}) {  // one wide sample anywhere fails the check
      const uint16_t keep = px[at];
      px[at] = 0x1000;
      CHECK(!fits12(px.data(), n));
      CHECK(!pack_stream_checked(px.data(), n, dc.data()));
      px[at] = keep;
    }
    CHECK(!pack_stream_checked(px.data(), n - 8, dc.data()));  // not a multiple of 16: refused
  }
}

// ---- JPEG container ------------------------------------------------------------------------------
TEST(jpeg_container) {
  std::vector<uint8_t> img(64 * 48);
  for (size_t i = 0; i < img.size(); ++i) img[i] = (uint8_t)(i % 251);
  const auto j = nm03::jpeg::encode_gray(img.data(), 64, 48, 64, 75);
  CHECK(j.size() > 200 && j[0] == 0xFF && j[1] == 0xD8);                    // SOI
  CHECK(j[j.size() - 2] == 0xFF && j[j.size() - 1] == 0xD9);                  // EOI
  const auto t = nm03::jpeg::make_tables(75);
  const auto hdr = nm03::jpeg::make_header(64, 48, t);
  CHECK(hdr.size() < j.size() && std::equal(hdr.begin(), hdr.end(), j.begin()));
  // the scan never contains an unstuffed 0xFF followed by a non-zero, non-RST byte
  bool ok = true;
  for (size_t i = hdr.size(); i + 2 < j.size(); ++i)
    if (j[i] == 0xFF && j[i + 1] != 0x00) ok = false;
  CHECK(ok);
}

TEST(xcd_tile_order_is_a_bijection) {
  // Every grid size: each workgroup gets a distinct tile, all tiles are covered, and the workgroups
  // of one XCD (b mod 8) take a contiguous run.
  for (uint32_t n = 1; n <= 2100; ++n) {
    std::vector<int> seen(n, 0);
    std::vector<uint32_t> lo(8, UINT32_MAX), hi(8, 0), cnt(8, 0);
    for (uint32_t b = 0; b < n; ++b) {
      const uint32_t t = nm03::gpu::xcd_tile(b, n);
      CHECK(t < n);
      ++seen[t];
      lo[b & 7] = std::min(lo[b & 7], t);
      hi[b & 7] = std::max(hi[b & 7], t);
      ++cnt[b & 7];
    }
    for (uint32_t t = 0; t < n; ++t) CHECK(seen[t] == 1);
    for (int x = 0; x < 8; ++x)
      if (cnt[x]) CHECK(hi[x] - lo[x] + 1 == cnt[x]);
  }
}

TEST(fdct_dot_form_bit_equal) {
  // fdct_islow_dot (the kernel's v_dot2 form) against the multiply/add islow FDCT: random blocks,
  // extremes, flat blocks, 2x2-duplicated label blocks and single impulses.
  std::mt19937 rng(17);
  auto check = [&](const int32_t* blk) {
    int32_t a[64], b[64];
    std::copy(blk, blk + 64, a);
    std::copy(blk, blk + 64, b);
    nm03::jpeg::fdct_islow(a);
    nm03::jpeg::fdct_islow_dot(b);
    return std::equal(a, a + 64, b);
  };
  int32_t blk[64];
  bool ok = true;
  for (int it = 0; it < 200000 && ok; ++it) {
    const int kind = it % 5;
    for (int i = 0; i < 64; ++i) {
      switch (kind) {
        case 0: blk[i] = (int32_t)(rng() & 255); break;
        case 1: blk[i] = (rng() & 1) ? 255 : 0; break;
        case 2: blk[i] = (int32_t)(it & 255); break;
        case 3: blk[i] = ((i >> 3) + (i & 7)) * 17 % 256; break;
        default: blk[i] = i == (it % 64) ? 255 : 0; break;
      }
    }
    ok = check(blk);
  }
  CHECK(ok);
  for (int v : {0, 255}) {  // checkerboards and stripes at both extremes
    for (int pat = 0; pat < 4 && ok; ++pat) {
      for (int i = 0; i < 64; ++i) {
        const int r = i >> 3, c = i & 7;
        const bool on = pat == 0 ? ((r + c) & 1) : pat == 1 ? (r & 1) : pat == 2 ? (c & 1) : (c < 4) != (r < 4);
        blk[i] = on ? v : 255 - v;
      }
      ok = check(blk);
    }
  }
  CHECK(ok);
}

TEST(jpeg_write_in_place_and_create_hint) {
  // write_jpeg_at: overwrite in place (longer old file cut, shorter grown), and the per-directory
  // hint — existing files opened without O_CREAT, the first missing one flips the directory to
  // create mode — never changes the bytes on disk.
  char tmpl[] = "/tmp/nm03_jw_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  if (!dir) return;
  const int dfd = ::open(dir, O_PATH | O_DIRECTORY | O_CLOEXEC);
  CHECK(dfd >= 0);
  const std::vector<uint8_t> hdr = {0xFF, 0xD8, 1, 2, 3};
  std::vector<uint8_t> big(5000, 0x11), small(7, 0x22);
  auto read_all = [&](const std::string& name) {
    std::vector<uint8_t> b;
    FILE* f = std::fopen((std::string(dir) + "/" + name).c_str(), "rb");
    if (!f) return b;
    int c;
    while ((c = std::fgetc(f)) != EOF) b.push_back((uint8_t)c);
    std::fclose(f);
    return b;
  };
  auto expect = [&](const std::vector<uint8_t>& scan) {
    std::vector<uint8_t> e = hdr;
    e.insert(e.end(), scan.begin(), scan.end());
    e.push_back(0xFF);
    e.push_back(0xD9);
    return e;
  };
  std::atomic<uint8_t> hint{0};
  nm03::jpeg::write_jpeg_at(dfd, dir, "a.jpg", hdr, big.data(), big.size(), &hint);  // missing: created
  CHECK(hint.load() == 1);
  CHECK(read_all("a.jpg") == expect(big));
  std::atomic<uint8_t> hint2{0};
  nm03::jpeg::write_jpeg_at(dfd, dir, "a.jpg", hdr, small.data(), small.size(), &hint2);  // exists: cut
  CHECK(hint2.load() == 0);
  CHECK(read_all("a.jpg") == expect(small));
  nm03::jpeg::write_jpeg_at(dfd, dir, "a.jpg", hdr, big.data(), big.size(), &hint2);  // grown again
  CHECK(read_all("a.jpg") == expect(big));
  nm03::jpeg::write_jpeg_at(dfd, dir, "b.jpg", hdr, small.data(), small.size(), &hint2);  // flips the hint
  CHECK(hint2.load() == 1 && read_all("b.jpg") == expect(small));
  nm03::jpeg::write_jpeg_at(dfd, dir, "a.jpg", hdr, small.data(), small.size(), &hint2);  // create mode, existing
  CHECK(read_all("a.jpg") == expect(small));
  nm03::jpeg::write_jpeg_at(dfd, dir, "c.jpg", hdr, small.data(), small.size(), nullptr);  // no hint
  CHECK(read_all("c.jpg") == expect(small));
  for (const char* n : {"a.jpg", "b.jpg", "c.jpg"}) ::unlinkat(dfd, n, 0);
  ::close(dfd);
  ::rmdir(dir);
}

// ---- golden operators vs brute-force definitions --------------------------------------------------
TEST(golden_median_brute_force) {
  const int w = 23, h = 17;
  std::mt19937 rng(3);
  std::vector<float> img(w * h);
  for (auto& v : img) v = (float)(rng() % 1000);
  for (int k : {3, 5, 7}) {
    const auto m = nm03::golden::median(img, w, h, k);
    bool ok = true;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        std::vector<float> win;
        for (int dy = -k / 2; dy <= k / 2; ++dy)
          for (int dx = -k / 2; dx <= k / 2; ++dx)
            win.push_back(img[std::clamp(y + dy, 0, h - 1) * w + std::clamp(x + dx, 0, w - 1)]);
        std::nth_element(win.begin(), win.begin() + win.size() / 2, win.end());
        ok &= m[y * w + x] == win[win.size() / 2];
      }
    CHECK(ok);
  }
}

std::vector<uint8_t> bfs_grow(const std::vector<uint8_t>& band, int w, int h, const std::vector<nm03::Seed>& seeds,
                              int conn) {
  std::vector<uint8_t> r(w * h, 0);
  std::queue<std::pair<int, int>> q;
  for (const auto& s : seeds)
    if (s.x >= 0 && s.y >= 0 && s.x < w && s.y < h && band[s.y * w + s.x] && !r[s.y * w + s.x]) {
      r[s.y * w + s.x] = 1;
      q.push({s.x, s.y});
    }
  while (!q.empty()) {
    auto [x, y] = q.front();
    q.pop();
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if ((dx == 0 && dy == 0) || (conn == 4 && dx != 0 && dy != 0)) continue;
        const int nx = x + dx, ny = y + dy;
        if (nx < 0 || ny < 0 || nx >= w || ny >= h || !band[ny * w + nx] || r[ny * w + nx]) continue;
        r[ny * w + nx] = 1;
        q.push({nx, ny});
      }
  }
  return r;
}

TEST(golden_region_grow_vs_bfs) {
  const int w = 61, h = 45;
  std::mt19937 rng(9);
  std::vector<uint8_t> band(w * h);
  for (auto& b : band) b = (rng() % 100) < 58;
  const auto seeds = nm03::reference_seeds(w, h);
  for (int conn : {4, 8}) CHECK(nm03::golden::region_grow(band, w, h, seeds, conn) == bfs_grow(band, w, h, seeds, conn));
}

TEST(golden_morphology_brute_force) {
  const int w = 29, h = 21;
  std::mt19937 rng(4);
  std::vector<uint8_t> m(w * h);
  for (auto& b : m) b = (rng() % 100) < 30;
  for (int size : {3, 5}) {
    const auto d = nm03::golden::dilate(m, w, h, size), e = nm03::golden::erode(m, w, h, size);
    bool ok = true;
    const int r = size / 2;
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        int any = 0, all = 1;
        for (int dy = -r; dy <= r; ++dy)
          for (int dx = -r; dx <= r; ++dx) {
            const int nx = x + dx, ny = y + dy;
            if (nx < 0 || ny < 0 || nx >= w || ny >= h) continue;  // out-of-image samples ignored
            any |= m[ny * w + nx];
            all &= m[ny * w + nx];
          }
        ok &= d[y * w + x] == any && e[y * w + x] == all;
      }
    CHECK(ok);
  }
}

TEST(reference_seed_pattern) {
  // centre ± (W/8, H/8) + grid x, y ∈ [W/4, 3W/4) step W/10 (main_sequential.cpp:214-241)
  const auto s = nm03::reference_seeds(256, 256);
  CHECK(s.size() == 41);
  std::set<std::pair<int, int>> uniq;
  for (const auto& p : s) {
    CHECK(p.x >= 0 && p.x < 256 && p.y >= 0 && p.y < 256);
    uniq.insert({p.x, p.y});
  }
  CHECK(uniq.count({128, 128}) == 1);
  CHECK(!nm03::reference_seeds(8, 8).empty());  // step clamped ≥ 1: no infinite loop below 10 px
}

// ---- host runtime ----------------------------------------------------------------------------------
TEST(thread_pool_for_each_exactly_once) {
  nm03::ThreadPool pool(4);
  for (size_t n : {0u, 1u, 3u, 100u, 1000u}) {
    std::vector<std::atomic<int>> hits(n);
    nm03::TaskGroup tg(pool);
    tg.for_each(n, [&](size_t i) { hits[i].fetch_add(1); }, 5);
    tg.wait();
    bool ok = true;
    for (auto& h : hits) ok &= h.load() == 1;
    CHECK(ok);
  }
}

TEST(thread_pool_for_each_max_runners_exactly_once_and_bounded) {
  nm03::ThreadPool pool(6);
  for (int cap : {0, 1, 3, 6, 9}) {
    for (size_t n : {0u, 1u, 7u, 500u}) {
      std::vector<std::atomic<int>> hits(n);
      std::atomic<int> live{0}, peak{0};
      nm03::TaskGroup tg(pool);
      tg.for_each(
          n,
          [&](size_t i) {
            const int now = live.fetch_add(1) + 1;
            int p = peak.load();
            while (now > p && !peak.compare_exchange_weak(p, now)) {
            }
            hits[i].fetch_add(1);
            std::this_thread::sleep_for(std::chrono::microseconds(20));
            live.fetch_sub(1);
          },
          3, nullptr, cap);
      tg.wait();
      bool ok = true;
      for (auto& h : hits) ok &= h.load() == 1;
      CHECK(ok);
      CHECK(peak.load() <= (cap > 0 ? std::min(cap, 6) : 6));
    }
  }
}

TEST(output_reaper_wipes_in_background) {
  char tmpl[] = "/tmp/nm03_reaper_XXXXXX";
  const std::string root = mkdtemp(tmpl);
  std::vector<std::string> dirs;
  for (int d = 0; d < 6; ++d) {
    dirs.push_back(root + "/PGBM-" + std::to_string(d));
    nm03::cohort::make_dirs(dirs.back());
    for (int f = 0; f < 20; ++f) {
      FILE* fp = std::fopen((dirs.back() + "/" + std::to_string(f) + ".jpg").c_str(), "wb");
      std::fputs("x", fp);
      std::fclose(fp);
    }
  }
  {
    nm03::cohort::OutputReaper r(3);
    for (int pass = 0; pass < 3; ++pass) {
      r.wipe(dirs);
      for (auto& d : dirs) {  // empty at once, written right away while the old files are deleted
        FILE* fp = std::fopen((d + "/new.jpg").c_str(), "wb");
        CHECK(fp != nullptr);
        std::fclose(fp);
      }
    }
    r.drain();
    CHECK(r.files_reaped() == 6 * 20 + 2 * 6);
  }
  int entries = 0;
  DIR* dd = opendir(root.c_str());
  while (dirent* e = readdir(dd)) entries += e->d_name[0] != '.';
  closedir(dd);
  CHECK(entries == 6);  // no trash left behind
  nm03::cohort::setup_output_dirs(dirs, 2);
  for (auto& d : dirs) rmdir(d.c_str());
  rmdir(root.c_str());
}

TEST(thread_pool_priorities_order_a_single_worker) {
  nm03::ThreadPool pool(1);
  std::vector<int> order;
  std::mutex m;
  std::atomic<bool> go{false};
  nm03::TaskGroup tg(pool);
  tg.run([&] { while (!go.load()) std::this_thread::yield(); }, 0);  // hold the worker
  for (int p : {5, 1, 3, 1, 0}) tg.run([&, p] { std::lock_guard<std::mutex> g(m); order.push_back(p); }, (uint64_t)p);
  go = true;
  tg.wait();
  CHECK((order == std::vector<int>{0, 1, 1, 3, 5}));
}

TEST(loopback_collectives) {
  for (int n : {1, 2, 4}) {
    auto group = nm03::make_loopback_group(n);
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    for (int r = 0; r < n; ++r)
      th.emplace_back([&, r] {
        nm03::Comm& c = *group[r];
        std::vector<uint8_t> b = r == 0 ? std::vector<uint8_t>{1, 2, 3} : std::vector<uint8_t>{};
        c.broadcast_bytes(b, 0);
        if (b != std::vector<uint8_t>{1, 2, 3}) ++bad;
        const auto all = c.allgather_bytes(std::vector<uint8_t>(r + 1, (uint8_t)r));
        for (int k = 0; k < n; ++k)
          if (all[k] != std::vector<uint8_t>(k + 1, (uint8_t)k)) ++bad;
        int64_t s = r + 1;
        c.allreduce_sum_i64(&s, 1);
        if (s != (int64_t)n * (n + 1) / 2) ++bad;
        double mx = r * 1.5;
        c.allreduce_max_f64(&mx, 1);
        if (mx != (n - 1) * 1.5) ++bad;
        c.barrier();
      });
    for (auto& t : th) t.join();
    CHECK(bad.load() == 0);
  }
}

TEST(wire_format_round_trip) {
  nm03::ByteWriter w;
  w.u32(0xDEADBEEF);
  w.i32(-7);
  w.u64(0x0123456789ABCDEFull);
  w.f64(-2.5);
  w.str("PGBM-017/1-14.dcm");
  w.str("");
  nm03::ByteReader r(w.b.data(), w.b.size());
  CHECK(r.u32() == 0xDEADBEEF);
  CHECK(r.i32() == -7);
  CHECK(r.u64() == 0x0123456789ABCDEFull);
  CHECK(r.f64() == -2.5);
  CHECK(r.str() == "PGBM-017/1-14.dcm");
  CHECK(r.str().empty());
  CHECK(r.pos == w.b.size());
}

TEST(numa_cpulist) {
  using nm03::numa::parse_cpulist;
  CHECK((parse_cpulist("0-3,8,10-11") == std::vector<int>{0, 1, 2, 3, 8, 10, 11}));
  CHECK(parse_cpulist("").empty());
  CHECK((parse_cpulist("5") == std::vector<int>{5}));
}

TEST(cli_defaults_are_reference_literals) {
  char prog[] = "img_processing_parallel";
  char* argv[] = {prog, nullptr};
  const nm03::app::AppConfig c = nm03::app::parse_args(1, argv, "parallel");
  const nm03::PipelineParams& p = c.engine.pipe;
  CHECK(c.engine.batch_size == 25 && c.engine.threads == 16);                       // main_parallel.cpp:33,401
  CHECK(p.median_window == 7 && p.sharpen_mask == 9 && p.sharpen_gain == 2.0f);     // :204-210
  CHECK(p.srg_min == 0.74f && p.srg_max == 0.91f && p.dilation_size == 3);          // :232-252
  CHECK(p.norm_low == 0.5f && p.norm_high == 2.5f && p.clip_min == 0.68f && p.clip_max == 4000.0f);
  CHECK(c.out_dir.find("out-parallel") != std::string::npos);
}

TEST(copy_engine_policy) {
  // --copy-engine auto: shader copies for 2D jobs up to kBlitMaxSlicesPerRank slices per rank (all
  // --repeat passes counted by the caller), unless HSA_ENABLE_SDMA is already set; sdma never
  // touches the environment; blit always sets it; volumes keep the DMA engines under auto.
  using namespace nm03::app;
  const char* saved = std::getenv("HSA_ENABLE_SDMA");
  const std::string keep = saved ? saved : "";
  const char* savedq = std::getenv("GPU_MAX_HW_QUEUES");
  const std::string keepq = savedq ? savedq : "";
  AppConfig c;
  unsetenv("HSA_ENABLE_SDMA");
  setenv("GPU_MAX_HW_QUEUES", "4", 1);  // HIP's default, as the boxes export it
  CHECK(apply_copy_engine(c, 465) && std::string(copy_engine_name()) == "blit");
  CHECK(std::string(std::getenv("GPU_MAX_HW_QUEUES")) == "1");  // --hw-queues auto with shader copies
  unsetenv("HSA_ENABLE_SDMA");
  setenv("GPU_MAX_HW_QUEUES", "3", 1);  // a deliberate choice is kept
  CHECK(apply_copy_engine(c, 465) && std::string(std::getenv("GPU_MAX_HW_QUEUES")) == "3");
  unsetenv("HSA_ENABLE_SDMA");
  unsetenv("GPU_MAX_HW_QUEUES");
  CHECK(!apply_copy_engine(c, kBlitMaxSlicesPerRank + 1) && std::string(copy_engine_name()) == "sdma");
  CHECK(std::getenv("GPU_MAX_HW_QUEUES") == nullptr);  // long jobs: environment untouched
  CHECK(!apply_copy_engine(c, -1));  // unknown size: leave the DMA engines
  setenv("HSA_ENABLE_SDMA", "1", 1);
  CHECK(!apply_copy_engine(c, 10));  // the user's setting wins
  unsetenv("HSA_ENABLE_SDMA");
  c.mode = "3d";
  CHECK(!apply_copy_engine(c, 10));
  c.mode = "2d";
  c.copy_engine = kCopySdma;
  CHECK(!apply_copy_engine(c, 10) && std::getenv("HSA_ENABLE_SDMA") == nullptr);
  c.copy_engine = kCopyBlit;
  CHECK(apply_copy_engine(c, 1 << 20) && std::string(copy_engine_name()) == "blit");
  if (saved)
    setenv("HSA_ENABLE_SDMA", keep.c_str(), 1);
  else
    unsetenv("HSA_ENABLE_SDMA");
  if (savedq)
    setenv("GPU_MAX_HW_QUEUES", keepq.c_str(), 1);
  else
    unsetenv("GPU_MAX_HW_QUEUES");
}

// ---- deferred data plane + start-up hand-off (run under TSan by sanitize_check.sh) --
// Ranks are threads sharing one anonymous segment (its futex barrier and flags work across threads as
// across processes); the data plane is a fake whose readiness, failure and stalls are chosen per rank.
struct FakeSpec {
  bool make_throws = false;   // factory.make fails on this rank
  int ready_after_ms = 0;     // poll_ready true after this long (-1: never)
  bool poll_throws = false;   // poll_ready reports a transport error
  int make_sleep_ms = 0;      // make() blocks this long first
};

class FakeDataPlane final : public nm03::Comm {
 public:
  FakeDataPlane(nm03::Comm* lb, int ready_after_ms, bool poll_throws, std::atomic<int>* aborts)
      : lb_(lb), poll_throws_(poll_throws), aborts_(aborts),
        ready_at_(ready_after_ms < 0 ? std::chrono::steady_clock::time_point::max()
                                     : std::chrono::steady_clock::now() + std::chrono::milliseconds(ready_after_ms)) {}
  int rank() const override { return lb_->rank(); }
  int size() const override { return lb_->size(); }
  const char* backend() const override { return "fake"; }
  void broadcast(void* b, size_t n, int root) override { lb_->broadcast(b, n, root); }
  void allgather(const void* s, size_t n, void* r) override { lb_->allgather(s, n, r); }
  void allreduce_sum_i64(int64_t* v, size_t n) override { lb_->allreduce_sum_i64(v, n); }
  void allreduce_max_f64(double* v, size_t n) override { lb_->allreduce_max_f64(v, n); }
  void barrier() override { lb_->barrier(); }
  void sendrecv(const void* s, size_t sb, int d, void* r, size_t rb, int src) override { lb_->sendrecv(s, sb, d, r, rb, src); }
  bool poll_ready() override {
    if (aborted_) throw nm03::CommError("fake transport was aborted");
    if (poll_throws_) throw nm03::CommError("fake transport error");
    return std::chrono::steady_clock::now() >= ready_at_;
  }
  void abort_transport() override {
    if (!aborted_) aborts_->fetch_add(1);
    aborted_ = true;
  }

 private:
  nm03::Comm* lb_;
  bool poll_throws_;
  std::atomic<int>* aborts_;
  std::chrono::steady_clock::time_point ready_at_;
  bool aborted_ = false;  // start-up thread only (settle), or the main thread after it
};

struct FakeWorld {
  int n;
  std::shared_ptr<nm03::ShmSegment> seg;
  std::vector<std::unique_ptr<nm03::Comm>> lb;  // what the fake transports carry
  std::vector<FakeSpec> spec;
  std::atomic<int> aborts{0}, made{0};
  explicit FakeWorld(int n_) : n(n_), seg(nm03::ShmSegment::create_anonymous(n_, 1 << 16)), lb(nm03::make_loopback_group(n_)),
                               spec((size_t)n_) {}
  nm03::DataPlaneFactory factory() {
    nm03::DataPlaneFactory f;
    f.unique_id = [] { return std::vector<uint8_t>(16, 7); };
    f.make = [this](int r, int, const std::vector<uint8_t>& uid, int, std::shared_ptr<nm03::ShmSegment>, double)
        -> std::unique_ptr<nm03::Comm> {
      if (uid != std::vector<uint8_t>(16, 7)) throw nm03::CommError("bad uid");
      const FakeSpec& sp = spec[(size_t)r];
      if (sp.make_sleep_ms) std::this_thread::sleep_for(std::chrono::milliseconds(sp.make_sleep_ms));
      if (sp.make_throws) throw nm03::CommError("fake make failed on rank " + std::to_string(r));
      made.fetch_add(1);
      return std::make_unique<FakeDataPlane>(lb[(size_t)r].get(), sp.ready_after_ms, sp.poll_throws, &aborts);
    };
    return f;
  }
};

struct RankOutcome {
  std::string backend, fallback, error;
  int64_t sum = 0;
  double promote_s = 0;
};

// Every rank: a start-up thread (start + settle, or fail_data_plane when `fail_start`) while its main
// thread runs a control-plane collective, then promote() and one collective on whatever plane won.
std::vector<RankOutcome> run_fake_world(FakeWorld& w, double timeout_s, std::vector<bool> fail_start = {},
                                        int abort_rank_after_ms = -1) {
  fail_start.resize((size_t)w.n, false);
  std::vector<RankOutcome> out((size_t)w.n);
  std::vector<std::thread> ranks;
  const auto f = w.factory();
  for (int r = 0; r < w.n; ++r)
    ranks.emplace_back([&, r] {
      RankOutcome& o = out[(size_t)r];
      try {
        auto c = nm03::make_deferred_comm(r, w.n, 0, w.seg, timeout_s, f);
        std::atomic<bool> began{false};
        std::thread su([&] {
          if (fail_start[(size_t)r]) {
            c->fail_data_plane("injected start-up failure");
            began.store(true);
          } else {
            began.store(true);  // start_data_plane() moves the state off kIdle before it can block
            c->start_data_plane();
            c->settle_data_plane(nullptr);
          }
        });
        c->barrier();  // control plane meanwhile
        // As in the CLI, promote() comes after the start-up thread's hand-off: a promote() that found
        // the plane idle would start it on this thread (a loaded host could otherwise let rank 0's main
        // thread overtake its injected start-up failure).
        while (!began.load()) std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (abort_rank_after_ms >= 0 && r == 0) {
          std::this_thread::sleep_for(std::chrono::milliseconds(abort_rank_after_ms));
          w.seg->raise_abort(w.n - 1);  // rank n-1 "died" while the others start
        }
        const auto t0 = std::chrono::steady_clock::now();
        try {
          c->promote();
        } catch (const std::exception& e) {
          o.error = e.what();
        }
        o.promote_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        su.join();
        if (o.error.empty()) {
          int64_t v = r + 1;
          c->allreduce_sum_i64(&v, 1);
          o.sum = v;
          o.backend = c->backend();
          o.fallback = c->fallback_error();
        }
      } catch (const std::exception& e) {
        o.error = std::string("outer: ") + e.what();
      }
    });
  for (auto& t : ranks) t.join();
  return out;
}

TEST(deferred_comm_all_ranks_promote) {
  FakeWorld w(4);
  for (int r = 0; r < 4; ++r) w.spec[(size_t)r].ready_after_ms = 5 * r;
  const auto o = run_fake_world(w, 20.0);
  for (const auto& x : o) {
    CHECK(x.error.empty());
    CHECK(x.backend == "fake");
    CHECK(x.fallback.empty());
    CHECK(x.sum == 10);
  }
  CHECK(w.made.load() == 4 && w.aborts.load() == 0);
}

TEST(deferred_comm_one_rank_fails_make_all_fall_back_fast) {
  // one rank failing in make_rccl_comm left the healthy ranks in ready() until the deadline.
  FakeWorld w(3);
  w.spec[1].make_throws = true;
  w.spec[0].ready_after_ms = -1;  // would never be ready by itself: only the failure flag ends its wait
  w.spec[2].ready_after_ms = -1;
  const auto t0 = std::chrono::steady_clock::now();
  const auto o = run_fake_world(w, 30.0);
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (const auto& x : o) {
    CHECK(x.error.empty());
    CHECK(x.backend == "host");
    CHECK(!x.fallback.empty());
    CHECK(x.sum == 6);  // the control plane carries the collective
  }
  CHECK(s < 5.0);
  CHECK(w.aborts.load() == 2);  // the two healthy transports were abandoned
  CHECK(w.seg->data_plane_failed_rank() == 1);
}

TEST(deferred_comm_rank0_startup_failure_unblocks_uid_waiters) {
  // rank 0's start-up failing before start_data_plane left the others in wait_uid().
  FakeWorld w(3);
  const auto t0 = std::chrono::steady_clock::now();
  const auto o = run_fake_world(w, 30.0, {true, false, false});
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  for (const auto& x : o) {
    CHECK(x.error.empty());
    CHECK(x.backend == "host" && !x.fallback.empty() && x.sum == 6);
  }
  CHECK(s < 5.0);
  CHECK(w.made.load() == 0);
}

TEST(deferred_comm_stalled_rank_times_out_and_all_fall_back) {
  FakeWorld w(3);
  w.spec[2].ready_after_ms = -1;  // never ready: its own settle times out
  w.spec[0].ready_after_ms = -1;  // the others only become ready with every peer (as RCCL's bootstrap)
  w.spec[1].ready_after_ms = -1;
  const auto o = run_fake_world(w, 0.5);
  for (const auto& x : o) {
    CHECK(x.error.empty());
    CHECK(x.backend == "host" && !x.fallback.empty() && x.sum == 6);
  }
  CHECK(w.aborts.load() == 3);
}

TEST(deferred_comm_transport_error_falls_back) {
  FakeWorld w(2);
  w.spec[0].poll_throws = true;
  w.spec[1].ready_after_ms = -1;
  const auto o = run_fake_world(w, 30.0);
  for (const auto& x : o) CHECK(x.error.empty() && x.backend == "host" && x.sum == 3);
}

TEST(deferred_comm_peer_abort_during_start_ends_the_job) {
  // A dead peer is not a fallback: promote() throws on every live rank once the abort flag is up,
  // while start-up threads are still inside make() / settle.
  FakeWorld w(3);
  for (auto& sp : w.spec) {
    sp.make_sleep_ms = 100;
    sp.ready_after_ms = -1;
  }
  const auto o = run_fake_world(w, 30.0, {}, 20);
  for (const auto& x : o) CHECK(!x.error.empty());
  CHECK(w.seg->aborted() && w.seg->abort_rank() == 2);
}

TEST(engine_startup_hands_over_and_settles_first) {
  // The start-up thread settles the data plane before it builds; build() sees the hook's engine.
  FakeWorld w(1);
  w.spec[0].ready_after_ms = 30;
  auto c = nm03::make_deferred_comm(0, 1, 0, w.seg, 10.0, w.factory());
  std::atomic<int> order{0};
  int prepared_at = -1, built_at = -1;
  nm03::app::EngineStartup::Hooks h;
  h.prepare = [&](nm03::app::EngineStartup::Times& t) {
    prepared_at = order++;
    t.hip_init_s = 0.001;
  };
  h.build = [&](const nm03::EngineConfig& ec) {
    built_at = order++;
    return std::make_unique<nm03::Engine>(ec);
  };
  nm03::EngineConfig ec;
  ec.host_only = true;
  ec.threads = 1;
  ec.streams = 1;
  ec.batch_size = 1;
  ec.max_dim = 64;
  std::unique_ptr<nm03::Engine> e;
  std::string err;
  {
    nm03::app::EngineStartup su(h, c.get());
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
    e = su.build(ec, &err);
    CHECK(su.times().data_plane_s >= 0.02);  // waited for the transport before building
    CHECK(su.times().engine_ctor_s > 0);
  }
  CHECK(err.empty() && e != nullptr);
  CHECK(prepared_at == 0 && built_at == 1);
  c->promote();
  CHECK(std::string(c->backend()) == "fake");
  CHECK(c->data_plane_times().settle_s >= 0.02);
}

TEST(engine_startup_prepare_failure_tells_peers) {
  FakeWorld w(2);
  w.spec[1].ready_after_ms = -1;
  auto c0 = nm03::make_deferred_comm(0, 2, 0, w.seg, 30.0, w.factory());
  auto c1 = nm03::make_deferred_comm(1, 2, 0, w.seg, 30.0, w.factory());
  nm03::app::EngineStartup::Hooks bad, good;
  bad.prepare = [](nm03::app::EngineStartup::Times&) { throw std::runtime_error("injected hipInit failure"); };
  bad.build = [](const nm03::EngineConfig&) -> std::unique_ptr<nm03::Engine> { return nullptr; };
  good.prepare = [](nm03::app::EngineStartup::Times&) {};
  good.build = [](const nm03::EngineConfig&) -> std::unique_ptr<nm03::Engine> { return nullptr; };
  const auto t0 = std::chrono::steady_clock::now();
  std::string err0, err1, b0, b1;
  std::thread r1([&] {
    nm03::app::EngineStartup su(good, c1.get());
    nm03::EngineConfig ec;
    (void)su.build(ec, &err1);
    c1->promote();
    b1 = c1->backend();
  });
  {
    nm03::app::EngineStartup su(bad, c0.get());
    nm03::EngineConfig ec;
    (void)su.build(ec, &err0);
    c0->promote();
    b0 = c0->backend();
  }
  r1.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(err0.find("injected hipInit failure") != std::string::npos);
  CHECK(err1 == "engine not built");
  CHECK(b0 == "host" && b1 == "host");
  CHECK(s < 5.0);
}

TEST(engine_startup_cancel_while_settling) {
  // Destroyed without build() while its data plane can never become ready: cancel ends the settle.
  FakeWorld w(1);
  w.spec[0].ready_after_ms = -1;
  auto c = nm03::make_deferred_comm(0, 1, 0, w.seg, 60.0, w.factory());
  nm03::app::EngineStartup::Hooks h;
  h.prepare = [](nm03::app::EngineStartup::Times&) {};
  h.build = [](const nm03::EngineConfig&) -> std::unique_ptr<nm03::Engine> { return nullptr; };
  const auto t0 = std::chrono::steady_clock::now();
  {
    nm03::app::EngineStartup su(h, c.get());
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  CHECK(s < 2.0);
  CHECK(w.aborts.load() == 1);
  c->promote();  // one rank: agrees with itself on the fallback
  CHECK(std::string(c->backend()) == "host");
}

}  // namespace

int main(int argc, char** argv) {
  const std::string filter = argc > 1 ? argv[1] : "";
  int run = 0;
  for (const Test& t : registry()) {
    if (!filter.empty() && std::string(t.name).find(filter) == std::string::npos) continue;
    g_test = t.name;
    const int before = g_failed;
    try {
      t.fn();
    } catch (const std::exception& e) {
      ++g_failed;
      std::fprintf(stderr, "FAIL [%s] exception: %s\n", t.name, e.what());
    }
    std::printf("%s %s\n", g_failed == before ? "ok  " : "FAIL", t.name);
    ++run;
  }
  std::printf("%d tests, %d checks, %d failed\n", run, g_checks, g_failed);
  std::string cleanup = "rm -rf " + tmpdir();
  if (tmpdir().rfind("/tmp/nm03_unit_", 0) == 0) (void)std::system(cleanup.c_str());
  return g_failed ? 1 : 0;
}
