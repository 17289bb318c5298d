// Host-path microbenchmark: the per-slice CPU cost of each step of the engine's loader and writer,
// single-threaded, over a synthetic cohort (run on tmpfs). Used to decide what to cut from the
// per-slice host work (the bench is host-CPU bound once passes are pipelined).
//   build: see tools/host_path_bench.sh      run: host_path_bench <data_root> <out_dir> [reps]
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "nm03/cohort.h"
#include "nm03/dicom.h"
#include "nm03/jpeg.h"
#include "nm03/pack12.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string root = argv[1], out = argv[2];
  const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
  const std::string base = nm03::cohort::cohort_dir(root);
  std::vector<std::string> files, dirs;
  for (auto& p : nm03::cohort::find_patient_dirs(base)) {
    auto s = nm03::cohort::list_patient_series(base, p);
    for (auto& f : s.files) files.push_back(f);
  }
  std::vector<uint8_t> stage(1 << 20), pk(1 << 20);
  std::vector<uint16_t> dst(1 << 20);
  const size_t nf = files.size();
  auto run = [&](const char* name, auto&& fn) {
    fn(0);  // warm
    double best = 1e9;
    for (int r = 0; r < reps; ++r) {
      const double t0 = now();
      for (size_t i = 0; i < nf; ++i) fn(i);
      best = std::min(best, now() - t0);
    }
    std::printf("%-44s %8.2f us/slice\n", name, best * 1e6 / nf);
  };
  run("open+fstat+close", [&](size_t i) {
    int fd = open(files[i].c_str(), O_RDONLY | O_CLOEXEC);
    struct stat st;
    fstat(fd, &st);
    close(fd);
  });
  run("open+pread(all)+close", [&](size_t i) {
    int fd = open(files[i].c_str(), O_RDONLY | O_CLOEXEC);
    if (pread(fd, stage.data(), stage.size(), 0) < 0) std::abort();
    close(fd);
  });
  run("SliceFile staged header", [&](size_t i) {
    nm03::dicom::SliceFile f(files[i], nm03::dicom::ReadMode::kStaged);
    f.header(stage);
  });
  run("SliceFile staged header + pack12", [&](size_t i) {
    nm03::dicom::SliceFile f(files[i], nm03::dicom::ReadMode::kStaged);
    const auto& h = f.header(stage);
    nm03::pack12::pack(f.staged_samples(), (size_t)h.rows * h.cols, pk.data());
  });
  run("... + stream_copy packed", [&](size_t i) {
    nm03::dicom::SliceFile f(files[i], nm03::dicom::ReadMode::kStaged);
    const auto& h = f.header(stage);
    size_t b = nm03::pack12::pack(f.staged_samples(), (size_t)h.rows * h.cols, pk.data());
    nm03::dicom::stream_copy(dst.data(), pk.data(), b);
  });
  run("staged header + fits12 + pack_stream", [&](size_t i) {
    nm03::dicom::SliceFile f(files[i], nm03::dicom::ReadMode::kStaged);
    const auto& h = f.header(stage);
    const size_t npix = (size_t)h.rows * h.cols;
    if (nm03::pack12::fits12(f.staged_samples(), npix))
      nm03::pack12::pack_stream(f.staged_samples(), npix, reinterpret_cast<uint8_t*>(dst.data()));
  });
  run("SliceFile direct header + pixels16", [&](size_t i) {
    nm03::dicom::SliceFile f(files[i], nm03::dicom::ReadMode::kDirect);
    f.header(stage);
    f.pixels16(dst.data());
  });
  // writer
  nm03::cohort::make_dirs(out);
  std::vector<uint8_t> hdr(623, 0x11), seg(22000, 0x22);
  std::vector<std::string> outs;
  for (size_t i = 0; i < nf; ++i) outs.push_back(out + "/" + std::to_string(i % 20) + "_" + std::to_string(i));
  for (int d = 0; d < 20; ++d) nm03::cohort::make_dirs(out);
  run("write_jpeg_file x2 (open/pwritev/fstat/close)", [&](size_t i) {
    nm03::jpeg::write_jpeg_file(outs[i] + "_a.jpg", hdr, seg.data(), seg.size());
    nm03::jpeg::write_jpeg_file(outs[i] + "_b.jpg", hdr, seg.data(), seg.size());
  });
  const int dfd = open(out.c_str(), O_RDONLY | O_DIRECTORY);
  run("openat+pwritev x2, no fstat", [&](size_t i) {
    for (const char* sfx : {"_a.jpg", "_b.jpg"}) {
      std::string nm = outs[i].substr(out.size() + 1) + sfx;
      int fd = openat(dfd, nm.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      static const uint8_t eoi[2] = {0xFF, 0xD9};
      struct iovec iov[3] = {{(void*)hdr.data(), hdr.size()}, {(void*)seg.data(), seg.size()}, {(void*)eoi, 2}};
      if (pwritev(fd, iov, 3, 0) < 0) std::abort();
      close(fd);
    }
  });
  run("open(path)+pwritev x2, no fstat", [&](size_t i) {
    for (const char* sfx : {"_a.jpg", "_b.jpg"}) {
      int fd = open((outs[i] + sfx).c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      struct iovec iov[2] = {{(void*)hdr.data(), hdr.size()}, {(void*)seg.data(), seg.size()}};
      if (pwritev(fd, iov, 2, 0) < 0) std::abort();
      close(fd);
    }
  });
  run("openat+pwritev+fstat x2", [&](size_t i) {
    for (const char* sfx : {"_a.jpg", "_b.jpg"}) {
      std::string nm = outs[i].substr(out.size() + 1) + sfx;
      int fd = openat(dfd, nm.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      struct iovec iov[2] = {{(void*)hdr.data(), hdr.size()}, {(void*)seg.data(), seg.size()}};
      if (pwritev(fd, iov, 2, 0) < 0) std::abort();
      struct stat st;
      fstat(fd, &st);
      close(fd);
    }
  });
  run("write_jpeg_file x2 again", [&](size_t i) {
    nm03::jpeg::write_jpeg_file(outs[i] + "_a.jpg", hdr, seg.data(), seg.size());
    nm03::jpeg::write_jpeg_file(outs[i] + "_b.jpg", hdr, seg.data(), seg.size());
  });
  run("pwritev x2 only (fds kept open)", [&](size_t i) {
    static std::vector<int> fds;
    if (fds.empty())
      for (size_t k = 0; k < 2 * nf; ++k) fds.push_back(open((outs[k / 2] + (k & 1 ? "_b.jpg" : "_a.jpg")).c_str(), O_WRONLY));
    for (int k = 0; k < 2; ++k) {
      struct iovec iov[2] = {{(void*)hdr.data(), hdr.size()}, {(void*)seg.data(), seg.size()}};
      if (pwritev(fds[2 * i + k], iov, 2, 0) < 0) std::abort();
    }
  });
  run("O_TRUNC rewrite x2", [&](size_t i) {
    for (const char* sfx : {"_a.jpg", "_b.jpg"}) {
      int fd = open((outs[i] + sfx).c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
      struct iovec iov[2] = {{(void*)hdr.data(), hdr.size()}, {(void*)seg.data(), seg.size()}};
      if (pwritev(fd, iov, 2, 0) < 0) std::abort();
      close(fd);
    }
  });
  return 0;
}
