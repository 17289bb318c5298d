// I/O probe: per-file costs of the engine's loader and writer paths on the current filesystem,
// single-threaded and with N threads. Build: see tools/gpu_io.sh.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "nm03/cohort.h"
#include "nm03/dicom.h"
#include "nm03/jpeg.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const std::string root = argv[1], out = argv[2];
  const int threads = argc > 3 ? std::atoi(argv[3]) : 16;
  const std::string base = nm03::cohort::cohort_dir(root);
  std::vector<std::string> files;
  for (auto& p : nm03::cohort::find_patient_dirs(base))
    for (auto& f : nm03::cohort::list_patient_series(base, p).files) files.push_back(f);
  nm03::cohort::make_dirs(out);
  std::vector<uint8_t> hdr(623, 0x11), seg(15000, 0x22);
  for (int d = 0; d < 20; ++d) nm03::cohort::make_dirs(out + "/d" + std::to_string(d));
  for (int nt : {1, 4, 8, threads}) {
    for (int rep = 0; rep < 2; ++rep) {
      std::atomic<size_t> next{0};
      const int odfd = open(out.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
      auto work = [&](int phase) {
        std::vector<uint8_t> scratch;
        std::vector<uint16_t> px(512 * 512);
        for (size_t i; (i = next.fetch_add(1)) < files.size();) {
          if (phase == 0) {
            nm03::dicom::SliceFile sf(files[i]);
            sf.header(scratch);
            sf.pixels16(px.data());
          } else if (phase == 1) {  // like the engine: 20 patient directories
            const std::string b = out + "/d" + std::to_string(i % 20) + "/" + std::to_string(i);
            nm03::jpeg::write_jpeg_file(b + "_a.jpg", hdr, seg.data(), seg.size());
            nm03::jpeg::write_jpeg_file(b + "_b.jpg", hdr, seg.data(), seg.size());
          } else {  // phase 2: same writes relative to a directory fd (openat)
            for (const char* sfx : {"_a.jpg", "_b.jpg"}) {
              const std::string nm = std::to_string(i) + sfx;
              const int fd = openat(odfd, nm.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
              if (pwrite(fd, seg.data(), seg.size(), 0) < 0) std::abort();
              struct stat st;
              fstat(fd, &st);
              close(fd);
            }
          }
        }
      };
      double t[3];
      for (int phase = 0; phase < 3; ++phase) {
        next = 0;
        const double t0 = now();
        std::vector<std::thread> th;
        for (int k = 0; k < nt; ++k) th.emplace_back(work, phase);
        for (auto& x : th) x.join();
        t[phase] = now() - t0;
      }
      close(odfd);
      std::printf("{\"threads\": %d, \"load_us_per_slice\": %.2f, \"write_us_per_slice_pair\": %.2f, "
                  "\"write_openat_us_per_pair\": %.2f, \"load_slices_per_s\": %.0f, \"write_pairs_per_s\": %.0f}\n",
                  nt, t[0] * 1e6 * nt / files.size(), t[1] * 1e6 * nt / files.size(), t[2] * 1e6 * nt / files.size(),
                  files.size() / t[0], files.size() / t[1]);
    }
  }
}
