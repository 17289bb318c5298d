#include "nm03/synth.h"

#include <atomic>
#include <cmath>
#include <cstdio>
#include <thread>

#include "nm03/cohort.h"
#include "nm03/dicom.h"

namespace nm03::synth {
namespace {

inline uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() { return splitmix(s); }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  // Irwin–Hall(4) approximation of N(0,1): fast and deterministic.
  float gauss() {
    uint64_t r = next();
    float a = (float)(r & 0xFFFF) + (float)((r >> 16) & 0xFFFF) + (float)((r >> 32) & 0xFFFF) + (float)(r >> 48);
    return (a * (1.0f / 65536.0f) - 2.0f) * 1.7320508f;
  }
};

uint64_t mix(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xD6E8FEB86659FD93ull ^ (c + 17) * 0xCA5A826395121157ull;
  return splitmix(s);
}

}  // namespace

void phantom_slice(int rows, int cols, int patient, int slice, int nslices, uint64_t seed, uint16_t* out) {
  // Per-patient anatomy (independent of the slice), per-slice noise.
  Rng pr(mix(seed, (uint64_t)patient, 0xA11));
  const double W = cols, H = rows;
  const double cx = W * (0.5 + 0.03 * (pr.uni() - 0.5)), cy = H * (0.5 + 0.03 * (pr.uni() - 0.5));
  const double ax = W * (0.36 + 0.04 * pr.uni()), ay = H * (0.43 + 0.04 * pr.uni());
  const double lx = cx + W * 0.06 * (pr.uni() - 0.5), ly = cy + H * 0.06 * (pr.uni() - 0.5);
  const double lr0 = W * (0.13 + 0.07 * pr.uni());  // peak lesion radius
  const double lz = 0.5 + 0.2 * (pr.uni() - 0.5);   // lesion centre along the series
  const double lzr = 0.35 + 0.15 * pr.uni();
  const double rim_level = 1600 + 120 * pr.uni();
  const double bias_phase = 6.283 * pr.uni();
  // Slice geometry: head shrinks towards the ends of the series.
  const double z = nslices > 1 ? (double)slice / (double)(nslices - 1) : 0.5;
  const double head_scale = std::sqrt(std::fmax(0.15, 1.0 - std::pow(2.0 * (z - 0.5), 2) * 0.7));
  const double hx = ax * head_scale, hy = ay * head_scale;
  const double dz = (z - lz) / lzr;
  const double lr = dz * dz < 1.0 ? lr0 * std::sqrt(1.0 - dz * dz) : 0.0;
  Rng nr(mix(seed, (uint64_t)patient, 0xB00 + (uint64_t)slice));
  for (int y = 0; y < rows; ++y) {
    for (int x = 0; x < cols; ++x) {
      const double px = x + 0.5, py = y + 0.5;
      const double ex = (px - cx) / hx, ey = (py - cy) / hy;
      const double e = ex * ex + ey * ey;
      double v;
      if (e > 1.0) {
        v = std::fabs(nr.gauss() * 15.0);  // air: Rician-like magnitude noise
      } else {
        if (e > 0.82) {
          v = 2400.0;  // skull / scalp (above the SRG band)
        } else {
          v = 900.0 + 110.0 * std::sin(bias_phase + 3.0 * px / W + 2.0 * py / H);
          // ventricles
          const double vx1 = (px - (cx - 0.07 * W)) / (0.035 * W), vy1 = (py - cy) / (0.09 * H);
          const double vx2 = (px - (cx + 0.07 * W)) / (0.035 * W);
          if (vx1 * vx1 + vy1 * vy1 < 1.0 || vx2 * vx2 + vy1 * vy1 < 1.0) v = 450.0;
          if (lr > 0.0) {
            const double d = std::sqrt((px - lx) * (px - lx) + (py - ly) * (py - ly));
            if (d < lr) v = d > 0.55 * lr ? rim_level : 1000.0;  // enhancing rim, necrotic core
          }
        }
        v += nr.gauss() * 40.0;
      }
      if (v < 0) v = 0;
      if (v > 65535) v = 65535;
      out[(size_t)y * cols + x] = (uint16_t)std::lround(v);
    }
  }
}

namespace {

std::string uid(uint64_t a, uint64_t b, uint64_t c) {
  char buf[96];
  std::snprintf(buf, sizeof(buf), "1.2.826.0.1.3680043.10.543.%llu.%llu.%llu", (unsigned long long)a,
                (unsigned long long)b, (unsigned long long)c);
  return buf;
}

void write_slice(const std::string& path, int rows, int cols, int patient, int slice, int nslices, uint64_t seed,
                 const std::string& pid, PixelType type, bool rescale) {
  std::vector<uint16_t> px((size_t)rows * cols);
  phantom_slice(rows, cols, patient, slice, nslices, seed, px.data());
  dicom::WriteSpec w;
  w.rows = rows;
  w.cols = cols;
  w.type = type;
  w.bits_stored = 16;
  if (type == kI16)
    for (auto& v : px) v = (uint16_t)(int16_t)std::min<int>(v, 32767);
  w.pixels = px.data();
  w.write_rescale = rescale;
  w.spacing_x = w.spacing_y = 0.9375f;
  w.slice_thickness = 5.0;
  w.instance_number = slice + 1;
  w.position[0] = -120;
  w.position[1] = -120;
  w.position[2] = slice * 5.0;
  w.patient_id = pid;
  w.study_uid = uid(seed, (uint64_t)patient, 1);
  w.series_uid = uid(seed, (uint64_t)patient, 2);
  w.sop_uid = uid(seed, (uint64_t)patient, 100 + (uint64_t)slice);
  dicom::write_file(path, w);
}

}  // namespace

size_t generate_cohort(const CohortSpec& s) {
  const std::string root = cohort::cohort_dir(s.data_root);
  struct Job {
    std::string path, pid;
    int patient, slice, nslices;
  };
  std::vector<Job> jobs;
  for (int p = 0; p < s.patients; ++p) {
    char pid[32];
    std::snprintf(pid, sizeof(pid), "PGBM-%03d", p + 1);
    Rng r(mix(s.seed, (uint64_t)p, 0xC0));
    int n = s.min_slices + (int)(r.next() % (uint64_t)(s.max_slices - s.min_slices + 1));
    char series[64];
    std::snprintf(series, sizeof(series), "%d.000000-T1post-%05d", 10 + p, (int)(r.next() % 100000));
    const std::string sdir = root + pid + "/" + series;
    cohort::make_dirs(sdir);
    if (s.decoy_series) cohort::make_dirs(root + pid + "/zz-decoy-series");
    for (int k = 0; k < n; ++k) {
      char fn[32];
      std::snprintf(fn, sizeof(fn), "1-%02d.dcm", k + 1);
      jobs.push_back({sdir + "/" + fn, pid, p, k, n});
    }
  }
  if (s.test_slice) {
    const std::string tp = cohort::test_slice_path(s.data_root);
    cohort::make_dirs(tp.substr(0, tp.find_last_of('/')));
    jobs.push_back({tp, "PGBM-017", 16, 13, 25});
  }
  std::atomic<size_t> next{0};
  auto worker = [&] {
    for (size_t i; (i = next.fetch_add(1)) < jobs.size();) {
      const Job& j = jobs[i];
      write_slice(j.path, s.rows, s.cols, j.patient, j.slice, j.nslices, s.seed, j.pid, s.type, s.write_rescale);
    }
  };
  std::vector<std::thread> ts;
  int nt = s.threads > 0 ? s.threads : 1;
  for (int t = 0; t < nt; ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  return jobs.size();
}

size_t generate_flat(const std::string& cohort_root, int count, int rows, int cols, uint64_t seed, int threads) {
  const std::string sdir = cohort::with_slash(cohort_root) + "PGBM-STRESS/1.000000-T1post-00000";
  cohort::make_dirs(sdir);
  std::atomic<int> next{0};
  auto worker = [&] {
    for (int i; (i = next.fetch_add(1)) < count;) {
      char fn[32];
      std::snprintf(fn, sizeof(fn), "/1-%d.dcm", i + 1);
      write_slice(sdir + fn, rows, cols, i % 97, i % 25, 25, seed, "PGBM-STRESS", kU16, false);
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < (threads > 0 ? threads : 1); ++t) ts.emplace_back(worker);
  for (auto& t : ts) t.join();
  return (size_t)count;
}

}  // namespace nm03::synth
