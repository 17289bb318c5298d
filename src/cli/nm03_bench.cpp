// nm03_bench — native benchmark driver: the BASELINE configs on the engine without the CLI's
// message catalogue. Prints one JSON line.
//   --config cohort  (2/3)   full synthetic T1+C cohort, end-to-end (read → GPU → JPEG files)
//   --config volume  (5)     one patient series as a volume, 3D SRG + cube dilation
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <string>

#include "nm03/cohort.h"
#include "nm03/engine.h"
#include "nm03/volume.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  std::string config = "cohort", root = nm03::cohort::default_data_root(), out = "/tmp/nm03_bench_out";
  int steps = 10, warmup = 2;
  nm03::EngineConfig ec;
  int dil3d = 7;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto v = [&] { return std::string(argv[++i]); };
    if (a == "--config") config = v();
    else if (a == "--data-root") root = nm03::cohort::with_slash(v());
    else if (a == "--out") out = v();
    else if (a == "--steps") steps = std::atoi(v().c_str());
    else if (a == "--warmup") warmup = std::atoi(v().c_str());
    else if (a == "--batch-size") ec.batch_size = std::atoi(v().c_str());
    else if (a == "--streams") ec.streams = std::atoi(v().c_str());
    else if (a == "--threads") ec.threads = std::atoi(v().c_str());
    else if (a == "--median-window") ec.pipe.median_window = std::atoi(v().c_str());
    else if (a == "--max-dim") ec.max_dim = std::atoi(v().c_str());
    else if (a == "--dilation-3d") dil3d = std::atoi(v().c_str());
    else if (a == "--device") ec.device = std::atoi(v().c_str());
    else {
      std::cerr << "unknown option " << a << std::endl;
      return 2;
    }
  }
  try {
    const std::string base = nm03::cohort::cohort_dir(root);
    auto pids = nm03::cohort::find_patient_dirs(base);
    if (config == "cohort") {
      std::vector<nm03::WorkItem> items;
      for (const auto& p : pids) {
        auto s = nm03::cohort::list_patient_series(base, p);
        const std::string od = out + "/" + p;
        nm03::cohort::make_dirs(od);
        for (const auto& f : s.files) items.push_back({f, od});
      }
      nm03::Engine eng(ec);
      for (int w = 0; w < warmup; ++w) eng.run(items);
      nm03::StageTimes t, acc;
      const double t0 = now_s();
      for (int k = 0; k < steps; ++k) {
        eng.run(items, &t);
        acc.load_s += t.load_s;
        acc.kernels_s += t.kernels_s;
        acc.h2d_s += t.h2d_s;
        acc.write_s += t.write_s;
        acc.slices_ok += t.slices_ok;
      }
      const double dt = now_s() - t0;
      std::cout << "{\"config\": \"cohort\", \"slices_per_step\": " << items.size() << ", \"steps\": " << steps
                << ", \"ms_per_step\": " << dt * 1e3 / steps << ", \"slices_per_s\": " << acc.slices_ok / dt
                << ", \"load_s\": " << acc.load_s << ", \"h2d_s\": " << acc.h2d_s << ", \"kernels_s\": " << acc.kernels_s
                << ", \"write_s\": " << acc.write_s << "}" << std::endl;
    } else if (config == "volume") {
      if (pids.empty()) throw std::runtime_error("no patients");
      auto s = nm03::cohort::list_patient_series(base, pids[0]);
      nm03::VolumeInput v = nm03::load_volume(s.files);
      nm03::VolumeParams vp;
      vp.pipe = ec.pipe;
      vp.dilation_size = dil3d;
      for (int w = 0; w < warmup; ++w) nm03::run_volume(v, vp, ec.device, false);
      double ks = 0;
      int sweeps = 0;
      const double t0 = now_s();
      for (int k = 0; k < steps; ++k) {
        auto r = nm03::run_volume(v, vp, ec.device, false);
        ks += r.kernels_s;
        sweeps = r.sweeps;
      }
      const double dt = now_s() - t0;
      std::cout << "{\"config\": \"volume\", \"dims\": [" << v.w << ", " << v.h << ", " << v.d << "], \"steps\": " << steps
                << ", \"ms_per_volume\": " << dt * 1e3 / steps << ", \"gpu_ms_per_volume\": " << ks * 1e3 / steps
                << ", \"sweeps\": " << sweeps << "}" << std::endl;
    } else {
      throw std::runtime_error("unknown config " + config);
    }
  } catch (const std::exception& e) {
    std::cerr << "Fatal error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
