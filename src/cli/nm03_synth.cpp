// nm03_synth — writes the synthetic T1+C cohort that stands in for the TCIA
// Brain-Tumor-Progression data (README.md:98-100), plus the config-4 stress set.
#include <cstdlib>
#include <iostream>
#include <string>

#include "nm03/cohort.h"
#include "nm03/synth.h"

int main(int argc, char** argv) {
  nm03::synth::CohortSpec s;
  s.data_root = nm03::cohort::default_data_root();
  int stress = 0, stress_dim = 512;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto v = [&] { return std::string(argv[++i]); };
    if (a == "--data-root") s.data_root = nm03::cohort::with_slash(v());
    else if (a == "--patients") s.patients = std::atoi(v().c_str());
    else if (a == "--min-slices") s.min_slices = std::atoi(v().c_str());
    else if (a == "--max-slices") s.max_slices = std::atoi(v().c_str());
    else if (a == "--rows") s.rows = std::atoi(v().c_str());
    else if (a == "--cols") s.cols = std::atoi(v().c_str());
    else if (a == "--seed") s.seed = std::strtoull(v().c_str(), nullptr, 10);
    else if (a == "--threads") s.threads = std::atoi(v().c_str());
    else if (a == "--decoy-series") s.decoy_series = true;
    else if (a == "--signed") s.type = nm03::kI16;
    else if (a == "--stress") stress = std::atoi(v().c_str());
    else if (a == "--stress-dim") stress_dim = std::atoi(v().c_str());
    else {
      std::cout << "usage: nm03_synth [--data-root D] [--patients N] [--min-slices A] [--max-slices B]\n"
                   "                  [--rows R] [--cols C] [--seed S] [--threads T] [--decoy-series] [--signed]\n"
                   "                  [--stress COUNT [--stress-dim 512]]\n";
      return a == "--help" ? 0 : 2;
    }
  }
  try {
    size_t n;
    if (stress > 0)
      n = nm03::synth::generate_flat(nm03::cohort::cohort_dir(s.data_root), stress, stress_dim, stress_dim, s.seed, s.threads);
    else
      n = nm03::synth::generate_cohort(s);
    std::cout << "Wrote " << n << " DICOM files under " << s.data_root << std::endl;
  } catch (const std::exception& e) {
    std::cerr << "Fatal error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}
