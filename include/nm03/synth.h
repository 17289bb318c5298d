// nm03/synth.h — deterministic synthetic T1+C cohort. The TCIA
// Brain-Tumor-Progression data used by the reference (README.md:98-100) is not available offline,
// so every test and benchmark runs on phantoms of the same shape and directory layout:
//   <root>/Brain-Tumor-Progression/T1-Post-Combined-P001-P020/PGBM-0NN/<series>/1-KK.dcm
// plus the fixed test_pipeline slice (test_pipeline.cpp:33-36).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "nm03/common.h"

namespace nm03::synth {

struct CohortSpec {
  std::string data_root = "../data/";
  int patients = 20;
  int min_slices = 21, max_slices = 25;
  int rows = 256, cols = 256;
  uint64_t seed = 20250404;
  int threads = 8;
  bool test_slice = true;      // also write the fixed test_pipeline file
  bool decoy_series = false;   // add a second (lexicographically later) series dir per patient
  PixelType type = kU16;
  bool write_rescale = false;  // write RescaleSlope/Intercept = 1/0 tags
};

// Render one phantom slice (rows×cols raw 16-bit samples).
//   background ≈ |N(0,15)|, skull ring ≈ 2400, brain ≈ 900±bias, ventricles ≈ 450,
//   ring-enhancing lesion: rim ≈ 1650 (inside the SRG band after normalisation), core ≈ 1000,
//   additive noise σ = 40; deterministic per (seed, patient, slice).
void phantom_slice(int rows, int cols, int patient, int slice, int nslices, uint64_t seed, uint16_t* out);

// Writes the cohort; returns the number of files written.
size_t generate_cohort(const CohortSpec& spec);

// Flat stress set (config 4): <dir>/PGBM-STRESS/<series>/1-N.dcm, `count` slices of rows×cols.
size_t generate_flat(const std::string& cohort_root, int count, int rows, int cols, uint64_t seed, int threads);

}  // namespace nm03::synth
