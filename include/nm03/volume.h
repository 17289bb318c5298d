// nm03/volume.h — 3D mode (BASELINE config 5): a patient series loaded as one volume
// (the reference forces 2D with setLoadSeries(false), test_pipeline.cpp:38-41; FAST itself
// supports 3D SeededRegionGrowing/Dilation, which this mode provides on the GPU).
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "nm03/app.h"
#include "nm03/comm.h"
#include "nm03/engine.h"

namespace nm03 {

struct VolumeInput {
  int w = 0, h = 0, d = 0;
  PixelType type = kU16;
  int stored_bits = 16;
  float slope = 1.f, intercept = 0.f, spacing_x = 1.f, spacing_y = 1.f;
  std::vector<uint16_t> raw;  // d planes of h×w
};

// Load a series directory's slices (ordered like the 2D path) as a volume; all slices must share
// dimensions and pixel format.
VolumeInput load_volume(const std::vector<std::string>& files);

struct VolumeResult {
  int w = 0, h = 0, d = 0;
  int sweeps = 0;
  std::vector<uint8_t> band, region, dilated;  // 0/1 per voxel (when requested)
  double kernels_s = 0;
};

struct VolumeExportStats {
  double export_s = 0;         // wall time of render + encode (GPU) incl. D2H of the JPEG bytes
  int64_t jpeg_fallbacks = 0;  // images re-encoded on the host (GPU capacity overflow)
};

struct VolumeParams {
  PipelineParams pipe;        // median/sharpen/band per slice, then 3D SRG
  int connectivity = 6;       // 6 | 26
  int dilation_size = 7;      // cube edge (7×7×7 in config 5)
  bool preprocess = true;     // median + sharpen per slice before the band test
  std::vector<Seed> seeds;    // empty → reference seed pattern on the middle slice
};

// Runs the 3D pipeline on `device`; copies masks back when `want_masks`. A VolumeRunner keeps
// its device buffers, stream and events between runs (rebuilt when the volume shape changes);
// run_volume() is the one-shot form.
class VolumeRunner {
 public:
  explicit VolumeRunner(int device);
  ~VolumeRunner();
  VolumeRunner(const VolumeRunner&) = delete;
  VolumeRunner& operator=(const VolumeRunner&) = delete;
  VolumeResult run(const VolumeInput& v, const VolumeParams& p, bool want_masks);
  // After run() on the same volume: the 2·d exported JPEG files of the 3D cohort mode, in plane
  // order (original, processed), rendered and encoded on the GPU (K3/K4) from the volume still on
  // the device — byte-identical to the golden host renderer + encoder.
  std::vector<std::vector<uint8_t>> export_jpegs(const VolumeInput& v, const VolumeParams& p, const RenderParams& rp,
                                                 struct VolumeExportStats* stats = nullptr);
  // One rank's z-slab of a `depth`-deep volume (volume_slabs.h): `slab` holds planes
  // [z0, z0 + slab.d); seeds (p.seeds, or the reference pattern on plane depth / 2) are in volume
  // coordinates. Preprocesses the slab's planes, runs the global region-growing fixpoint and the
  // halo cube dilation with the other ranks of `comm` (collective), leaving the slab on the device:
  // export_jpegs(slab, ...) then exports its planes. Masks (when requested) are the slab's.
  VolumeResult run_slab(Comm& comm, const VolumeInput& slab, int z0, int depth, const VolumeParams& p, bool want_masks,
                        struct SlabStats* stats = nullptr);

 private:
  struct Impl;
  std::unique_ptr<Impl> impl_;
};
VolumeResult run_volume(const VolumeInput& v, const VolumeParams& p, int device, bool want_masks);

namespace app {
int run_volume_cohort(const AppConfig& cfg);
}

}  // namespace nm03
