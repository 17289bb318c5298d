// nm03/volume_slabs.h — one 3D volume decomposed into z-slabs over the ranks of a Comm: the
// spatial analogue of context parallelism for this workload. The reference has no 3D
// path (it forces 2D with setLoadSeries(false), test_pipeline.cpp:38-41) and no multi-process code;
// this splits volumes (or volume stacks) that should use several MI355X over RCCL/xGMI.
//
// Rank r owns planes [z0, z1) = slab_bounds(D, r, n) (contiguous, ±1 plane):
//  1. per-plane preprocessing (median → sharpen → band) is in-plane only: no halo;
//  2. seeded region growing is a global fixpoint: every rank grows its slab to a local fixpoint
//     (K5: one cooperative launch, convergence on the device), then neighbours exchange their
//     boundary region planes — bit-packed, Comm::sendrecv (grouped ncclSend/ncclRecv) — and add the
//     in-band voxels of their own boundary planes that touch the neighbour's region (6-connected:
//     the voxel across the boundary; 26: its 3×3 in-plane neighbourhood). An all-reduce of the
//     added-voxel counts decides another round. The union of the slab regions is then exactly the
//     single-volume region: it holds the seeds, is closed under in-band adjacency inside slabs
//     (local fixpoints) and across them (the last round added nothing), and every voxel was reached
//     along an in-band path;
//  3. the cube dilation of size s needs r = s / 2 halo planes from each side: the neighbours' r
//     boundary region planes by sendrecv (all-gather when a slab is thinner than r), then the slab
//     plus halo is dilated and the halo dropped (out-of-volume samples are ignored).
// Traffic per round is two bit planes per rank (8 KiB for 256²), independent of the slab depth.
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

#include "nm03/comm.h"
#include "nm03/common.h"
#include "nm03/params.h"

namespace nm03 {

inline std::pair<int, int> slab_bounds(int depth, int rank, int ranks) {
  return {depth * rank / ranks, depth * (rank + 1) / ranks};
}

// One rank's slab of bit planes [d][h][ceil(w/64)] (d = z1 − z0) on some backend: the GPU
// (VolumeRunner::run_slab) or the golden CPU model (tests, hosts without a GPU).
class SlabGrower {
 public:
  virtual ~SlabGrower() = default;
  // Grow the region to the slab's local fixpoint: from the seeds (first call, region reset) or
  // from the current region (later calls). Returns the sweep count (diagnostics).
  virtual int grow(bool first) = 0;
  virtual std::vector<uint64_t> band_plane(int zl) = 0;
  virtual std::vector<uint64_t> region_plane(int zl) = 0;
  virtual void or_region_plane(int zl, const std::vector<uint64_t>& bits) = 0;
  // Cube dilation of size `size` of the slab's region with `below` / `above` halo planes
  // (nearest plane last / first, possibly fewer than size/2 at the volume's ends).
  virtual void dilate(int size, const std::vector<std::vector<uint64_t>>& below,
                      const std::vector<std::vector<uint64_t>>& above) = 0;
  // Structuring element of dilate(): the digital ball of radius size/2 instead of the cube
  // (PipelineParams::se_shape; the r-plane halo covers both).
  bool ball = false;
};

struct SlabStats {
  int rounds = 0;            // local-grow rounds until no rank added a boundary voxel
  int sweeps = 0;            // K5 sweeps summed over the rounds (this rank)
  int64_t exchanged_bytes = 0;  // boundary + halo bytes this rank sent
};

// Steps 2 and 3 above for this rank's slab [z0, z1) of a D-deep w×h volume. Collective over comm.
SlabStats grow_and_dilate_slabs(Comm& comm, SlabGrower& g, int w, int h, int depth, int z0, int z1,
                                int connectivity, int dilation);

// Golden-model slab backend on unpacked 0/1 voxels (band of the slab, seeds in slab coordinates).
class GoldenSlabGrower final : public SlabGrower {
 public:
  GoldenSlabGrower(std::vector<uint8_t> band, int w, int h, int d, std::vector<Seed> seeds, int connectivity);
  int grow(bool first) override;
  std::vector<uint64_t> band_plane(int zl) override;
  std::vector<uint64_t> region_plane(int zl) override;
  void or_region_plane(int zl, const std::vector<uint64_t>& bits) override;
  void dilate(int size, const std::vector<std::vector<uint64_t>>& below,
              const std::vector<std::vector<uint64_t>>& above) override;
  const std::vector<uint8_t>& region() const { return region_; }
  const std::vector<uint8_t>& dilated() const { return dilated_; }

 private:
  std::vector<uint8_t> band_, region_, dilated_;
  int w_, h_, d_, conn_;
  std::vector<Seed> seeds_;
};

// The seeds of slab [z0, z0 + d) in slab coordinates: `seeds` (volume coordinates) or, when empty,
// the reference pattern (main_sequential.cpp:214-241) on plane depth / 2 — as the single-volume run.
std::vector<Seed> slab_seeds(const std::vector<Seed>& seeds, int w, int h, int depth, int z0, int d);

// Bit-plane helpers (row-major [h][ceil(w/64)] words, bit x%64 of word x/64).
std::vector<uint64_t> pack_plane(const uint8_t* px, int w, int h);
void unpack_plane(const std::vector<uint64_t>& bits, int w, int h, uint8_t* px);
// 3×3 in-plane dilation (out-of-plane samples ignored).
std::vector<uint64_t> dilate_plane3(const std::vector<uint64_t>& bits, int w, int h);

}  // namespace nm03
