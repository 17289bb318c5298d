// nm03/engine.h — the per-GPU batch engine (SURVEY §1.2 L3 stream scheduler).
//
// A run is a list of WorkItems (DICOM file → output directory). Items are cut into batches of
// `batch_size` (DEFAULT_BATCH_SIZE = 25 in main_parallel.cpp:33) and pushed through a ring of
// `streams` independent slots, each with its own HIP stream, pinned upload blob, device buffers
// and host-mapped JPEG output. While slot k's kernels run, other slots' loader tasks read/parse
// DICOMs and writer tasks write JPEGs, so disk I/O, PCIe and compute overlap (the reference runs
// load → compute → export strictly in sequence per batch, main_parallel.cpp:330-347).
//
// Per batch on the GPU:  one H2D of the blob → K1a median → K1b sharpen/band → K2 SRG+morph →
// K3 render → K4 JPEG (entropy-coded bytes land directly in host memory).
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "nm03/golden.h"
#include "nm03/params.h"

namespace nm03 {

struct WorkItem {
  std::string path;     // DICOM file
  std::string out_dir;  // directory receiving <stem>_original.jpg / <stem>_processed.jpg
};

enum SliceCode : int32_t {
  kSliceOk = 0,
  kSliceLoadError = 1,   // unreadable / unsupported DICOM
  kSliceTooSmall = 2,    // width<100 || height<100 (main_sequential.cpp:189-192)
  kSliceDeviceError = 3, // HIP failure in the slice's batch
  kSliceExportError = 4, // JPEG write failed
  kSliceNotRun = 5,
};

struct SliceStatus {
  int32_t code = kSliceNotRun;
  std::string message;
};

struct StageTimes {
  double load_s = 0;       // wall time summed over loader tasks
  double h2d_s = 0;        // device time of uploads
  double kernels_s = 0;    // device time K1..K4
  double write_s = 0;      // wall time summed over writer tasks
  double load_cpu_s = 0;   // thread CPU time of the loader tasks
  double write_cpu_s = 0;  // thread CPU time of the writer tasks
  double slot_cpu_s = 0;   // thread CPU time of the slot threads (descriptors, launches, waits)
  double wall_s = 0;     // run() wall time
  int64_t batches = 0, slices_ok = 0, slices_failed = 0;
  int64_t bytes_in = 0, bytes_out = 0;
  int64_t jpeg_fallbacks = 0;  // images re-encoded on the CPU after a GPU capacity overflow
};

struct EngineConfig {
  int device = 0;
  int batch_size = 25;  // main_parallel.cpp:33
  int streams = 3;      // batches in flight
  int threads = 16;     // host pool (omp_set_num_threads(16), main_parallel.cpp:401)
  // CPUs the pool, slot threads and pinned allocations are bound to (a rank's partition of its
  // GPU's NUMA node, numa::rank_partition). Empty: the whole node of the GPU (multi-node hosts).
  std::vector<int> cpus;
  int max_dim = 512;    // buffers sized for slices up to max_dim × max_dim
  PipelineParams pipe;
  RenderParams render;
  bool export_jpeg = true;
  bool resume = false;  // skip items whose two JPEGs already exist (SURVEY §5.4 --resume)
  // Host path only: no HIP call at all. Every load, parse,
  // 12-bit pack into the (pageable) upload blob and every JPEG file write runs exactly as in a
  // GPU run; the GPU stages are replaced by streaming a fixed pair of pre-encoded JPEG segments
  // into the output buffer (what the encoder's PCIe stores would leave in memory). Measures the
  // host side's CPU per slice on its own, on any machine (bench.py --host-only).
  bool host_only = false;
  // Host-mapped bytes per image for the GPU encoder's stuffed output (0 = 3/8 of the canvas: 96 KiB
  // for 512² — full-contrast noise renders to 86.6 KB, a phantom slice to 14 KB; round 5 used half
  // the canvas, whose pinning was a third of a cold CLI's engine constructor). Larger images are CPU
  // re-encoded (StageTimes counts them); tests force that path with a tiny capacity.
  uint32_t jpeg_out_cap = 0;
  // Every slot and the uploads on ONE HIP stream (false: a stream per slot plus a shared upload
  // stream). For processes limited to one HW queue (GPU_MAX_HW_QUEUES=1, the CLIs' short jobs), where
  // separate streams add no device concurrency — they all feed the same queue in submission order —
  // but each costs ≈ 3.8 ms to create on a cold process. The slots' host work (loads, writes) still
  // overlaps: each slot waits on its own batch's event.
  bool shared_stream = false;
  // Slack in each slot's raw region for single-pass packing of slices wider than 12 bits (u16 elements
  // per pool thread; -1 = one 3/4-size slice per thread, 0 = none: such slices are range-checked
  // first and packed in a second pass). The CLIs pass 0 when rank 0's header scan saw no slice with
  // more than 12 stored bits: 1.5 MB less pinned memory per slot.
  int pack_slack = -1;
  // Progressive upload: a batch's finished prefix of raw pixels is queued for H2D once it has grown
  // by this many KiB while its loads still run (-1 = 2048; 0 = one upload per batch after all loads).
  int upload_chunk_kb = -1;
  // At most this many pool workers write a batch's JPEGs at once when its output directories are
  // being filled (files created, not rewritten; 0 = no limit). tmpfs inode allocation serialises on
  // per-filesystem locks: a JPEG pair costs ≈10 µs of CPU to create on one thread, ≈13–15 µs with
  // 4 creating at once and 35–44 µs with 16 (tools/create_probe.cpp, profiles/r4/create_probe/);
  // the other workers take the next batches' loads meanwhile.
  int create_writers = 4;
  // Slots 1..streams-1 built by their own worker threads while slot 0 already runs (true), or all
  // in the constructor (false, default). Measured in round 5 (profiles/r5/cold/): a slot's HW-queue
  // creation (hipStreamCreate, 10–50 ms on a cold process) and its pinned/device allocations hold
  // HIP runtime locks, so lazily built slots stalled the first batch's copies and launches for
  // 20–40 ms; built up front, a cold 465-slice pass takes ≈ 4 ms after the constructor.
  bool lazy_slots = false;
};

// Everything test_pipeline exports / tests inspect for one slice (host copies).
struct SingleResult {
  int w = 0, h = 0;
  std::vector<uint16_t> median_keys;
  std::vector<float> sharpened;
  std::vector<uint8_t> band, region, eroded, dilated;               // 0/1 per pixel
  std::vector<uint8_t> border_region, border_eroded, border_dilated;
  int srg_iterations = 0;
  // canvases and JPEG files: original, preprocessed, segmentation, erosion, dilation
  std::vector<std::vector<uint8_t>> canvases, jpegs;
};

struct RunHandle;  // a submitted run (Engine::submit)
using RunTicket = std::shared_ptr<RunHandle>;

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  // Process all items (blocking). on_start(i) is called when item i starts loading (used by the
  // sequential CLI to print "Processing: ..." at the right moment).
  // `batch_cap` > 0: batches of at most that many slices for this run (≤ batch_size). A short list
  // (a rank's shard under strong scaling) cut into ⌈n / streams⌉-slice batches spreads over every
  // slot, so its loads, uploads, kernels and writes overlap instead of running as one batch.
  std::vector<SliceStatus> run(const std::vector<WorkItem>& items, StageTimes* times = nullptr,
                               const std::function<void(size_t)>& on_start = {}, int batch_cap = 0);

  // Asynchronous form: queue a run and return at once. Runs are processed in submission order,
  // and the slots move on to a queued run's batches while the previous run drains, so a caller
  // that keeps the next run submitted (double buffering) never pays the slot ring's fill/drain
  // between runs. `items` stays shared with the engine until the run finished. Two runs in flight
  // must not write the same output files.
  RunTicket submit(std::shared_ptr<const std::vector<WorkItem>> items, std::function<void(size_t)> on_start = {},
                   int batch_cap = 0);
  // Blocks until the run finished; rethrows an engine error of that run.
  std::vector<SliceStatus> wait(const RunTicket& ticket, StageTimes* times = nullptr);

  // One slice through every stage with all intermediate outputs copied back (test_pipeline).
  // Waits for queued runs; not to be called concurrently with submit().
  SingleResult run_single(const golden::SliceInput& s);

  const EngineConfig& config() const;

  // Returns once no engine thread can be inside the HIP runtime between runs: the slots built
  // lazily by their own threads are built (or given up). For a process that exits without
  // destroying the engine (the CLIs' fast exit): exit handlers registered after the engine's
  // libraries — the HIP runtime's own among them — must not run while a slot thread is still
  // allocating (a hipHostMalloc faulted inside the HSA runtime that way, gpurun_out/r4j).
  void quiesce();

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

// Device count without initialising anything else (hipGetDeviceCount).
int device_count();

// Creates `n` non-blocking HIP streams on `device` now and parks them for the next engines built on
// that device (one per slot plus the shared upload stream: streams + 1). A stream costs 3–4 ms to
// create and the first ones a HW queue each, 20 ms then ≈ 9 ms (tools/queue_probe.cpp,
// profiles/r5/queues/): a cold CLI reserves them on its start-up thread right after hipInit, while
// rank 0 still plans, so the engine constructor only allocates buffers. Returns the seconds spent.
double reserve_streams(int device, int n);

}  // namespace nm03
