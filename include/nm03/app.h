// nm03/app.h — cohort orchestration shared by the three reference CLIs.
//   img_processing_sequential  ≙ SequentialImageProcessor  (main_sequential.cpp:9-363)
//   img_processing_parallel    ≙ OptimizedParallelProcessor (main_parallel.cpp:19-411), now
//                                 data-parallel over N MI355X ranks
//   test_pipeline              ≙ test_pipeline.cpp:29-182 (headless)
// All three keep the reference's stdout/stderr message catalogue, output layout
// out-*/PGBM-XXXX/<stem>_{original,processed}.jpg and no-argument defaults.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nm03/comm.h"
#include "nm03/engine.h"

namespace nm03::app {

// A CLI's cold start: one start-up thread, begun at construction, owns every HIP call until the engine
// exists — hipInit, every kernel code object, `nstreams` reserved streams plus the copy engine's first
// use — then, for RCCL ranks, starts AND settles the data plane (`comm->start_data_plane()`,
// `settle_data_plane()`: RCCL is up before the engine's construction begins, never concurrent with
// it), and then builds the engine from the configuration the caller hands to build() once it is
// known (the caller plans meanwhile). A failed HIP start-up is published to the peers
// (`fail_data_plane`) so that they do not wait for this rank's RCCL. Destruction without build()
// cancels (an unsettled data plane is abandoned) and joins.
class EngineStartup {
 public:
  struct Times {
    double hip_init_s = 0, kernel_load_s = 0, streams_s = 0, data_plane_s = 0, config_wait_s = 0, engine_ctor_s = 0;
  };
  // What the start-up thread does, in order; the CLI's are HIP calls (the device constructor),
  // tests inject fakes (tests/native/unit_tests.cpp, run under TSan by tools/sanitize_check.sh).
  struct Hooks {
    std::function<void(Times&)> prepare;                                  // throws on failure
    std::function<std::unique_ptr<Engine>(const EngineConfig&)> build;    // throws on failure
  };
  EngineStartup(int device, int nstreams, Comm* comm = nullptr);
  EngineStartup(Hooks hooks, Comm* comm);
  ~EngineStartup();
  EngineStartup(const EngineStartup&) = delete;
  EngineStartup& operator=(const EngineStartup&) = delete;
  // Hands over the configuration and waits for the engine; nullptr with *error set on failure.
  std::unique_ptr<Engine> build(const EngineConfig& ec, std::string* error);
  const Times& times() const { return times_; }  // valid after build()

 private:
  void start(Hooks hooks, Comm* comm);
  std::mutex m_;
  std::condition_variable cv_;
  bool have_cfg_ = false, cancel_ = false, done_ = false;
  std::atomic<bool> cancel_flag_{false};  // cancel_, readable by the data plane's settle loop
  EngineConfig ec_;
  std::unique_ptr<Engine> engine_;
  std::string error_;
  Times times_;
  std::thread warm_;
};

struct AppConfig {
  std::string data_root;  // default: cohort::default_data_root()
  std::string out_dir;    // default per CLI: ../out-sequential, ../out-parallel, ../out-test
  EngineConfig engine;
  // Ranks, one process per GPU (--gpus). kGpusAuto (default): as many visible GPUs as the cohort
  // repays (resolve_gpus); kGpusAll (--gpus all): every visible GPU, as the reference's
  // omp_set_num_threads(16) uses the whole laptop (main_parallel.cpp:401); N ≥ 1: exactly N.
  int gpus = -1;
  bool quiet = false;
  bool cpu = false;        // test_pipeline: golden CPU path (BASELINE config 1)
  bool montage = true;     // test_pipeline: 5-view montage JPEG (headless MultiViewWindow)
  bool html = false;       // test_pipeline --html: the five views as a page (MultiViewWindow 2300×450)
  std::string json;        // metrics file
  std::string mode = "2d"; // 2d | 3d
  std::string input;       // test_pipeline: explicit slice path
  std::string dump_mhd;    // test_pipeline: directory for MetaImage stage dumps (empty = off)
  int repeat = 1;
  bool dilation_set = false;  // --dilation-size given (3D mode defaults to 7, BASELINE config 5)
  bool max_dim_set = false;   // --max-dim given (else the parallel CLI sizes buffers from the slice headers)
  // --threads given. Otherwise every rank of the parallel CLI sizes its pool to its CPU partition
  // and its share of the CPU budget (numa::rank_partition), at most the reference's 16.
  bool threads_set = false;
  bool streams_set = false;  // --streams given (else a one-HW-queue job uses 2 slots, see parallel_rank)
  // --mode 3d --split-volume: every patient's volume is decomposed into z-slabs over all ranks
  // (volume_slabs.h) instead of sharding whole patients over the ranks.
  bool split_volume = false;
  // CLOCK_REALTIME when parse_args began (the --json record's "main_unix_s"): with the launcher's
  // own clock it splits a cold run's wall into process start-up (exec → main) and the rest.
  double main_unix_s = 0;
  // GPU_MAX_HW_QUEUES for the process (--hw-queues; 0 = leave the environment's value; -1 = auto:
  // 1 for the short jobs that take shader copies, else 2 — see apply_copy_engine).
  int hw_queues = -1;
  // Host↔device copies (--copy-engine): kCopySdma (the DMA engines), kCopyBlit (shader copies on the
  // compute queues: HSA_ENABLE_SDMA=0) or kCopyAuto (blit for short 2D jobs, see apply_copy_engine).
  int copy_engine = 0;
};

enum CopyEngine : int { kCopyAuto = 0, kCopySdma = 1, kCopyBlit = 2 };
// kCopyAuto picks blit copies up to this many slices per rank (all --repeat passes counted): a
// process's first DMA copy costs
// ≈ 9 ms (the copy engine's queue), shader copies ≈ 0.7 µs more per 256² slice than DMA.
constexpr int kBlitMaxSlicesPerRank = 4096;

// Parse the shared flag set; `which` selects CLI-specific defaults. Exits on --help.
AppConfig parse_args(int argc, char** argv, const std::string& which);

// End of a CLI process without teardown: the engines are drained (every run waited for, no slot
// thread inside HIP: Engine::quiesce) and left to the kernel instead of unpinning host buffers and
// releasing device memory and contexts (≈70–130 ms of a cold CLI run). main registers an exit
// handler before any HIP call (arm_fast_exit; parse_args does) and ends with `return cli_exit(rc)`:
// a profiler that finalises when main returns (rocprofv3 writes its results there; a CLI that called
// exit() from inside main lost them, profiles/r4/exit_order/) and every handler registered after the
// armed one still run, then the armed handler _exits before the shared libraries' static
// destructors (HIP's teardown, which faulted under rocprofv3: profiles/r4/probe/). NM03_FAST_EXIT=0:
// normal exit with full teardown.
void arm_fast_exit();
// Flushes stdout/stderr and returns rc (for `return cli_exit(rc);` in main).
int cli_exit(int rc);
bool fast_exit_enabled();

int run_sequential(const AppConfig& cfg);
int run_parallel(const AppConfig& cfg);
int run_test_pipeline(const AppConfig& cfg);

// Number of GPUs visible to this process, counted WITHOUT initialising HIP (KFD topology +
// HIP/ROCR_VISIBLE_DEVICES), so the launcher can still fork safely afterwards.
int visible_gpu_count();

constexpr int kGpusAuto = -1, kGpusAll = 0;
// A rank is worth its start-up only with this many slices to process: a cold rank costs ≈ 150–300 ms
// of ROCm start-up (hipInit, HW queues) that does not shrink with more ranks (started concurrently,
// 8 processes on one GPU finish within 1.3–3× of one: profiles/r5/startup/), while a cold MI355X
// pass runs ≈ 35–40k slices/s; below ≈ 4k slices per rank the extra ranks only add their start-up
// and RCCL's (profiles/r5/cold/, docs/ROUND5_RESPONSE.md).
constexpr int kAutoSlicesPerRank = 4096;

// Ranks for img_processing_parallel: --gpus N; every visible GPU for --gpus all; for the default
// (auto) ceil(slices / kAutoSlicesPerRank) clamped to [1, visible] when `slices` ≥ 0 is known, else
// every visible GPU. Throws when N exceeds the visible GPUs and no NM03_DEVICE_OVERRIDE shares one
// device between ranks.
int resolve_gpus(const AppConfig& cfg, const LaunchOptions& lo, int64_t slices = -1);
// The auto policy alone: ceil(slices / kAutoSlicesPerRank) clamped to [1, max(1, visible)].
int auto_gpus(int64_t slices, int visible);

// Slices of the cohort under cfg.data_root, counted from the directory listings only (no file is
// opened, no HIP call): what the auto rank count needs before the ranks are forked. -1 on error.
int64_t count_cohort_slices(const AppConfig& cfg);

// Sets the process's copy path before anything initialises HIP (rank processes inherit it):
// HSA_ENABLE_SDMA=0 for kCopyBlit, and for kCopyAuto when 0 ≤ slices_per_rank ≤ kBlitMaxSlicesPerRank
// and the environment does not already set HSA_ENABLE_SDMA; with --hw-queues auto also
// GPU_MAX_HW_QUEUES (1 with shader copies, else 2). Returns whether blit copies were chosen.
bool apply_copy_engine(const AppConfig& cfg, int64_t slices_per_rank);
// "blit" when the process runs with HSA_ENABLE_SDMA=0, else "sdma" (the CLI --json records it).
const char* copy_engine_name();
// The process runs with one HIP hardware queue (GPU_MAX_HW_QUEUES=1): the CLIs then give their
// engine one shared stream (EngineConfig::shared_stream).
bool one_hw_queue();

}  // namespace nm03::app
