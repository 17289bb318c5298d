// Cohort processors behind the three CLIs. Message texts are the reference's;
// file:line citations point at the reference statement each message reproduces.
#include <dirent.h>
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <mutex>
#include <sstream>
#include <thread>

#include "nm03/app.h"
#include "nm03/cohort.h"
#include "nm03/comm.h"
#include "nm03/dicom.h"
#include "nm03/golden.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg.h"
#include "nm03/kernels.h"
#include "nm03/log.h"
#include "nm03/metaimage.h"
#include "nm03/numa.h"
#include "nm03/volume.h"

namespace nm03::app {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void usage(const std::string& which) {
  std::cout << "usage: " << which << " [options]\n"
            << "  --data-root DIR        dataset root (default $NM03_DATA_ROOT or ../data/)\n"
            << "  --out DIR              output root (default ../out-" << (which == "test_pipeline" ? "test" : which == "img_processing_sequential" ? "sequential" : "parallel") << ")\n"
            << "  --gpus N|all|auto      data-parallel ranks, one process per MI355X (parallel CLI; default auto:\n"
            << "                         one rank per 4096 slices of the cohort, at most every visible GPU)\n"
            << "  --device N             GPU for a single-rank run\n"
            << "  --batch-size N         slices per GPU batch (default 25)\n"
            << "  --streams N            batches in flight per GPU (default 3)\n"
            << "  --threads N            host I/O threads per rank (parallel default: the rank's CPU share, ≤ 16)\n"
            << "  --median-window K      3|5|7|9 (default 7)\n"
            << "  --srg-connectivity C   4|8 (2D) / 6|26 (3D)\n"
            << "  --dilation-size S      (default 3; 7 in --mode 3d)    --erosion-size S (default 3)\n"
            << "  --se-shape square|disc structuring element of dilation/erosion (3D: cube|ball; default square)\n"
            << "  --render-filter bilinear|nearest  interpolation of the gray renders (default bilinear)\n"
            << "  --quality Q            JPEG quality (default 75)\n"
            << "  --jpeg-sampling 420|444|gray  JPEG component layout: YCbCr 4:2:0 (default), 4:4:4, one gray component\n"
            << "  --mode 2d|3d           3d: whole series as a volume (SRG 6-conn + cube dilation)\n"
            << "  --split-volume         3d: each volume split into z-slabs over all ranks (halo exchange)\n"
            << "  --input FILE           test_pipeline: slice to process\n"
            << "  --cpu                  test_pipeline / --mode 3d: golden CPU model instead of the GPU\n"
            << "  --no-montage           test_pipeline: skip the 5-view montage JPEG\n"
            << "  --html                 test_pipeline: also write multi_view.html, the five views in a 2300x450 window\n"
            << "  --dump-mhd DIR         test_pipeline: write stage arrays as MetaImage (.mhd/.raw)\n"
            << "  --repeat N             process the cohort N times (benchmarking)\n"
            << "  --json FILE            write run metrics as JSON\n"
            << "  --resume               keep existing outputs; skip slices whose two JPEGs exist\n"
            << "  --frame K              import frame K of multi-frame DICOM files (default: reject them)\n"
            << "  --hw-queues N|auto     HIP hardware queues of this process (GPU_MAX_HW_QUEUES, 1..32; auto: 1 for short\n"
            << "                         2D jobs on shader copies unless the environment chose a value, else unchanged;\n"
            << "                         0 = environment)\n"
            << "  --copy-engine auto|sdma|blit  host<->GPU copies: DMA engines or shader copies (auto: blit for\n"
            << "                         2D jobs of <= 4096 slices per rank, whose cold start the DMA queue's set-up dominates)\n"
            << "  --quiet                suppress per-slice progress lines\n"
            << "env: NM03_DATA_ROOT, NM03_LOG=info|warn|error|none, NM03_ROCTX=1,\n"
            << "     NM03_FAULT=corrupt_dicom:<i>,fail_batch:<k>,fail_write:<j>,rank_exit:<r>\n"
            << "     NM03_COMM=auto|rccl|host, NM03_DEVICE_OVERRIDE=<device>, NM03_COMM_TIMEOUT_S=<s>\n";
}

void write_json(const std::string& path, const std::string& body) {
  if (path.empty()) return;
  std::ofstream f(path, std::ios::trunc);
  f << body << "\n";
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char ch : s) {
    if (ch == '"' || ch == '\\') o += '\\';
    if ((unsigned char)ch < 0x20) ch = ' ';
    o += ch;
  }
  return o;
}

std::string fmt(double v, int p = 6) {
  std::ostringstream o;
  o << std::setprecision(p) << v;
  return o.str();
}

}  // namespace

int visible_gpu_count() {
  int n = 0;
  DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
  if (d) {
    while (dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      std::ifstream f(std::string("/sys/class/kfd/kfd/topology/nodes/") + e->d_name + "/properties");
      std::string k;
      long v = 0;
      while (f >> k >> v)
        if (k == "simd_count" && v > 0) {
          ++n;
          break;
        }
    }
    closedir(d);
  }
  for (const char* var : {"HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"}) {
    const char* s = std::getenv(var);
    if (s && *s) {
      int c = 1;
      for (const char* p = s; *p; ++p) c += *p == ',';
      n = std::min(n > 0 ? n : c, c);
    }
  }
  return n;
}

AppConfig parse_args(int argc, char** argv, const std::string& which) {
  const double main_unix = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
  arm_fast_exit();
  install_crash_handler();
  AppConfig c;
  c.main_unix_s = main_unix;
  c.data_root = cohort::default_data_root();
  c.out_dir = which == "test_pipeline" ? "../out-test" : which == "img_processing_sequential" ? "../out-sequential" : "../out-parallel";
  if (which == "img_processing_sequential") {
    c.engine.batch_size = 1;
    c.engine.streams = 1;
    c.engine.threads = 2;
  }
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::cerr << "missing value for " << a << std::endl;
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "--help" || a == "-h") {
      usage(which);
      std::exit(0);
    } else if (a == "--data-root") c.data_root = cohort::with_slash(val());
    else if (a == "--out") c.out_dir = val();
    else if (a == "--gpus") {
      std::string v = val();
      c.gpus = v == "all" ? kGpusAll : v == "auto" ? kGpusAuto : std::max(1, std::atoi(v.c_str()));
    } else if (a == "--device") c.engine.device = std::atoi(val().c_str());
    else if (a == "--batch-size") c.engine.batch_size = std::atoi(val().c_str());
    else if (a == "--streams") {
      c.engine.streams = std::atoi(val().c_str());
      c.streams_set = true;
    }
    else if (a == "--threads") {
      c.engine.threads = std::atoi(val().c_str());
      c.threads_set = true;
    }
    else if (a == "--median-window") c.engine.pipe.median_window = std::atoi(val().c_str());
    else if (a == "--srg-connectivity") c.engine.pipe.srg_connectivity = std::atoi(val().c_str());
    else if (a == "--dilation-size") {
      c.engine.pipe.dilation_size = std::atoi(val().c_str());
      c.dilation_set = true;
    }
    else if (a == "--erosion-size") c.engine.pipe.erosion_size = std::atoi(val().c_str());
    else if (a == "--quality") c.engine.render.jpeg_quality = std::atoi(val().c_str());
    else if (a == "--mode") c.mode = val();
    else if (a == "--input") c.input = val();
    else if (a == "--cpu") c.cpu = true;
    else if (a == "--no-montage") c.montage = false;
    else if (a == "--html") c.html = true;
    else if (a == "--dump-mhd") c.dump_mhd = val();
    else if (a == "--repeat") c.repeat = std::max(1, std::atoi(val().c_str()));
    else if (a == "--json") c.json = val();
    else if (a == "--quiet") c.quiet = true;
    else if (a == "--max-dim") {
      c.engine.max_dim = std::atoi(val().c_str());
      c.max_dim_set = true;
    }
    else if (a == "--resume") c.engine.resume = true;
    else if (a == "--frame") c.engine.pipe.frame = std::atoi(val().c_str());
    else if (a == "--hw-queues") {
      const std::string v = val();
      char* end = nullptr;
      const long q = v == "auto" ? -1 : std::strtol(v.c_str(), &end, 10);
      if (v != "auto" && (end == v.c_str() || *end || q < 0 || q > 32)) {  // the runtime refuses more than 32
        std::cerr << "--hw-queues must be auto or 0..32 (0 = leave GPU_MAX_HW_QUEUES as the environment sets it)"
                  << std::endl;
        std::exit(2);
      }
      c.hw_queues = (int)q;
    }
    else if (a == "--copy-engine") {
      const std::string v = val();
      if (v != "auto" && v != "sdma" && v != "blit") {
        std::cerr << "--copy-engine must be auto, sdma or blit" << std::endl;
        std::exit(2);
      }
      c.copy_engine = v == "sdma" ? kCopySdma : v == "blit" ? kCopyBlit : kCopyAuto;
    }
    else if (a == "--jpeg-sampling") {
      const std::string v = val();
      if (v != "420" && v != "444" && v != "gray") {
        std::cerr << "--jpeg-sampling must be 420, 444 or gray" << std::endl;
        std::exit(2);
      }
      c.engine.render.jpeg_sampling = v == "gray" ? jpeg::kSamplingGray : v == "444" ? jpeg::kSampling444 : jpeg::kSampling420;
    }
    else if (a == "--render-filter") {
      const std::string v = val();
      if (v != "bilinear" && v != "nearest") {
        std::cerr << "--render-filter must be bilinear or nearest" << std::endl;
        std::exit(2);
      }
      c.engine.render.filter = v == "nearest" ? kFilterNearest : kFilterBilinear;
    }
    else if (a == "--se-shape") {
      const std::string v = val();
      if (v != "square" && v != "disc") {
        std::cerr << "--se-shape must be square or disc" << std::endl;
        std::exit(2);
      }
      c.engine.pipe.se_shape = v == "disc" ? kSeDisc : kSeSquare;
    }
    else if (a == "--split-volume") c.split_volume = true;
    else {
      std::cerr << "unknown option " << a << " (see --help)" << std::endl;
      std::exit(2);
    }
  }
  // HW queues of the process, set before anything initialises HIP (rank processes inherit it).
  // Every stream past the first costs a new HW queue (≈ 9 ms cold) until GPU_MAX_HW_QUEUES is
  // reached, then ≈ 3–4 ms on a shared one: 2 queues cut the start-up thread's stream reservation from
  // 56 to 45 ms (interleaved cold runs, profiles/r5/cold/cli_wall.jsonl) with the same warm throughput
  // (--repeat 30: 121k vs 117k slices/s, profiles/r5/queues/). auto (-1) is resolved with the copy path
  // (apply_copy_engine).
  if (c.hw_queues > 0) setenv("GPU_MAX_HW_QUEUES", std::to_string(c.hw_queues).c_str(), 1);
  return c;
}

// =============================================================================================
// img_processing_sequential
// =============================================================================================
int run_sequential(const AppConfig& cfg) {
  try {
    const int64_t cohort_slices = cfg.copy_engine == kCopyAuto ? count_cohort_slices(cfg) : -1;
    apply_copy_engine(cfg, cohort_slices < 0 ? -1 : cohort_slices * std::max(1, cfg.repeat));
    // HIP start-up and the engine's construction on the start-up thread while the output root is set up.
    EngineConfig ec = cfg.engine;
    ec.shared_stream = one_hw_queue();  // as in parallel_rank
    EngineStartup su(ec.device, ec.shared_stream ? 1 : std::max(1, ec.streams) + 1);
    // SequentialImageProcessor ctor: base output dir (main_sequential.cpp:81-91).
    cohort::make_dirs(cfg.out_dir);
    const std::string base = cohort::cohort_dir(cfg.data_root);
    std::string setup_error;
    auto engine_p = su.build(ec, &setup_error);
    if (!engine_p) throw std::runtime_error(setup_error);
    Engine& engine = *engine_p;
    // The process ends in cli_exit: the engine's buffers are left to the kernel, not unpinned.
    struct Leak {
      std::unique_ptr<Engine>& e;
      ~Leak() {
        if (fast_exit_enabled() && e) {
          e->quiesce();
          (void)e.release();
        }
      }
    } leak{engine_p};
    // Patient directories are wiped by renaming them aside; the deletions run on background threads
    // while the engine works (cohort.h OutputReaper) and are waited for before the run ends.
    cohort::OutputReaper reaper(4);
    const double t0 = now_s();
    StageTimes total;
    int64_t slices = 0, slices_ok = 0;
    for (int rep = 0; rep < cfg.repeat; ++rep) {
      std::cout << "\n=== Starting Sequential Processing for All Patients ===\n" << std::endl;  // :317
      std::vector<std::string> patients;
      try {
        patients = cohort::find_patient_dirs(base);
        std::cout << "Found " << patients.size() << " patient directories." << std::endl;  // :110
      } catch (const std::exception& e) {
        std::cerr << "Error finding patient directories: " << e.what() << std::endl;  // :113
        throw;
      }
      if (patients.empty()) {
        std::cout << "No patient directories found. Exiting." << std::endl;  // :324
        return 0;
      }
      int successful = 0;
      for (const auto& pid : patients) {
        try {
          try {
            std::cout << "\n=== Processing Patient: " << pid << " ===\n" << std::endl;  // :276
            const std::string out = cfg.out_dir + "/" + pid;
            try {
              if (cfg.engine.resume)
                cohort::make_dirs(out);
              else
                reaper.wipe(out);
            } catch (const std::exception& e) {
              throw std::runtime_error(std::string("Error setting up output directory: ") + e.what());
            }
            std::cout << "Created clean output directory: " + out << std::endl;  // :41
            cohort::Series series;
            try {
              series = cohort::list_patient_series(base, pid);
              std::cout << "Using series directory: " << series.series_dir << std::endl;  // :140
              std::cout << "Found " << series.files.size() << " DICOM files for patient " << pid << std::endl;
            } catch (const std::exception& e) {
              std::cerr << "Error loading DICOM files for patient " << pid << ": " << e.what() << std::endl;  // :164
              throw;
            }
            std::vector<WorkItem> items;
            for (const auto& f : series.files) items.push_back({f, out});
            StageTimes t;
            // Batch 1, one stream: strictly one slice at a time, like the reference loop (:287).
            auto st = engine.run(
                items, &t, [&](size_t i) {
                  if (!cfg.quiet) std::cout << "Processing: \"" << cohort::filename(items[i].path) << "\"" << std::endl;  // :172
                });
            int ok = 0;
            for (size_t i = 0; i < st.size(); ++i) {
              if (st[i].code == kSliceOk) {
                ++ok;
              } else if (st[i].code == kSliceDeviceError) {
                // Not a pipeline (fast::Exception-class) error: the reference's outer per-image
                // catch reports these (main_sequential.cpp:291-293).
                std::cerr << "Failed to process image " << (i + 1) << " for patient " << pid
                          << ". Moving to next image." << std::endl;
              } else {
                std::string e = st[i].message;
                if (st[i].code == kSliceExportError) {
                  // exportProcessedImage logs and rethrows (main_sequential.cpp:74-76), then
                  // processSingleImage logs the same error again (:267-269).
                  static const std::string kPrefix = "Error in export stage: ";
                  if (e.compare(0, kPrefix.size(), kPrefix) == 0) e = e.substr(kPrefix.size());
                  std::cerr << kPrefix << e << std::endl;
                }
                std::cerr << "Error processing file " << items[i].path << ":\n"
                          << "Detailed error: " << e << std::endl;  // :268-269
              }
            }
            total.load_s += t.load_s;
            total.h2d_s += t.h2d_s;
            total.kernels_s += t.kernels_s;
            total.write_s += t.write_s;
            slices += (int64_t)st.size();
            slices_ok += ok;
            // Successes are counted correctly (the reference also counts swallowed failures,
            // SURVEY §2.8 quirk 1).
            std::cout << "\nPatient " << pid << " completed. Successfully processed " << ok << "/" << items.size()
                      << " images." << std::endl;  // :297-299
          } catch (const std::exception& e) {
            std::cerr << "Error processing patient " << pid << ": " << e.what() << std::endl;  // :302
          }
          ++successful;
        } catch (const std::exception& e) {
          std::cerr << "Failed to process patient " << pid << ". Moving to next patient." << std::endl;  // :335
        }
      }
      std::cout << "\n=== All Processing Completed ===\n" << std::endl;                              // :340
      std::cout << "Successfully processed " << successful << "/" << patients.size() << " patients." << std::endl;  // :341
    }
    reaper.drain();
    const double wall = now_s() - t0;
    write_json(cfg.json, std::string("{\"mode\": \"sequential\", \"gpus\": 1, \"wall_s\": ") + fmt(wall) +
                             ", \"slices\": " + std::to_string(slices) + ", \"slices_ok\": " + std::to_string(slices_ok) +
                             ", \"slices_per_s\": " + fmt(slices_ok / std::max(wall, 1e-9)) +
                             ", \"load_s\": " + fmt(total.load_s) + ", \"h2d_s\": " + fmt(total.h2d_s) +
                             ", \"kernels_s\": " + fmt(total.kernels_s) + ", \"write_s\": " + fmt(total.write_s) + "}");
  } catch (const std::exception& e) {
    std::cerr << "Fatal error: " << e.what() << std::endl;  // :359-360
    return 1;
  }
  return 0;
}

// =============================================================================================
// img_processing_parallel — N ranks, one MI355X each, global work list sharded in contiguous
// blocks; rank 0 plans (directories, ordering) and prints; the shared-memory control plane (or RCCL,
// NM03_COMM=rccl) carries plan and results.
// =============================================================================================
namespace {

struct PatientPlan {
  std::string id, out_dir, series_dir, error;
  bool setup_ok = false, listed = false;
  std::vector<std::string> files;
};

std::vector<uint8_t> encode_plan(const std::vector<PatientPlan>& pl) {
  ByteWriter w;
  w.u32((uint32_t)pl.size());
  for (const auto& p : pl) {
    w.str(p.id);
    w.str(p.out_dir);
    w.str(p.series_dir);
    w.str(p.error);
    w.u32(p.setup_ok);
    w.u32(p.listed);
    w.u32((uint32_t)p.files.size());
    for (const auto& f : p.files) w.str(f);
  }
  return w.b;
}

std::vector<PatientPlan> decode_plan(const std::vector<uint8_t>& b) {
  ByteReader r(b.data(), b.size());
  std::vector<PatientPlan> pl(r.u32());
  for (auto& p : pl) {
    p.id = r.str();
    p.out_dir = r.str();
    p.series_dir = r.str();
    p.error = r.str();
    p.setup_ok = r.u32();
    p.listed = r.u32();
    p.files.resize(r.u32());
    for (auto& f : p.files) f = r.str();
  }
  return pl;
}

// Per-rank figures all-gathered to rank 0 for the --json report.
constexpr const char* kRankFields[] = {"slices",      "slices_ok", "wall_s",  "engine_setup_s", "load_s",
                                       "load_cpu_s",  "h2d_s",     "kernels_s", "write_s",      "write_cpu_s",
                                       "slot_cpu_s",  "jpeg_fallbacks"};
constexpr size_t kNumRankFields = sizeof(kRankFields) / sizeof(kRankFields[0]);

std::string per_rank_json(const std::vector<std::vector<double>>& rows) {
  std::ostringstream o;
  o << "{";
  for (size_t f = 0; f < kNumRankFields; ++f) {
    o << (f ? ", " : "") << "\"" << kRankFields[f] << "\": [";
    for (size_t r = 0; r < rows.size(); ++r) o << (r ? ", " : "") << fmt(rows[r][f], 9);
    o << "]";
  }
  // Imbalance of the processing wall time across ranks (max / min), the first thing to look at
  // when a scaling curve bends.
  double mx = 0, mn = 1e300;
  for (const auto& r : rows) {
    mx = std::max(mx, r[2]);
    mn = std::min(mn, r[2]);
  }
  o << ", \"wall_imbalance\": " << fmt(mn > 0 ? mx / mn : 1.0, 6) << "}";
  return o.str();
}

// Largest slice dimension and largest BitsStored over the plan's files (16 KiB header prefix per
// file, parsed on a small thread pool); unreadable files are skipped (they fail in the engine's loader
// as usual). The engine is sized from them: buffers for the largest slice instead of the 512² maximum,
// and no single-pass packing slack when no slice stores more than 12 bits.
struct HeaderScan {
  int max_dim = 0, max_bits = 0;
};
HeaderScan scan_headers(const std::vector<PatientPlan>& plan, int threads) {
  std::vector<const std::string*> files;
  for (const auto& p : plan)
    for (const auto& f : p.files) files.push_back(&f);
  std::atomic<int> md{0}, mb{0};
  std::atomic<size_t> next{0};
  auto raise = [](std::atomic<int>& a, int v) {
    int cur = a.load();
    while (v > cur && !a.compare_exchange_weak(cur, v)) {
    }
  };
  auto work = [&] {
    std::vector<uint8_t> buf;
    for (size_t i; (i = next.fetch_add(1)) < files.size();) {
      try {
        dicom::SliceFile f(*files[i], dicom::ReadMode::kDirect, 16384);
        const dicom::Header& h = f.header(buf);
        raise(md, std::max(h.rows, h.cols));
        raise(mb, h.bits_stored > 0 ? h.bits_stored : h.bits_allocated);
      } catch (const std::exception&) {
      }
    }
  };
  const int nt = std::max(1, std::min({threads, 16, (int)files.size()}));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return {md.load(), mb.load()};
}

}  // namespace

// Cold start (round 5). ONE start-up thread owns every HIP call until the engine exists: it brings up
// the runtime and the device context, loads every kernel code object, reserves the engine's streams
// (HW queues) and brings up the copy engine, starts and settles RCCL when a comm is given (round 6:
// settled BEFORE the engine is built, so RCCL's own threads never allocate, create streams or load
// code objects while the engine is constructed or launches — the hazard class of round 4's HSA
// fault), and — as soon as the caller hands it the engine configuration (build()) —
// builds the whole engine: every slot's events, pinned and device buffers. Meanwhile the calling
// thread plans (cohort discovery, output wipe, header scan), exchanges the plan over the
// shared-memory control plane and computes the rank's CPU partition. In round 4, slots built on their
// workers held the runtime's locks (HW-queue creation 10–50 ms) while the first batch tried to copy
// and launch, and a cold 465-slice pass took 37–70 ms instead of ≈ 4.5 ms (profiles/r5/cold/).
EngineStartup::EngineStartup(int device, int nstreams, Comm* comm) {
  Hooks h;
  h.prepare = [device, nstreams](Times& t) {
    const double t0 = now_s();
    gpu::check_hip(hipSetDevice(device), "hipSetDevice");
    void* p = nullptr;
    gpu::check_hip(hipMalloc(&p, 4096), "hipMalloc");
    (void)hipFree(p);
    t.hip_init_s = now_s() - t0;
    // The kernels' code objects (HIP would load each translation unit's at its first launch):
    // loaded here, on one thread, before any launch (kernels.h preload_kernels).
    const double t1 = now_s();
    gpu::preload_kernels(/*with_volume=*/false);  // the 2D engine's code objects
    t.kernel_load_s = now_s() - t1;
    // The engine's streams (HW queues) need only the slot count: created before the configuration
    // arrives, while rank 0 may still be planning.
    t.streams_s = reserve_streams(device, nstreams);
  };
  h.build = [](const EngineConfig& ec) { return std::make_unique<Engine>(ec); };
  start(std::move(h), comm);
}

EngineStartup::EngineStartup(Hooks hooks, Comm* comm) { start(std::move(hooks), comm); }

void EngineStartup::start(Hooks hooks, Comm* comm) {
  warm_ = std::thread([this, hooks = std::move(hooks), comm] {
    std::string err;
    Times t;
    try {
      hooks.prepare(t);
    } catch (const std::exception& e) {
      err = e.what();
    }
    if (comm) {
      const double td = now_s();
      if (err.empty()) {
        // RCCL's non-blocking initialisation, settled here: every rank's start-up thread waits for
        // its own communicator (or learns through the segment that some rank's failed) before any
        // engine exists. Errors surface at promote(), where the ranks agree on them.
        comm->start_data_plane();
        comm->settle_data_plane(&cancel_flag_);
      } else {
        comm->fail_data_plane("rank start-up failed: " + err);  // peers stop waiting for this rank
      }
      t.data_plane_s = now_s() - td;
    }
    std::unique_lock<std::mutex> g(m_);
    times_ = t;
    const double tw = now_s();
    cv_.wait(g, [&] { return have_cfg_ || cancel_; });
    times_.config_wait_s = now_s() - tw;
    if (!cancel_ && err.empty()) {
      const EngineConfig ec = ec_;
      g.unlock();
      const double t2 = now_s();
      std::unique_ptr<Engine> e;
      try {
        e = hooks.build(ec);
        if (!e) err = "engine not built";
      } catch (const std::exception& ex) {
        err = ex.what();
      }
      g.lock();
      times_.engine_ctor_s = now_s() - t2;
      engine_ = std::move(e);
    }
    error_ = err;
    done_ = true;
    cv_.notify_all();
  });
}

EngineStartup::~EngineStartup() {
  {
    std::lock_guard<std::mutex> g(m_);
    cancel_ = true;
  }
  cancel_flag_.store(true, std::memory_order_release);
  cv_.notify_all();
  if (warm_.joinable()) warm_.join();
}

std::unique_ptr<Engine> EngineStartup::build(const EngineConfig& ec, std::string* error) {
  std::unique_ptr<Engine> e;
  {
    std::unique_lock<std::mutex> g(m_);
    ec_ = ec;
    have_cfg_ = true;
    cv_.notify_all();
    cv_.wait(g, [&] { return done_; });
    e = std::move(engine_);
    if (error) *error = error_;
  }
  warm_.join();
  if (!e && error && error->empty()) *error = "engine not built";
  return e;
}

namespace {

// `rank_devices`: the HIP device of every rank (one node), for the CPU partition of this rank.
int parallel_rank(const AppConfig& cfg, int rank, int size, Comm& comm, int device, const std::vector<int>& rank_devices,
                  int64_t work_per_rank) {
  const std::string base = cohort::cohort_dir(cfg.data_root);
  EngineConfig ec = cfg.engine;
  ec.device = device;
  const double t_setup = now_s();
  // Cold start (round 5). ONE start-up thread owns every HIP call until the engine exists: it
  // brings up the runtime and the device context, loads the 2D kernels' code objects, starts and
  // settles RCCL (data-plane jobs only, see below), and — as soon as the main thread hands it the
  // engine configuration — builds the whole engine: every slot's streams, events, pinned and device
  // buffers. Meanwhile the main thread plans (rank 0: patient discovery, output wipe, header scan),
  // exchanges the plan over the shared-memory control plane and computes the rank's CPU partition.
  // Nothing else touches HIP before the first batch: in round 4, slots built on their workers held
  // the runtime's locks (HW-queue creation 10–50 ms) while the first batch tried to copy and
  // launch, and a cold 465-slice pass took 37–70 ms instead of ≈ 4 ms (profiles/r5/cold/).
  // A 2D job's collectives are control data (the work list, counts, timing rows: a few KB in all).
  // RCCL is brought up on the start-up thread — started and settled before the engine is built — and
  // carries the collectives after the run (promote()) when the job is long enough to amortise it —
  // more than kBlitMaxSlicesPerRank slices per rank (all --repeat passes), the same bound as the copy
  // path — or when NM03_COMM=rccl asks for it (also at one rank: launch_ranks then gives the rank the
  // deferred communicator); a short job stays on the node's shared-memory control plane and never
  // waits for, or loads, RCCL (NM03_COMM=host: never). Device data exchange (--split-volume) brings
  // RCCL up by itself.
  const char* comm_env = std::getenv("NM03_COMM");
  const std::string comm_mode = comm_env && *comm_env ? comm_env : "auto";
  const bool data_plane =
      comm_mode == "rccl" || (size > 1 && comm_mode == "auto" && work_per_rank > kBlitMaxSlicesPerRank);
  // One HW queue (--hw-queues auto for short jobs on shader copies, or the user's 1): every slot
  // shares one HIP stream — separate streams would feed the same queue anyway — and the start-up
  // thread creates one stream instead of slots + 1 (≈ 3.8 ms each on a cold process).
  ec.shared_stream = one_hw_queue();
  // With one stream the slots only overlap host work; 2 of them pin a third less memory than 3 for
  // the same cold pass (interleaved cold CLIs: constructor 6.6 → 4.4 ms, processing 5.1 → 5.6 ms;
  // one slot: 2.7 ms but 9.2 ms processing, profiles/r6/cold_cli/).
  if (ec.shared_stream && !cfg.streams_set) ec.streams = std::min(ec.streams, 2);
  EngineStartup su(device, ec.shared_stream ? 1 : std::max(1, cfg.engine.streams) + 1, data_plane ? &comm : nullptr);
  double engine_wait_s = 0, plan_s = 0, setup_tail_s = 0;
  std::unique_ptr<Engine> engine_p;
  std::vector<RankDevice> devices;
  double t_start = 0, setup_s = 0;
  double proc_wall = 0, my_wall = 0;
  int64_t total_ok = 0, total_slices = 0, my_slices = 0, my_ok = 0;
  StageTimes agg;
  // Rank 0 wipes the patient directories by renaming them aside; 4 background threads delete the
  // old files while the ranks process (cohort.h OutputReaper), waited for before the run ends.
  std::unique_ptr<cohort::OutputReaper> reaper;
  if (rank == 0 && !cfg.engine.resume) reaper = std::make_unique<cohort::OutputReaper>(4);
  for (int rep = 0; rep < cfg.repeat; ++rep) {
    // ---- plan on rank 0 --------------------------------------------------------------------
    std::vector<uint8_t> plan_bytes;
    int64_t fatal = 0;
    std::string fatal_msg;
    if (rank == 0) {
      std::cout << "\n=== Starting Parallel Processing for All Patients ===\n" << std::endl;  // :360
      std::vector<PatientPlan> plan;
      try {
        std::vector<std::string> pids;
        try {
          pids = cohort::find_patient_dirs(base);
          std::cout << "Found " << pids.size() << " patient directories." << std::endl;  // :250
        } catch (const std::exception& e) {
          std::cerr << "Error finding patient directories: " << e.what() << std::endl;  // :253
          throw;
        }
        for (const auto& pid : pids) {
          PatientPlan p;
          p.id = pid;
          p.out_dir = cfg.out_dir + "/" + pid;
          try {
            if (cfg.engine.resume)
              cohort::make_dirs(p.out_dir);
            else
              reaper->wipe(p.out_dir);
            p.setup_ok = true;
            cohort::Series s = cohort::list_patient_series(base, pid);
            p.series_dir = s.series_dir;
            p.files = std::move(s.files);
            p.listed = true;
          } catch (const std::exception& e) {
            p.error = p.setup_ok ? e.what() : std::string("Error setting up output directory: ") + e.what();
          }
          plan.push_back(std::move(p));
        }
      } catch (const std::exception& e) {
        fatal = 1;
        fatal_msg = e.what();
      }
      plan_bytes = encode_plan(plan);
      ByteWriter dims;
      HeaderScan hs;
      if (!engine_p && !cfg.max_dim_set) hs = scan_headers(plan, cfg.engine.threads);
      dims.u32((uint32_t)hs.max_bits);
      dims.u32((uint32_t)hs.max_dim);
      plan_bytes.insert(plan_bytes.end(), dims.b.begin(), dims.b.end());
    }
    comm.allreduce_sum_i64(&fatal, 1);
    if (fatal) {
      if (rank == 0) std::cerr << "Fatal error: " << fatal_msg << std::endl;
      return 1;
    }
    comm.broadcast_bytes(plan_bytes, 0);  // ncclBroadcast of the serialized work list
    uint32_t seen_dim = 0, seen_bits = 0;
    if (plan_bytes.size() >= 8) {
      ByteReader dr(plan_bytes.data() + plan_bytes.size() - 8, 8);
      seen_bits = dr.u32();
      seen_dim = dr.u32();
      plan_bytes.resize(plan_bytes.size() - 8);
    }
    if (!engine_p) {
      // Buffers sized for the largest slice of the cohort (headers scanned by rank 0) instead of
      // the 512² maximum: less pinned memory to allocate and register at start-up.
      if (seen_dim > 0) ec.max_dim = std::min(gpu::kMaxSliceDim, std::max(64, (int)((seen_dim + 63) / 64 * 64)));
      // No slice stores more than 12 bits: every packable slice packs in one pass without a
      // reservation that might have to be abandoned, so the slots need no slack (a wider slice
      // arriving anyway still loads: range check, then pack).
      if (seen_bits > 0 && seen_bits <= 12) ec.pack_slack = 0;
      // Where this rank runs: its GPU's PCI bus id, and a CPU partition of that GPU's NUMA node
      // disjoint from every other rank's, with a pool sized to it and to the rank's share of the
      // CPU budget (the reference's one machine-wide omp_set_num_threads(16), main_parallel.cpp:401).
      // All-gathered: a record of N distinct devices, or a fatal error when two ranks resolved to
      // the same GPU without NM03_DEVICE_OVERRIDE asking for that.
      {
        RankDevice me;
        me.device = device;
        me.bus_id = numa::device_bus_id(device);
        std::vector<int> rank_nodes;
        for (int d : rank_devices) rank_nodes.push_back(numa::device_node(d));
        const numa::RankCpus part = numa::rank_partition(numa::read_topology(), rank_nodes, rank, numa::cpu_budget());
        if (!cfg.threads_set) ec.threads = part.threads;
        ec.cpus = part.cpus;
        me.node = part.node;
        me.cpus = numa::format_cpulist(part.cpus);
        me.threads = ec.threads;
        // (the transport's own view — ncclCommCount / ncclCommCuDevice — is filled in after
        // promote(), once RCCL is up)
        devices = gather_rank_devices(comm, me);
        const std::string dup = duplicate_device(devices);
        if (!dup.empty() && LaunchOptions::from_env().device_override < 0) {
          if (rank == 0)
            std::cerr << "Fatal error: " << dup << " (set NM03_DEVICE_OVERRIDE=<device> to share one GPU deliberately)"
                      << std::endl;
          return 1;
        }
      }
      // Hand the configuration to the start-up thread and wait for its engine. An engine that
      // fails to come up on one rank must not leave the others blocked in the next collective:
      // agree on it before going on.
      std::string setup_error;
      const double t_wait = now_s();
      plan_s = t_wait - t_setup;
      engine_p = su.build(ec, &setup_error);
      engine_wait_s = now_s() - t_wait;
      if (!engine_p && setup_error.empty()) setup_error = "engine not built";
      int64_t setup_failed = setup_error.empty() ? 0 : 1;
      comm.allreduce_sum_i64(&setup_failed, 1);
      if (setup_failed) {
        if (!setup_error.empty())
          std::cerr << "Fatal error: rank " << rank << " (device " << device << "): " << setup_error << std::endl;
        return 1;
      }
      t_start = now_s();
      setup_s = t_start - t_setup;
      setup_tail_s = t_start - t_wait - engine_wait_s;
    }
    Engine& engine = *engine_p;
    if (fault_plan().rank_exit == rank && size > 1) {  // NM03_FAULT=rank_exit:<r>: a rank dies mid-job
      std::cerr << "injected fault: rank " << rank << " exits" << std::endl;
      _exit(9);
    }
    std::vector<PatientPlan> plan = decode_plan(plan_bytes);
    std::vector<WorkItem> items;
    std::vector<int> owner;
    for (size_t p = 0; p < plan.size(); ++p)
      for (const auto& f : plan[p].files) {
        items.push_back({f, plan[p].out_dir});
        owner.push_back((int)p);
      }
    // Contiguous equal blocks per rank (deterministic, ±1 slice).
    const size_t n = items.size();
    const size_t lo = n * rank / size, hi = n * (rank + 1) / size;
    std::vector<WorkItem> mine(items.begin() + lo, items.begin() + hi);
    comm.barrier();
    const double t0 = now_s();
    StageTimes t;
    std::vector<SliceStatus> st = engine.run(mine, &t);
    my_wall += now_s() - t0;  // this rank's own processing time (before waiting for the others)
    comm.barrier();
    double wall = now_s() - t0;
    // With NM03_COMM=rccl, RCCL (initialising since the start-up thread's hipInit) carries every
    // collective from here on: the processing-time reduction, the status and metric all-gathers.
    if (data_plane) comm.promote();
    comm.allreduce_max_f64(&wall, 1);
    proc_wall += wall;
    agg.load_s += t.load_s;
    agg.load_cpu_s += t.load_cpu_s;
    agg.h2d_s += t.h2d_s;
    agg.kernels_s += t.kernels_s;
    agg.write_s += t.write_s;
    agg.write_cpu_s += t.write_cpu_s;
    agg.slot_cpu_s += t.slot_cpu_s;
    agg.jpeg_fallbacks += t.jpeg_fallbacks;
    my_slices += (int64_t)mine.size();
    for (const auto& s : st) my_ok += s.code == kSliceOk;
    // ---- gather statuses -------------------------------------------------------------------
    ByteWriter w;
    w.u32((uint32_t)st.size());
    for (const auto& s : st) {
      w.i32(s.code);
      w.str(s.message);
    }
    auto all = comm.allgather_bytes(w.b);
    if (rank == 0) {
      std::vector<SliceStatus> gst;
      for (auto& b : all) {
        ByteReader r(b.data(), b.size());
        uint32_t k = r.u32();
        for (uint32_t i = 0; i < k; ++i) {
          SliceStatus s;
          s.code = r.i32();
          s.message = r.str();
          gst.push_back(std::move(s));
        }
      }
      // ---- print the per-patient blocks in patient order ------------------------------------
      size_t cursor = 0;
      int successful = 0;
      for (size_t p = 0; p < plan.size(); ++p) {
        const PatientPlan& pp = plan[p];
        std::cout << "\n=== Processing Patient: " << pp.id << " using Parallel Processing ===\n" << std::endl;  // :313-315
        if (pp.setup_ok) std::cout << "Created output directory: " + pp.out_dir << std::endl;  // :58
        if (!pp.listed) {
          if (pp.setup_ok) std::cerr << "Error loading DICOM files for patient " << pp.id << ": " << pp.error << std::endl;  // :304
          std::cerr << "Error processing patient " << pp.id << ": " << pp.error << std::endl;  // :353
          ++successful;
          continue;
        }
        std::cout << "Using series directory: " << pp.series_dir << std::endl;                                 // :280
        std::cout << "Found " << pp.files.size() << " DICOM files for patient " << pp.id << std::endl;          // :301
        std::cout << "Found " << pp.files.size() << " images to process for patient " << pp.id << std::endl;    // :324
        std::cout << "Using " << engine.config().threads << " threads\n" << std::endl;                         // :326
        int ok = 0;
        for (size_t i = 0; i < pp.files.size(); ++i, ++cursor) {
          if (!cfg.quiet) std::cout << "Processing: \"" << cohort::filename(pp.files[i]) << "\"" << std::endl;  // :72-73
          const SliceStatus& s = gst[cursor];
          if (s.code == kSliceOk) {
            ++ok;
          } else if (s.code == kSliceExportError) {
            std::cerr << s.message << std::endl;  // "Error in export stage: ..." (:214)
          } else {
            std::cerr << "Error processing file " << pp.files[i] << ":\n"
                      << "Detailed error: " << s.message << std::endl;  // :165-166
          }
        }
        total_ok += ok;
        total_slices += (int64_t)pp.files.size();
        std::cout << "\nPatient " << pp.id << " completed. Successfully processed " << ok << "/" << pp.files.size()
                  << " images." << std::endl;  // :349-351
        ++successful;
      }
      if (plan.empty()) std::cout << "No patient directories found. Exiting." << std::endl;  // :367
      else {
        std::cout << "\n=== All Processing Completed ===\n" << std::endl;  // :383
        std::cout << "Successfully processed " << successful << "/" << plan.size() << " patients." << std::endl;
      }
    }
  }
  if (reaper) reaper->drain();
  double tot = now_s() - t_start;
  comm.allreduce_max_f64(&tot, 1);
  // Per-rank stage figures, all-gathered (fields: kRankFields).
  const double mine_row[kNumRankFields] = {(double)my_slices, (double)my_ok,     my_wall,          setup_s,
                                           agg.load_s,        agg.load_cpu_s,    agg.h2d_s,        agg.kernels_s,
                                           agg.write_s,       agg.write_cpu_s,   agg.slot_cpu_s,   (double)agg.jpeg_fallbacks};
  std::vector<double> all_rows(kNumRankFields * (size_t)size);
  comm.allgather(mine_row, sizeof(mine_row), all_rows.data());
  // The transport's own view of every rank, now that it is up (RCCL: ncclCommCount / ncclCommCuDevice).
  {
    const int32_t tv[2] = {comm.transport_size(), comm.transport_device()};
    std::vector<int32_t> all_tv(2 * (size_t)size);
    comm.allgather(tv, sizeof(tv), all_tv.data());
    for (size_t r = 0; r < devices.size() && r < (size_t)size; ++r) {
      devices[r].transport_size = all_tv[2 * r];
      devices[r].transport_device = all_tv[2 * r + 1];
    }
  }
  const Comm::DataPlaneTimes dp = comm.data_plane_times();
  if (rank == 0) {
    std::vector<std::vector<double>> rows((size_t)size);
    for (int r = 0; r < size; ++r)
      rows[r].assign(all_rows.begin() + (size_t)r * kNumRankFields, all_rows.begin() + (size_t)(r + 1) * kNumRankFields);
    const std::string req = cfg.gpus == kGpusAuto ? "\"auto\"" : cfg.gpus == kGpusAll ? "\"all\"" : std::to_string(cfg.gpus);
    write_json(cfg.json, std::string("{\"mode\": \"parallel\", \"gpus\": ") + std::to_string(size) +
                             ", \"gpus_requested\": " + req + ", \"main_unix_s\": " +
                             fmt(cfg.main_unix_s, 17) + ", \"backend\": \"" +
                             std::string(data_plane || size == 1 ? comm.backend() : "host") + "\", \"copy_engine\": \"" +
                             copy_engine_name() + "\", \"shared_stream\": " + (ec.shared_stream ? "true" : "false") +
                             ", \"pack_slack\": " + std::to_string(ec.pack_slack) + ", \"repeat\": " +
                             std::to_string(cfg.repeat) + ", \"engine_setup_s\": " +
                             fmt(setup_s) + ", \"hip_init_s\": " + fmt(su.times().hip_init_s) + ", \"engine_ctor_s\": " +
                             fmt(su.times().engine_ctor_s) + ", \"streams_s\": " + fmt(su.times().streams_s) + ", \"engine_wait_s\": " + fmt(engine_wait_s) + ", \"kernel_load_s\": " +
                             fmt(su.times().kernel_load_s) + ", \"data_plane_s\": " + fmt(su.times().data_plane_s) +
                             ", \"config_wait_s\": " + fmt(su.times().config_wait_s) + ", \"plan_s\": " + fmt(plan_s) +
                             ", \"setup_tail_s\": " + fmt(setup_tail_s) + ", \"data_plane\": " +
                             (data_plane ? "true" : "false") + ", \"comm_settle_s\": " + fmt(dp.settle_s) +
                             ", \"comm_start_s\": " + fmt(dp.start_s) + ", \"comm_wait_s\": " +
                             fmt(dp.wait_s) + ", \"comm_init_s\": " + fmt(dp.init_upper_s) + ", \"wall_s\": " + fmt(tot) +
                             ", \"processing_wall_s\": " + fmt(proc_wall) + ", \"slices\": " + std::to_string(total_slices) +
                             ", \"slices_ok\": " + std::to_string(total_ok) + ", \"slices_per_s\": " +
                             fmt(total_ok / std::max(proc_wall, 1e-9)) + ", \"rank0\": {\"load_s\": " + fmt(agg.load_s) +
                             ", \"h2d_s\": " + fmt(agg.h2d_s) + ", \"kernels_s\": " + fmt(agg.kernels_s) +
                             ", \"write_s\": " + fmt(agg.write_s) + ", \"jpeg_fallbacks\": " +
                             std::to_string(agg.jpeg_fallbacks) + "}, \"per_rank\": " + per_rank_json(rows) +
                             ", \"comm\": {\"backend\": \"" + std::string(data_plane || size == 1 ? comm.backend() : "host") +
                             "\", \"nranks\": " +
                             std::to_string(comm.transport_size()) +
                             (comm.fallback_error().empty() ? std::string() : ", \"rccl_error\": \"" + json_escape(comm.fallback_error()) + "\"") +
                             "}, \"devices\": " + rank_devices_json(devices) + "}");
  }
  if (fast_exit_enabled() && engine_p) {  // the process ends in cli_exit: no teardown
    engine_p->quiesce();
    (void)engine_p.release();
  }
  return 0;
}

}  // namespace

bool fast_exit_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NM03_FAST_EXIT");
    return !(e && std::string(e) == "0");
  }();
  return on;
}

namespace {
std::atomic<bool> g_exit_armed{false};
void fast_exit_handler(int status, void*) {  // on_exit: receives exit()'s status
  std::fflush(nullptr);
  _exit(status);
}
}  // namespace

void arm_fast_exit() {
  // Registered in main before any HIP call (app.h): runs after the handlers registered later and
  // after a profiler's end-of-main finalisation, before the libraries' static destructors.
  if (fast_exit_enabled() && !g_exit_armed.exchange(true)) on_exit(fast_exit_handler, nullptr);
}

int cli_exit(int rc) {
  std::cout.flush();
  std::cerr.flush();
  std::fflush(nullptr);
  return rc;
}

int64_t count_cohort_slices(const AppConfig& cfg) {
  try {
    const std::string base = cohort::cohort_dir(cfg.data_root);
    int64_t n = 0;
    for (const auto& pid : cohort::find_patient_dirs(base)) {
      try {
        n += (int64_t)cohort::list_patient_series(base, pid).files.size();
      } catch (const std::exception&) {
      }
    }
    return n;
  } catch (const std::exception&) {
    return -1;
  }
}

bool one_hw_queue() {
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  return q && std::string(q) == "1";
}

// What the process's HIP runtime uses (read from the environment it starts with).
const char* copy_engine_name() {
  const char* v = std::getenv("HSA_ENABLE_SDMA");
  return v && std::string(v) == "0" ? "blit" : "sdma";
}

bool apply_copy_engine(const AppConfig& cfg, int64_t slices_per_rank) {
  // The first DMA copy of a process sets up the copy engine's queue inside
  // hsa_amd_memory_async_copy_on_engine: 8.7 ms on the cold start's critical path (HIP + HSA API
  // trace, profiles/r5/cold_env/). Shader (blit) copies run on the compute queues that exist anyway:
  // interleaved cold CLIs on the 465-slice cohort, streams + warm-up 42.7 → 33.6 ms, processing
  // 4.2 → 4.5 ms (profiles/r5/cold_env2/). Large jobs keep the DMA engines (PCIe-bound config 4
  // measured 15% slower with shader uploads, ARCHITECTURE.md §6).
  bool blit = cfg.copy_engine == kCopyBlit;
  if (cfg.copy_engine == kCopyAuto)
    blit = cfg.mode != "3d" && slices_per_rank >= 0 && slices_per_rank <= kBlitMaxSlicesPerRank &&
           std::getenv("HSA_ENABLE_SDMA") == nullptr;
  if (blit) setenv("HSA_ENABLE_SDMA", "0", 1);
  // With shader copies the copies need no queue of their own and a short job no concurrency between
  // slots: one HW queue saves the second queue's creation (streams 32–35 → 25–26 ms, processing
  // 4.6–5.0 vs 4.8–4.9 ms, profiles/r5/cold_exitq/; 9 interleaved pairs: engine wait 41.5 vs 45.9 ms,
  // processing 5.1 vs 4.7 ms, profiles/r5/cold_hq/). Only that measured case is overridden: every
  // other job (DMA copies, volumes, long jobs, whose start-up is amortised) keeps the environment's
  // value, and so does a short job whose environment chose a value other than HIP's default of 4
  // (the boxes export the default itself).
  if (cfg.hw_queues < 0 && blit) {
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    if (!q || !*q || std::string(q) == "4") setenv("GPU_MAX_HW_QUEUES", "1", 1);
  }
  return blit;
}

int auto_gpus(int64_t slices, int visible) {
  const int64_t want = (std::max<int64_t>(slices, 0) + kAutoSlicesPerRank - 1) / kAutoSlicesPerRank;
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::max(1, visible), want));
}

int resolve_gpus(const AppConfig& cfg, const LaunchOptions& lo, int64_t slices) {
  const int visible = visible_gpu_count();
  int n = cfg.gpus > 0 ? cfg.gpus : std::max(1, visible);  // --gpus N, or every visible GPU
  if (cfg.gpus == kGpusAuto && slices >= 0) n = auto_gpus(slices, n);
  if (n > 1 && lo.device_override < 0 && visible > 0 && n > visible)
    throw std::runtime_error("--gpus " + std::to_string(n) + " exceeds the " + std::to_string(visible) +
                             " visible GPU(s); set NM03_DEVICE_OVERRIDE=<device> to run several ranks on one GPU");
  return n;
}

int run_parallel(const AppConfig& cfg) {
  try {
    cohort::make_dirs(cfg.out_dir);  // OptimizedParallelProcessor ctor (main_parallel.cpp:219-231)
    if (cfg.mode == "3d") {
      apply_copy_engine(cfg, -1);  // auto keeps the DMA engines for volumes (32 MB per 256³ upload)
      return run_volume_cohort(cfg);
    }
    LaunchOptions lo = LaunchOptions::from_env();
    // auto: size the job to the cohort, counted from its directory listings before any fork
    const int64_t slices = count_cohort_slices(cfg);  // rank count, copy path and comm policy (≈ 1 ms of listings)
    const int n = resolve_gpus(cfg, lo, cfg.gpus == kGpusAuto ? slices : -1);
    apply_copy_engine(cfg, slices < 0 ? -1 : (slices + n - 1) / n * std::max(1, cfg.repeat));  // per rank
    std::vector<int> rank_devices;
    for (int r = 0; r < n; ++r)
      rank_devices.push_back(n > 1 ? lo.device_of(r) : lo.device_override >= 0 ? lo.device_override : cfg.engine.device);
    const int64_t work_per_rank = slices < 0 ? -1 : (slices + n - 1) / n * std::max(1, cfg.repeat);
    return launch_ranks(n, [&](int rank, int size, Comm& comm) {
      return parallel_rank(cfg, rank, size, comm, rank_devices[(size_t)rank], rank_devices, work_per_rank);
    }, lo);
  } catch (const std::exception& e) {
    std::cerr << "Fatal error: " << e.what() << std::endl;  // :407-408
    return 1;
  }
}

// =============================================================================================
// test_pipeline — one slice, all stages, 5 exported stage images (test_pipeline.cpp:164-179),
// headless: the 5-view MultiViewWindow (:148-158) becomes a montage JPEG.
// =============================================================================================
int run_test_pipeline(const AppConfig& cfg) {
  try {
    // GPU path: HIP start-up and the engine's streams on the start-up thread while the slice loads.
    std::unique_ptr<EngineStartup> su;
    if (!cfg.cpu) {
      apply_copy_engine(cfg, 1);  // one slice
      su = std::make_unique<EngineStartup>(cfg.engine.device, 2);
    }
    const std::string path = cfg.input.empty() ? cohort::test_slice_path(cfg.data_root) : cfg.input;
    golden::SliceInput in = golden::load_slice(path, 0, cfg.engine.pipe.frame);  // the test pipeline has no <100 guard
    const PipelineParams& p = cfg.engine.pipe;
    const RenderParams& rp = cfg.engine.render;
    std::vector<std::vector<uint8_t>> canvases, jpegs;
    // Stage arrays for --dump-mhd: sharpened f32 and the four masks (band, SRG, erosion, dilation).
    std::vector<float> d_sharp;
    std::vector<std::vector<uint8_t>> d_masks;
    const double t0 = now_s();
    if (cfg.cpu) {
      golden::SliceResult st;
      golden::StageImages r = golden::test_pipeline_images(in, p, rp, cfg.dump_mhd.empty() ? nullptr : &st);
      canvases = std::move(r.canvases);
      jpegs = std::move(r.jpegs);
      d_sharp = std::move(st.sharpened);
      d_masks = {std::move(st.band), std::move(st.region), std::move(st.eroded), std::move(st.dilated)};
    } else {
      EngineConfig ec = cfg.engine;
      ec.batch_size = 1;
      ec.streams = 1;
      ec.max_dim = std::max({ec.max_dim, in.w, in.h});
      std::string setup_error;
      std::unique_ptr<Engine> engine = su->build(ec, &setup_error);
      if (!engine) throw std::runtime_error(setup_error);
      SingleResult r = engine->run_single(in);
      canvases = std::move(r.canvases);
      jpegs = std::move(r.jpegs);
      d_sharp = std::move(r.sharpened);
      d_masks = {std::move(r.band), std::move(r.region), std::move(r.eroded), std::move(r.dilated)};
    }
    if (!cfg.dump_mhd.empty()) {
      cohort::make_dirs(cfg.dump_mhd);
      const std::string b = cohort::with_slash(cfg.dump_mhd);
      mhd::write(b + "input", in.raw.data(), in.w, in.h, 1, in.type == kI16 ? mhd::MetType::kShort : mhd::MetType::kUShort,
                 in.spacing_x, in.spacing_y);
      mhd::write(b + "sharpened", d_sharp.data(), in.w, in.h, 1, mhd::MetType::kFloat, in.spacing_x, in.spacing_y);
      static const char* mnames[4] = {"band", "segmentation", "erosion", "dilation"};
      for (int k = 0; k < 4; ++k)
        mhd::write(b + mnames[k], d_masks[k].data(), in.w, in.h, 1, mhd::MetType::kUChar, in.spacing_x, in.spacing_y);
    }
    const double t1 = now_s();
    // exportImages: wipe + create the output directory, then the 5 stage images (:7-27).
    cohort::setup_output_dir(cfg.out_dir);
    static const char* names[5] = {"original_image", "preprocessed_image", "segmentation", "erosion_result",
                                   "final_dilated_result"};
    for (int k = 0; k < 5; ++k) {
      std::ofstream f(cfg.out_dir + "/" + names[k] + ".jpg", std::ios::binary | std::ios::trunc);
      f.write((const char*)jpegs[k].data(), (std::streamsize)jpegs[k].size());
    }
    if (cfg.montage) {
      // Headless MultiViewWindow(5, Black, ...): the five views side by side.
      const int cw = rp.out_width, ch = rp.out_height, mw = 5 * cw;
      std::vector<uint8_t> m((size_t)mw * ch, 0);
      for (int k = 0; k < 5; ++k)
        for (int y = 0; y < ch; ++y) std::memcpy(&m[(size_t)y * mw + k * cw], &canvases[k][(size_t)y * cw], cw);
      auto j = jpeg::encode_gray(m.data(), mw, ch, mw, rp.jpeg_quality, (jpeg::Sampling)rp.jpeg_sampling);
      std::ofstream f(cfg.out_dir + "/multi_view.jpg", std::ios::binary | std::ios::trunc);
      f.write((const char*)j.data(), (std::streamsize)j.size());
    }
    if (cfg.html) {
      // The reference's viewer, MultiViewWindow::create(5, Color::Black(), 2300, 450, false)
      // (test_pipeline.cpp:148-158): five views side by side on black in a 2300×450 window. A browser
      // shows the exported stage images the same way, each view scaled to fit its 460×450 cell.
      std::ofstream f(cfg.out_dir + "/multi_view.html", std::ios::trunc);
      f << "<!DOCTYPE html>\n<html><head><meta charset=\"utf-8\"><title>Medical Image Processing Stages</title>\n"
        << "<style>body{margin:0;background:#000}#w{display:flex;width:2300px;height:450px}"
        << "figure{margin:0;flex:1;display:flex;flex-direction:column;align-items:center;justify-content:center}"
        << "img{max-width:460px;max-height:420px}figcaption{color:#ccc;font:13px sans-serif}</style></head>\n"
        << "<body><div id=\"w\">\n";
      for (int k = 0; k < 5; ++k)
        f << "<figure><img src=\"" << names[k] << ".jpg\" alt=\"" << names[k] << "\"><figcaption>" << names[k]
          << "</figcaption></figure>\n";
      f << "</div></body></html>\n";
    }
    if (!cfg.quiet)
      std::cout << "Medical Image Processing Stages: " << (cfg.cpu ? "CPU golden model" : "MI355X") << ", "
                << in.w << "x" << in.h << " slice, pipeline " << fmt((t1 - t0) * 1e3, 4) << " ms, exported 5 images to "
                << cfg.out_dir << "/" << std::endl;
    write_json(cfg.json, std::string("{\"mode\": \"test_pipeline\", \"backend\": \"") + (cfg.cpu ? "cpu" : "gpu") +
                             "\", \"pipeline_ms\": " + fmt((t1 - t0) * 1e3) + "}");
  } catch (const std::exception& e) {
    std::cerr << "Fatal error: " << e.what() << std::endl;
    return 1;
  }
  return 0;
}

}  // namespace nm03::app
