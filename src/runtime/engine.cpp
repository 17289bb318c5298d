// Batch engine: host side of the MI355X pipeline (see include/nm03/engine.h).
#include "nm03/engine.h"

#include <hip/hip_runtime_api.h>
#include <fcntl.h>
#include <linux/capability.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <ctime>
#include <atomic>
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <unordered_map>
#include <mutex>
#include <tuple>
#include <thread>

#include "nm03/cohort.h"
#include "nm03/dicom.h"
#include "nm03/golden.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg.h"
#include "nm03/kernels.h"
#include "nm03/log.h"
#include "nm03/numa.h"
#include "nm03/pack12.h"
#include "nm03/synth.h"
#include "nm03/thread_pool.h"

namespace nm03 {

using namespace nm03::gpu;

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
// CPU time of the calling thread (ns): loader/writer tasks report it next to their wall time, so a
// CPU-quota stall or preemption (wall ≫ cpu) can be told apart from work (wall ≈ cpu).
inline int64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

enum Plane { kPBand = 0, kPRegion, kPDilated, kPEroded, kPBorderR, kPBorderE, kPBorderD, kNumPlanes };

struct LoadedSlice {
  bool ok = false;
  int w = 0, h = 0;
  uint8_t type = kU16, stored_bits = 16;
  float slope = 1.f, intercept = 0.f, sx = 1.f, sy = 1.f;
  uint32_t blob_off = 0;  // u16 offset of the uploaded samples in the blob's raw region
  bool packed = false;    // uploaded as 12-bit pairs (nm03/pack12.h)
};

// Per-image JPEG capacities. The entropy-coded segment of a 512² canvas is a few tens of KB;
// anything past these caps falls back to the CPU encoder (counted in StageTimes).

struct Slot {
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
  hipStream_t up = nullptr;  // stream of this slot's H2D copies: its own stream, or the engine's shared one
  bool owns_stream = true;   // false: EngineConfig::shared_stream (the engine destroys it)
  int cap_slices = 0, cap_canvases = 0;
  size_t cap_pixels = 0;  // u16 elements of expanded samples per batch (device raw/median buffers)
  // The blob's raw region also holds `hole_slack` u16 of slack for abandoned 12-bit reservations
  // (a checked single-pass pack that found a wide sample, see load_one); `hole_credit` is what is
  // left of it in the current batch (an atomic: taken and returned without a lock).
  size_t hole_slack = 0;
  std::atomic<size_t> hole_credit{0};
  // blob layout (byte offsets)
  size_t off_stats = 0, off_desc = 0, off_medt = 0, off_shpt = 0, off_seeds = 0, off_render = 0, off_jpeg = 0,
         raw_base = 0, blob_bytes = 0;
  size_t max_medt = 0, max_shpt = 0;
  uint8_t* h_blob = nullptr;
  // Where the loaders write the batch's raw pixels: h_blob + raw_base (pinned host memory, uploaded by
  // SDMA; host-only engines: anonymous memory).
  uint8_t* raw_cpu = nullptr;
  uint8_t* h_single = nullptr;  // run_single's pinned read-back area (allocated on first use)
  size_t single_bytes = 0;
  uint8_t* d_blob = nullptr;
  uint16_t* d_raw_x = nullptr;  // expanded 16-bit samples of the batch (K0 output, every kernel's input)
  uint16_t* d_med = nullptr;
  uint32_t* d_tile_mm = nullptr;  // per median tile (min, max) key
  float* d_f32 = nullptr;
  uint64_t* d_bits = nullptr;
  uint64_t* d_srg_scratch = nullptr;  // K2 bit planes of slices above kSrgMaxDim (global-memory form)
  size_t plane_words = 0;
  uint8_t* d_canvas = nullptr;
  JpegWork jw;
  // The encoder stores each canvas's stuffed bytes straight into host-mapped h_out over PCIe
  // (canvas k at k × out_cap). Measured alternatives, removed in round 4 (docs/ARCHITECTURE.md §6):
  // HBM + gather kernel + one SDMA copy (the D2H copies share the copy engines with the uploads:
  // 138-242k vs 286-340k slices/s) and HBM + a gather kernel storing into host memory (no gain).
  uint8_t* h_out = nullptr;
  uint8_t* d_out = nullptr;
  int32_t* h_sizes = nullptr;
  int32_t* d_sizes = nullptr;
  std::vector<LoadedSlice> loaded;
  // Progressive upload: raw-region allocations in offset order with a done flag each; the slot
  // thread uploads the longest finished prefix while later loads are still running.
  struct Alloc {
    size_t off = 0, len = 0;  // u16 elements; written before `done` is released
    std::atomic<bool> done{false};
  };
  std::unique_ptr<Alloc[]> allocs;
  size_t max_allocs = 0;
  // Allocation word, claimed lock-free by the loaders: the number of allocations (bits 40..63) and
  // the u16 elements of the raw region in use (bits 0..39), so that allocation k always lies at a
  // higher offset than allocation k−1 (one CAS per load; round 5 took alloc_m for it, and the
  // loaders' contention on that and on prog_m was ≈ 8% of the pool's CPU, profiles/r6/cpu_profile/).
  static constexpr int kAllocShift = 40;
  static constexpr uint64_t kUsedMask = (uint64_t(1) << kAllocShift) - 1;
  std::atomic<uint64_t> alloc_word{0};
  size_t raw_used() const { return (size_t)(alloc_word.load(std::memory_order_acquire) & kUsedMask); }
  size_t n_allocs() const { return (size_t)(alloc_word.load(std::memory_order_acquire) >> kAllocShift); }
  std::mutex prog_m;
  std::condition_variable prog_cv;
  std::atomic<size_t> loads_finished{0};
  std::atomic<bool> prog_waiting{false};  // the slot thread sleeps (or is about to) on prog_cv
  // The finished-load count at which the sleeping slot thread wants to be woken: the next upload
  // chunk's worth of slices (one wake-up per chunk, ≈ 4 per 96-slice batch, instead of one per 4 loads).
  std::atomic<size_t> wake_at{0};
  // Set by upload_progress when the whole batch fits in one upload chunk: loaders stop notifying
  // (a wake-up of the slot thread per load, on CPUs the loaders need, for nothing to upload early).
  std::atomic<bool> progress_quiet{false};
  size_t uploaded = 0;        // u16 elements of the raw region already queued for upload
  bool upload_started = false;
  // built per batch
  std::vector<int> live;  // batch-local indices of loaded slices, in order
  int ncanvas = 0;
  bool any_canvas = false;  // some image of the batch needs the generic render → canvas path
  int max_w = 0, max_h = 0;
  double batch_ema_s = 0;  // enqueue → completion time per slice of recent batches (wait_batch)
  // Host-only engine (EngineConfig::host_only): h_blob / h_out are plain mappings, no device side.
  bool host_only = false;
  // h_blob / h_out / h_sizes live in the engine's pinned arenas (freed with the engine, not here).
  bool arena = false;
  size_t out_bytes = 0;
};

// Private fd tables for the host pool's workers. Every open and
// close takes the process's fd-table lock; with 16 loader/writer threads doing three opens and
// three closes per slice that lock (and its cache line crossing CCDs) doubled the per-file cost:
// 23–24 µs per load and 31.7 µs per JPEG pair in 16 threads of one process vs 14.7–16.5 and
// 10.0–10.6 µs in 16 processes (tools/io_contention.cpp, profiles/r3/io_contention/). Each worker
// therefore starts with close_range(3, ~0U, CLOSE_RANGE_UNSHARE): its own table, holding only
// stdin/out/err (no duplicates of the process's other fds, so a pipe or file the process closes is
// not kept open by a worker). Such workers open files by full path.
static void make_fd_table_private() {
#ifndef CLOSE_RANGE_UNSHARE
#define CLOSE_RANGE_UNSHARE (1U << 1)
#endif
  (void)::syscall(SYS_close_range, 3u, ~0u, CLOSE_RANGE_UNSHARE);
}

// Every open() stores the opener's struct cred in the file (get_cred) and close() drops it (put_cred):
// two atomics on the cred's refcount, which all threads of a process share (forked processes get
// their own). Each pool worker therefore gets its own copy: capset() with the current capabilities
// commits a fresh, identical cred for the calling thread only (no privilege change). Bench, 5
// interleaved pairs: 385–402k vs 327–398k slices/s, JPEG-pair write CPU 0.17–0.22 vs 0.19–0.26 s
// per 40 steps (profiles/r3/private_cred/).
static void make_cred_private() {
  __user_cap_header_struct h{_LINUX_CAPABILITY_VERSION_3, 0};
  __user_cap_data_struct c[2]{};
  if (::syscall(SYS_capget, &h, c) == 0) (void)::syscall(SYS_capset, &h, c);
}

// Output directories of one run: an index per item and a creation hint per directory. Pool
// workers have private fd tables (above), so loads and writes take full paths: a per-worker cache
// of O_PATH directory fds had to be rebuilt for every run (each bench pass is a run), 16 workers ×
// ≈40 directories × open + close per pass, which cost more than the path walks (loads 28–32 vs
// 22–23 µs per slice, profiles/r3/depth/).
struct IoDirs {
  size_t ndirs = 0;
  // Per directory: 0 unknown, 1 being filled (files are created directly, see jpeg::write_jpeg_at),
  // 2 its files exist (opened without O_CREAT first).
  std::unique_ptr<std::atomic<uint8_t>[]> creating;
  std::vector<int32_t> out_dir;  // per item: its output directory's index
  explicit IoDirs(const std::vector<WorkItem>& items) {
    std::unordered_map<std::string, int32_t> idx;
    out_dir.resize(items.size());
    for (size_t i = 0; i < items.size(); ++i) {
      auto it = idx.emplace(items[i].out_dir, (int32_t)idx.size()).first;
      out_dir[i] = it->second;
    }
    ndirs = idx.size();
    creating.reset(new std::atomic<uint8_t>[std::max<size_t>(ndirs, 1)]);
    for (size_t k = 0; k < ndirs; ++k) creating[k].store(0, std::memory_order_relaxed);
  }
  IoDirs(const IoDirs&) = delete;
  IoDirs& operator=(const IoDirs&) = delete;
};

void hip_free_all(Slot& s) {
  if (s.host_only) {
    if (s.h_blob) munmap(s.h_blob, s.blob_bytes);
    if (s.h_out) munmap(s.h_out, s.out_bytes);
    delete[] s.h_sizes;
    return;
  }
  if (!s.arena) {
    if (s.h_blob) (void)hipHostFree(s.h_blob);
    if (s.h_out) (void)hipHostFree(s.h_out);
    if (s.h_sizes) (void)hipHostFree(s.h_sizes);
  }
  if (s.h_single) (void)hipHostFree(s.h_single);
  for (void* p : {(void*)s.d_blob, (void*)s.d_raw_x, (void*)s.d_med, (void*)s.d_tile_mm, (void*)s.d_f32, (void*)s.d_bits, (void*)s.d_srg_scratch, (void*)s.d_canvas,
                  (void*)s.jw.look, (void*)s.jw.ticket, (void*)s.jw.spill})
    if (p) (void)hipFree(p);
  if (s.ev0) (void)hipEventDestroy(s.ev0);
  if (s.ev1) (void)hipEventDestroy(s.ev1);
  if (s.ev2) (void)hipEventDestroy(s.ev2);
  if (s.stream && s.owns_stream) (void)hipStreamDestroy(s.stream);
}

// Streams created ahead of the engine (reserve_streams), per device.
std::mutex g_reserve_m;
std::vector<std::pair<int, hipStream_t>> g_reserved;
std::vector<int> g_copy_warm;  // devices whose copy path was brought up (warm_copy_path), guarded by g_reserve_m

// The first host→device copy of a process on `device` brings up the runtime's copy path: once per
// device, on the caller's stream, before any batch (reserve_streams or the engine constructor).
void warm_copy_once(int device, hipStream_t stream) {
  {
    std::lock_guard<std::mutex> g(g_reserve_m);
    if (std::find(g_copy_warm.begin(), g_copy_warm.end(), device) != g_copy_warm.end()) return;
    g_copy_warm.push_back(device);
  }
  warm_copy_path(stream);
}

hipStream_t take_stream(int device, const char* what) {
  {
    std::lock_guard<std::mutex> g(g_reserve_m);
    for (size_t i = 0; i < g_reserved.size(); ++i)
      if (g_reserved[i].first == device) {
        hipStream_t s = g_reserved[i].second;
        g_reserved.erase(g_reserved.begin() + (long)i);
        return s;
      }
  }
  hipStream_t s = nullptr;
  check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), what);
  return s;
}

template <class T>
T* dmalloc(size_t count, const char* what) {
  void* p = nullptr;
  check_hip(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)), what);
  return (T*)p;
}

}  // namespace

struct Engine::Impl {
  EngineConfig cfg;
  numa::Placement place;
  std::unique_ptr<ThreadPool> pool;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<uint8_t> jpeg_header;
  int32_t divs[64];
  PipeConsts pc{};
  // 12-bit transfer packing of slices whose samples fit (nm03/pack12.h); NM03_PACK12=0 disables.
  bool pack12_ = pack12::available();
  // Host-mapped bytes per image for the GPU encoder's stuffed output (EngineConfig::jpeg_out_cap).
  uint32_t out_cap_ = 0;
  bool host_only_ = false;  // EngineConfig::host_only
  // Host-only: the entropy-coded segments standing in for the GPU encoder's output (original,
  // processed) — the golden export of a phantom slice, so sizes match a real run.
  std::vector<uint8_t> tmpl_[2];

  explicit Impl(const EngineConfig& c) : cfg(c), place(c.device, c.cpus) {
    if (const char* e = std::getenv("NM03_PACK12"); e && *e && *e == '0') pack12_ = false;
    out_cap_ = cfg.jpeg_out_cap ? std::max<uint32_t>(64, cfg.jpeg_out_cap)
                                : (uint32_t)std::max<size_t>(32 * 1024, (size_t)cfg.render.out_width * cfg.render.out_height * 3 / 8) + 64;
    out_cap_ = (out_cap_ + 15u) & ~15u;  // 16-byte aligned segments (the encoder's dwordx4 stores)
    upload_chunk_ = cfg.upload_chunk_kb < 0 ? (size_t)2 << 20 : (size_t)cfg.upload_chunk_kb << 10;
    host_only_ = cfg.host_only;
    if (host_only_) upload_chunk_ = 0;  // nothing to upload
    if (cfg.batch_size < 1) cfg.batch_size = 1;
    if (cfg.streams < 1) cfg.streams = 1;
    if (cfg.max_dim < 16) cfg.max_dim = 16;
    if (cfg.max_dim > kMaxSliceDim) throw DeviceError("max_dim above " + std::to_string(kMaxSliceDim) + " not supported");
    const auto& p = cfg.pipe;
    if (p.median_window != 3 && p.median_window != 5 && p.median_window != 7 && p.median_window != 9)
      throw DeviceError("median window must be 3, 5, 7 or 9");
    if (p.sharpen_mask < 1 || p.sharpen_mask > 15 || !(p.sharpen_mask & 1))
      throw DeviceError("sharpen mask must be odd and ≤ 15");
    if (p.dilation_size < 1 || p.dilation_size > 63 || p.erosion_size < 1 || p.erosion_size > 63)
      throw DeviceError("morphology sizes must be in [1, 63]");
    pc.nmin = p.norm_min;
    pc.nmax = p.norm_max;
    pc.nlow = p.norm_low;
    pc.nhigh = p.norm_high;
    pc.cmin = p.clip_min;
    pc.cmax = p.clip_max;
    pc.gain = p.sharpen_gain;
    pc.band_lo = p.srg_min;
    pc.band_hi = p.srg_max;
    gaussian_taps(p.sharpen_sigma, p.sharpen_mask, pc.taps);
    pc.mask_radius = p.sharpen_mask / 2;
    pc.median_k = p.median_window;
    pc.connectivity = p.srg_connectivity == 8 ? 8 : 4;
    pc.dilation_size = p.dilation_size;
    pc.erosion_size = p.erosion_size;
    pc.border_radius = cfg.render.border_radius;
    pc.se_disc = p.se_shape == kSeDisc ? 1 : 0;
    jpeg::Tables t = jpeg::make_tables(cfg.render.jpeg_quality);
    for (int i = 0; i < 64; ++i) divs[i] = t.div_luma[i];
    if (cfg.render.jpeg_sampling < jpeg::kSampling420 || cfg.render.jpeg_sampling > jpeg::kSamplingGray)
      throw std::invalid_argument("jpeg_sampling must be 0 (4:2:0), 1 (4:4:4) or 2 (gray)");
    jpeg_header = jpeg::make_header(cfg.render.out_width, cfg.render.out_height, t,
                                    (jpeg::Sampling)cfg.render.jpeg_sampling);
    if (cfg.render.out_width % 16 || cfg.render.out_height % 16)
      throw DeviceError("canvas size must be a multiple of 16");
    if (host_only_) make_templates();
    const double t0 = now_s();
    if (!host_only_) {
      check_hip(hipSetDevice(cfg.device), "hipSetDevice");
      // Every code object loaded here, on one thread, before any batch is launched: HIP otherwise
      // loads a module at the first launch of one of its kernels, from whichever slot thread gets
      // there first (a no-op when the CLI's start-up thread already did it). The 2D engine never
      // launches the volume or threshold kernels.
      preload_kernels(/*with_volume=*/false);
      d_lut_ = dmalloc<float>(kLutArenaFloats, "hipMalloc norm tables");
    }
    const double t1 = now_s();
    // Host threads and pinned buffers on the GPU's socket (numa.h).
    pool = std::make_unique<ThreadPool>(cfg.threads, [this](int i) {
      place.bind_this_thread();
      make_fd_table_private();
      make_cred_private();
      // Asynchronous signals go to other threads: a pool worker's reads are never cut short.
      // Synchronous fault signals stay unblocked (a blocked SIGSEGV/SIGBUS is forced to SIG_DFL,
      // bypassing the crash handler and sanitizers), and so does SIGPROF for sampling profilers.
      sigset_t all;
      sigfillset(&all);
      for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGTRAP, SIGABRT, SIGPROF}) sigdelset(&all, sig);
      pthread_sigmask(SIG_BLOCK, &all, nullptr);
    });
    const double t2 = now_s();
    // Slot 0 is built here (its failure fails the constructor). The others too, unless
    // EngineConfig::lazy_slots hands them to their worker threads; a slot that cannot be built
    // (out of memory) leaves the engine with fewer streams, not failed.
    std::string slot_ms;
    slots.resize((size_t)cfg.streams);
    place.run_bound([&] {
      const double ts = now_s();
      std::string split;
      if (!host_only_ && !cfg.lazy_slots) make_arenas((int)slots.size());
      slots[0] = make_slot(&split, 0);
      slot_ms = std::to_string((int)((now_s() - ts) * 1e4) / 10.0).substr(0, 5) + " (" + split + ")";
      if (cfg.lazy_slots) return;
      for (size_t i = 1; i < slots.size(); ++i) {
        const double tb = now_s();
        try {
          slots[i] = make_slot(nullptr, (int)i);
        } catch (const std::exception& e) {
          log_warn("engine slot " + std::to_string(i) + " unavailable, running with fewer streams: " + e.what());
        }
        slot_ms += ", +" + std::to_string((int)((now_s() - tb) * 1e4) / 10.0).substr(0, 5);
      }
    });
    if (!host_only_ && slots[0]) warm_copy_once(cfg.device, slots[0]->stream);  // no-op after reserve_streams
    const double t3 = now_s();
    building_ = cfg.lazy_slots ? (int)slots.size() - 1 : 0;
    start_workers();
    const double t4 = now_s();
    log_info("engine on device " + std::to_string(cfg.device) + ": batch " + std::to_string(cfg.batch_size) + ", " +
             std::to_string(cfg.streams) + " streams, " + std::to_string(cfg.threads) + " host threads, max_dim " +
             std::to_string(cfg.max_dim) + ", " + place.describe() + "; set-up ms: device " +
             std::to_string((t1 - t0) * 1e3) + ", pool " + std::to_string((t2 - t1) * 1e3) + ", slots " + slot_ms +
             ", workers " + std::to_string((t4 - t3) * 1e3));
  }

  ~Impl() {
    stop_workers();
    if (!host_only_) (void)hipSetDevice(cfg.device);
    for (auto& s : slots)
      if (s) hip_free_all(*s);
    if (shared_up_) (void)hipStreamDestroy(shared_up_);
    if (d_lut_) (void)hipFree(d_lut_);
    if (pin_arena_) (void)hipHostFree(pin_arena_);
    if (map_arena_) (void)hipHostFree(map_arena_);
  }

  // ---- normalise+clip lookup tables (K1b) ------------------------------------------------------
  // norm_clip_key depends on the key and the slice's (type, stored bits, slope, intercept) only;
  // its IEEE division is ≈13 VALU per key in the sharpen's tile load. Each distinct parameter set
  // gets a table over its 2^stored_bits possible keys (16 KiB for 12-bit data), built once on the
  // host with the very same function and kept in a device arena; SliceDesc::lut_off / lut_base
  // point the kernel at it. A cohort has a handful of sets; when the arena is full (or the bit
  // depth is unusual) a slice keeps lut_off = kNoLut and the kernel evaluates the function.
  struct LutSet {
    uint8_t type, bits;
    uint32_t slope, intercept;  // bit patterns
    uint32_t off, base;
  };
  static constexpr size_t kLutArenaFloats = size_t(1) << 20;  // 4 MiB
  std::mutex lut_m_;
  std::vector<LutSet> luts_;
  float* d_lut_ = nullptr;  // allocated by the constructor, never moved
  size_t lut_used_ = 0;
  // Per-thread cache of the last set looked up, tagged with the engine's serial number (not its
  // address, which a later engine may reuse).
  static inline std::atomic<uint64_t> engine_serials_{0};
  const uint64_t serial_ = ++engine_serials_;
  static uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
  }
  // (lut_off, lut_base) for the parameter set; {kNoLut, 0} when there is no table. A new table is
  // built on the device on the calling slot's `stream` and waited for before it is published (once
  // per format and engine; other slots find it only when it is complete).
  std::pair<uint32_t, uint32_t> norm_lut(uint8_t type, uint8_t bits, float slope, float intercept, hipStream_t stream) {
    if (host_only_ || bits < 1 || bits > 16) return {kNoLut, 0u};
    const uint32_t sl = fbits(slope), ic = fbits(intercept);
    thread_local uint64_t last_owner = 0;
    thread_local LutSet last{};
    if (last_owner == serial_ && last.type == type && last.bits == bits && last.slope == sl && last.intercept == ic)
      return {last.off, last.base};
    std::lock_guard<std::mutex> g(lut_m_);
    for (const LutSet& e : luts_)
      if (e.type == type && e.bits == bits && e.slope == sl && e.intercept == ic) {
        last_owner = serial_;
        last = e;
        return {e.off, e.base};
      }
    const uint32_t n = 1u << bits;
    if (!d_lut_ || lut_used_ + n > kLutArenaFloats) return {kNoLut, 0u};
    // Keys of signed data are the sign-extended samples with bit 15 flipped: 0x8000 ± 2^(bits−1).
    const uint32_t base = type == kI16 ? 0x8000u - n / 2 : 0u;
    NormClip nc;
    nc.slope = slope;
    nc.intercept = intercept;
    nc.nmin = pc.nmin;
    nc.nmax = pc.nmax;
    nc.nlow = pc.nlow;
    nc.nhigh = pc.nhigh;
    nc.cmin = pc.cmin;
    nc.cmax = pc.cmax;
    launch_build_norm_lut(d_lut_ + lut_used_, n, base, type, nc, stream);
    check_hip(hipStreamSynchronize(stream), "norm table");
    const LutSet e{type, bits, sl, ic, (uint32_t)lut_used_, base};
    lut_used_ += n;
    luts_.push_back(e);
    last_owner = serial_;
    last = e;
    return {e.off, e.base};
  }

  // Every slot's H2D copies go through one engine-wide stream (each slot's own stream was the
  // round-3 alternative), so at most one SDMA upload runs at a time: two or more concurrent copies
  // from different streams drop the copy engine's aggregate rate on the MI355X boxes
  // (tools/h2d_probe.hip: 28 vs 53-57 GB/s), and in the bench 20-40% of the upload time had two or
  // more in flight (profiles/r3/timeline/). The slot's kernels wait on an event after its last copy.
  // Measured: rank-0 H2D time per 50 steps 0.056 vs 0.080-0.107 s, 377-399k vs 310-334k slices/s
  // (4 interleaved pairs, profiles/r3/upload_stream/).
  hipStream_t shared_up_ = nullptr;
  std::mutex shared_up_m_;
  hipStream_t upload_stream() {
    std::lock_guard<std::mutex> g(shared_up_m_);
    if (!shared_up_) shared_up_ = take_stream(cfg.device, "hipStreamCreate upload");
    return shared_up_;
  }

  // ---- per-batch timeline (NM03_BATCH_TRACE=1) --------------------------------------------------
  // One record per batch, in ms since the run was submitted: claimed by its slot, loads finished,
  // kernels enqueued, GPU done, exports done. Printed by finish(): where a cold run's time goes
  // (slot build, first-use costs, pipeline fill) without a profiler's own start-up in the way.
  struct BatchMark {
    int slot = 0;
    size_t first = 0, count = 0;
    double claim = 0, loaded = 0, enq = 0, gpu = 0, end = 0;
  };
  static bool batch_trace() {
    static const bool on = [] {
      const char* e = std::getenv("NM03_BATCH_TRACE");
      return e && *e && *e != '0';
    }();
    return on;
  }

  void make_templates() {
    golden::SliceInput in;
    in.w = in.h = 256;
    in.raw.resize(256 * 256);
    synth::phantom_slice(256, 256, 3, 12, 25, 20250404, in.raw.data());
    const golden::SliceResult r = golden::run(in, cfg.pipe, false);
    const golden::SliceJpegs j = golden::export_jpegs(in, r, cfg.pipe, cfg.render);
    const std::vector<uint8_t>* files[2] = {&j.original, &j.processed};
    for (int k = 0; k < 2; ++k) {
      const auto& f = *files[k];
      if (f.size() < jpeg_header.size() + 2 || !std::equal(jpeg_header.begin(), jpeg_header.end(), f.begin()))
        throw DeviceError("host-only engine: unexpected template JPEG layout");
      tmpl_[k].assign(f.begin() + (long)jpeg_header.size(), f.end() - 2);
      if (tmpl_[k].size() > out_cap_) throw DeviceError("host-only engine: template exceeds the output capacity");
    }
  }

  // Pinned host memory of every constructor-built slot in two allocations (one page-locked, one
  // host-mapped) instead of three per slot: each hipHostMalloc costs ≈ 0.7–1.1 ms on a cold process
  // whatever its size (tools/queue_probe.cpp), the bulk of the engine constructor.
  uint8_t* pin_arena_ = nullptr;
  uint8_t* map_arena_ = nullptr;
  uint8_t* map_arena_dev_ = nullptr;
  size_t pin_stride_ = 0, map_stride_ = 0;
  void make_arenas(int n) {
    Slot probe;
    layout(probe);
    pin_stride_ = align_up(probe.blob_bytes, 4096);
    map_stride_ = align_up((size_t)out_cap_ * probe.cap_canvases + sizeof(int32_t) * probe.cap_canvases, 4096);
    check_hip(hipHostMalloc((void**)&pin_arena_, pin_stride_ * n, hipHostMallocDefault), "hipHostMalloc blob arena");
    check_hip(hipHostMalloc((void**)&map_arena_, map_stride_ * n, hipHostMallocMapped), "hipHostMalloc out arena");
    check_hip(hipHostGetDevicePointer((void**)&map_arena_dev_, map_arena_, 0), "hipHostGetDevicePointer out arena");
  }

  // Capacities and blob layout of a slot (no allocation).
  void layout(Slot& s) const {
    const int B = cfg.batch_size;
    const int md = cfg.max_dim;
    s.cap_slices = B;
    s.cap_canvases = std::max(2 * B, 5);
    s.cap_pixels = (size_t)B * align_up((size_t)md * md, 8);
    const size_t tx_med = (md + kMedTileW - 1) / kMedTileW, ty_med = (md + kMedTileH - 1) / kMedTileH;
    const size_t tx_shp = (md + kShpTileW - 1) / kShpTileW, ty_shp = (md + kShpTileH - 1) / kShpTileH;
    s.max_medt = (size_t)B * tx_med * ty_med;
    s.max_shpt = (size_t)B * tx_shp * ty_shp;
    size_t o = 0;
    s.off_stats = o;
    o = align_up(o + (size_t)B * sizeof(SliceStats), kAlign);
    s.off_desc = o;
    o = align_up(o + (size_t)B * sizeof(SliceDesc), kAlign);
    s.off_medt = o;
    o = align_up(o + s.max_medt * sizeof(TileDesc), kAlign);
    s.off_shpt = o;
    o = align_up(o + s.max_shpt * sizeof(TileDesc), kAlign);
    s.off_seeds = o;
    o = align_up(o + (size_t)B * kMaxSeeds * sizeof(SeedXY), kAlign);
    s.off_render = o;
    o = align_up(o + (size_t)s.cap_canvases * sizeof(RenderDesc), kAlign);
    s.off_jpeg = o;
    o = align_up(o + (size_t)s.cap_canvases * sizeof(JpegDesc), kAlign);
    s.raw_base = o;
    s.hole_slack = cfg.pack_slack < 0 ? (size_t)std::max(cfg.threads, 1) * align_up((size_t)md * md / 4 * 3, 8)
                                      : (size_t)cfg.pack_slack * std::max(cfg.threads, 1);
    s.blob_bytes = o + (s.cap_pixels + s.hole_slack) * sizeof(uint16_t);
  }

  // `split` (optional): milliseconds per allocation phase, for the start-up log. `arena_slot` ≥ 0:
  // the slot's pinned buffers are that part of the engine's arenas (make_arenas).
  std::unique_ptr<Slot> make_slot(std::string* split = nullptr, int arena_slot = -1) {
    double tm = now_s();
    auto mark = [&](const char* what) {
      if (!split) return;
      const double t = now_s();
      *split += (split->empty() ? "" : ", ") + std::string(what) + " " + std::to_string((int)((t - tm) * 1e4) / 10.0).substr(0, 4);
      tm = t;
    };
    auto sp = std::make_unique<Slot>();
    Slot& s = *sp;
    layout(s);
    const int B = cfg.batch_size;
    const int md = cfg.max_dim;
    if (host_only_) {
      s.host_only = true;
      s.out_bytes = (size_t)out_cap_ * s.cap_canvases;
      auto map = [](size_t bytes) {
        void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        if (p == MAP_FAILED) throw DeviceError("host-only engine: cannot map slot buffers");
        return static_cast<uint8_t*>(p);
      };
      try {
        s.h_blob = map(s.blob_bytes);
        s.raw_cpu = s.h_blob + s.raw_base;
        s.h_out = map(s.out_bytes);
        s.h_sizes = new int32_t[(size_t)s.cap_canvases];
      } catch (...) {
        hip_free_all(s);
        throw;
      }
      return sp;
    }
    try {
      if (cfg.shared_stream) {
        s.stream = s.up = upload_stream();  // the engine's one stream (destroyed by ~Impl)
        s.owns_stream = false;
      } else {
        s.stream = take_stream(cfg.device, "hipStreamCreate");
        s.up = upload_stream();
      }
      mark("streams");
      // Timing events (the h2d / kernel split of StageTimes): events without timestamps and only the
      // records the stream order needs measured no different (profiles/r6/ab_pool/spin_mutex_rejected/
      // bench_new_noevt_*). Batch completion is polled by the slot thread (wait_batch): no
      // blocking-sync event.
      check_hip(hipEventCreateWithFlags(&s.ev0, hipEventDefault), "hipEventCreate");
      check_hip(hipEventCreateWithFlags(&s.ev1, hipEventDefault), "hipEventCreate");
      check_hip(hipEventCreateWithFlags(&s.ev2, hipEventDefault), "hipEventCreate");
      mark("events");
      if (arena_slot >= 0 && pin_arena_) {
        s.arena = true;
        s.h_blob = pin_arena_ + (size_t)arena_slot * pin_stride_;
      } else {
        check_hip(hipHostMalloc((void**)&s.h_blob, s.blob_bytes, hipHostMallocDefault), "hipHostMalloc blob");
      }
      mark("pinned blob");
      // +64 B tail slack: the median's packed-group loads read whole dwords (k1_median.hip).
      s.d_blob = dmalloc<uint8_t>(s.blob_bytes + 64, "hipMalloc blob");
      s.raw_cpu = s.h_blob + s.raw_base;
      s.d_raw_x = dmalloc<uint16_t>(s.cap_pixels, "hipMalloc raw");
      s.d_med = dmalloc<uint16_t>(s.cap_pixels, "hipMalloc median");
      s.d_tile_mm = dmalloc<uint32_t>(2 * s.max_medt, "hipMalloc tile ranges");
      s.d_f32 = dmalloc<float>(s.cap_pixels, "hipMalloc f32");
      s.plane_words = (size_t)B * md * ((md + 63) / 64);
      s.d_bits = dmalloc<uint64_t>(s.plane_words * kNumPlanes, "hipMalloc bits");
      if (md > kSrgMaxDim) s.d_srg_scratch = dmalloc<uint64_t>((size_t)B * 4 * srg_plane_words(md, md), "hipMalloc srg scratch");
      const int cw = cfg.render.out_width, ch = cfg.render.out_height;
      const size_t canvas_bytes = (size_t)cw * ch;
      const size_t blocks = canvas_bytes / 64;
      s.d_canvas = dmalloc<uint8_t>(canvas_bytes * s.cap_canvases, "hipMalloc canvas");
      s.jw.look_cap = (size_t)s.cap_canvases * ((blocks + 255) / 256);
      s.jw.look = dmalloc<uint64_t>(6 * s.jw.look_cap, "hipMalloc look-back");
      mark("device buffers");
      // Cleared on the slot's own stream, ahead of every kernel that reads them (look-back records,
      // tickets): no host wait here (the synchronous form cost ≈8 ms of a cold CLI's engine set-up).
      check_hip(hipMemsetAsync(s.jw.look, 0, 6 * s.jw.look_cap * sizeof(uint64_t), s.stream), "memset look-back");
      s.jw.ticket = dmalloc<uint32_t>(s.cap_canvases, "hipMalloc tickets");
      s.jw.spill = dmalloc<uint32_t>(s.jw.look_cap * 256 * 56, "hipMalloc jpeg spill");
      check_hip(hipMemsetAsync(s.jw.ticket, 0, sizeof(uint32_t) * s.cap_canvases, s.stream), "memset tickets");
      mark("memsets");
      const size_t out_bytes = (size_t)out_cap_ * s.cap_canvases;
      if (s.arena) {
        const size_t off = (size_t)arena_slot * map_stride_;
        s.h_out = map_arena_ + off;
        s.d_out = map_arena_dev_ + off;
        s.h_sizes = reinterpret_cast<int32_t*>(map_arena_ + off + out_bytes);
        s.d_sizes = reinterpret_cast<int32_t*>(map_arena_dev_ + off + out_bytes);
      } else {
        check_hip(hipHostMalloc((void**)&s.h_out, out_bytes, hipHostMallocMapped), "hipHostMalloc out");
        check_hip(hipHostGetDevicePointer((void**)&s.d_out, s.h_out, 0), "hipHostGetDevicePointer out");
        check_hip(hipHostMalloc((void**)&s.h_sizes, sizeof(int32_t) * s.cap_canvases, hipHostMallocMapped),
                  "hipHostMalloc sizes");
        check_hip(hipHostGetDevicePointer((void**)&s.d_sizes, s.h_sizes, 0), "hipHostGetDevicePointer sizes");
      }
      mark("mapped out");
    } catch (...) {
      hip_free_all(s);
      throw;
    }
    return sp;
  }

  // ---- progressive upload --------------------------------------------------------------------
  // While a batch loads, queue the H2D copy of every finished, contiguous prefix of the raw region
  // once it has grown by `upload_chunk_` bytes: the copy engine starts after a few loads instead
  // of after the whole batch (pipeline fill at the start of a run, load/upload overlap inside
  // every batch). EngineConfig::upload_chunk_kb (0 = one upload per batch after all loads) sets the minimum;
  // batches of large slices use a quarter of the batch (512² × 64: 8 MiB — many concurrent small
  // copies cost 10% of the upload rate there, profiles/iter5/c4_sweep.txt).
  size_t upload_chunk_ = 2u << 20;

  void upload_progress(Slot& s, size_t count) {
    size_t next = 0, seen = 0;
    size_t chunk = 0;  // bytes; at least upload_chunk_, and a quarter of the batch (large slices)
    for (;;) {
      bool all;
      {
        // Loaders count without the lock and take it only to wake this thread when it announced that
        // it sleeps (prog_waiting, seq_cst on both sides: a count that raced past the check is seen).
        std::unique_lock<std::mutex> g(s.prog_m);
        // Wake at the load count whose slices (of the first one's size) fill the next chunk; loads
        // that finish out of order just make a wake-up find a shorter prefix and sleep again.
        size_t target = seen + 1;
        if (chunk) {  // set once allocation 0 is done: its length is final
          const size_t per = s.allocs[0].len * 2;
          if (per) target = std::max(target, (s.uploaded * 2 + chunk + per - 1) / per);
        }
        s.wake_at.store(target, std::memory_order_seq_cst);
        s.prog_waiting.store(true, std::memory_order_seq_cst);
        s.prog_cv.wait(g, [&] { return s.loads_finished.load(std::memory_order_seq_cst) != seen; });
        s.prog_waiting.store(false, std::memory_order_relaxed);
        seen = s.loads_finished.load(std::memory_order_acquire);
        all = seen == count;
      }
      const size_t n = s.n_allocs();
      size_t end = s.uploaded;
      while (next < n && s.allocs[next].done.load(std::memory_order_acquire)) {
        end = s.allocs[next].off + s.allocs[next].len;
        ++next;
      }
      if (all) return;  // the remainder goes with the tables in build_and_run
      if (!chunk && next > 0) {
        chunk = std::max(upload_chunk_, count * s.allocs[0].len * 2 / 4);
        if (chunk >= count * s.allocs[0].len * 2) {  // a small batch: one upload with the tables
          s.progress_quiet.store(true, std::memory_order_relaxed);
          return;
        }
      }
      if (chunk && (end - s.uploaded) * 2 >= chunk) {
        if (!s.upload_started) {
          check_hip(hipEventRecord(s.ev0, s.up), "event");
          s.upload_started = true;
        }
        check_hip(hipMemcpyAsync(s.d_blob + s.raw_base + s.uploaded * 2, s.h_blob + s.raw_base + s.uploaded * 2,
                                 (end - s.uploaded) * 2, hipMemcpyHostToDevice, s.up),
                  "H2D pixels");
        s.uploaded = end;
      }
    }
  }

  // ---- batch completion ----------------------------------------------------------------------
  // The slot thread waits for its batch here. A blocking-sync hipEventSynchronize still spins in
  // the runtime before it sleeps, which cost ≈0.7 ms of slot-thread CPU per batch — CPU the
  // loader/writer pool needs. Instead the slot sleeps in short steps (timer slack lowered to 1 µs on
  // slot threads) and queries the event: a few µs of CPU per batch, ≤ 20 µs of added latency,
  // hidden by the other slots in flight (round-1 A/B, profiles/iter2/).
  //
  // The slot first sleeps through most of the time its recent batches took from enqueue to
  // completion (EMA, per slice × this batch's slices), then polls: ~10 wake-ups per batch instead of
  // one per poll interval over the whole batch (each wake-up is a context switch of host CPU the
  // loaders/writers need). Per slice, so a short batch after full ones (a strong-scaling shard cut
  // into ⌈shard / streams⌉-slice batches) is not slept through at the full batches' time: fixed
  // per-batch costs make small batches slower per slice, so the scaled estimate errs short (more
  // polls), never long.
  void wait_batch(Slot& s, hipEvent_t ev, double t_enq, int nslices) {
    // A small batch (≤ 16 slices: a strong-scaling shard's, latency-bound) spin-polls its event for
    // up to 1 ms instead of sleeping through the slot's recent per-slice mean: that mean comes from
    // full, queued batches, and scaled to 15 slices it overslept completed batches by 80–190 µs in
    // the single-pass trace (profiles/r3/small_upload/hip_trace_inline.txt).
    if (nslices <= 16) {
      const double until = t_enq + 1e-3;
      for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) check_hip(e, "batch sync");
        if (now_s() > until) break;
        for (int k = 0; k < 32; ++k) __builtin_ia32_pause();
      }
    }
    const double scale = (double)std::max(1, nslices);
    // Sleep through most of the batch's expected time (0.8 × the recent mean), in chunks of at
    // most 250 µs with an event check between them, then poll. One long sleep would feed itself:
    // a slow batch (GPU shared with another process, host CPU stolen) raises the mean, the next
    // batches oversleep by the same amount, and the mean — measured from these overslept waits —
    // decays by only ≈5% per batch. Chunked, a wait ends within one chunk of the batch's real
    // completion, so the mean tracks the GPU again after a few batches.
    const double target = 0.8 * s.batch_ema_s * scale;
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) check_hip(e, "batch sync");
      const double ahead = target - (now_s() - t_enq);
      if (ahead > 100e-6)
        std::this_thread::sleep_for(std::chrono::duration<double>(std::min(ahead, 250e-6)));
      else
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    const double took = (now_s() - t_enq) / scale;
    s.batch_ema_s = s.batch_ema_s > 0 ? 0.75 * s.batch_ema_s + 0.25 * took : took;
  }

  // ---- loading -------------------------------------------------------------------------------
  void load_into(Slot& s, int i, size_t item, const std::string& path, SliceStatus& st, std::atomic<int64_t>& load_ns,
                 std::atomic<int64_t>& bytes_in) {
    thread_local std::vector<uint8_t> buf;
    TraceRange tr("nm03.load");
    const double t0 = now_s();
    try {
      if (fault_plan().corrupt_dicom == (int64_t)item) throw SliceError("injected fault: corrupt DICOM data");
      // Staged read: one whole-file pread into a cache-resident scratch buffer, the pack/copy into
      // the pinned blob from there. Mapping the file instead measured 5x the loader CPU (mmap +
      // populate + munmap under the mm lock; 47.6k vs 267k slices/s, profiles/iter6/
      // mapped_load_ab.txt), and a pread of the pixels straight into the blob was slower too
      // (profiles/r4/): both removed in round 4.
      dicom::SliceFile file(AT_FDCWD, path.c_str(), path, dicom::ReadMode::kStaged);
      const dicom::Header& h = file.header(buf);
      const int frame = dicom::select_frame(h, cfg.pipe.frame);
      const size_t n = file.size();  // after header(): staged reads learn the size from the read
      const int md = cfg.pipe.min_dim;
      if (md > 0 && (h.cols < md || h.rows < md)) {
        st.code = kSliceTooSmall;
        st.message = "Image dimensions too small: " + std::to_string(h.cols) + "x" + std::to_string(h.rows);
      } else if (h.cols > cfg.max_dim || h.rows > cfg.max_dim) {
        st.code = kSliceLoadError;
        st.message = "Image dimensions " + std::to_string(h.cols) + "x" + std::to_string(h.rows) +
                     " exceed the engine limit " + std::to_string(cfg.max_dim);
      } else {
        const size_t npix = (size_t)h.rows * h.cols;
        // 12-bit transfer packing (staged or mapped raw 16-bit data), written straight into the
        // pinned blob with streaming stores:
        //  * BitsStored ≤ 12: every consumer masks samples to the stored bits (key_from_raw), so the
        //    low 12 bits are the slice — packed unconditionally, one pass;
        //  * wider: packed and range-checked in the same pass (pack_stream_checked) under a hole
        //    credit — if a sample needs more bits, the packed reservation is grown in place to the
        //    16-bit size when it is still the last one, or else abandoned (a hole, paid from the
        //    credit) for a new 16-bit one. Without credit left: range check first (fits12), then
        //    pack — two passes, no hole.
        const uint16_t* samples = pack12_ ? file.staged_samples(frame) : nullptr;
        const size_t plen = align_up(npix / 4 * 3, 8), ulen = align_up(npix, 8);  // u16 elements
        const bool packable = samples && pack12::available() && (npix & 15) == 0;
        const size_t cap = s.cap_pixels + s.hole_slack;
        size_t idx = 0, off = 0;
        bool packed = false, reserved = false, credit = false;
        // Claims `len` elements at the end of the raw region and the next allocation index in one
        // CAS (Slot::alloc_word); the entry's offset and length are published by its `done` flag.
        auto reserve = [&](size_t len) {
          uint64_t w = s.alloc_word.load(std::memory_order_relaxed);
          for (;;) {
            const size_t used = (size_t)(w & Slot::kUsedMask), n = (size_t)(w >> Slot::kAllocShift);
            if (used + len > cap) throw SliceError("batch pixel capacity exceeded");
            if (n >= s.max_allocs) throw SliceError("batch allocation table full");
            const uint64_t nw = ((uint64_t)(n + 1) << Slot::kAllocShift) | (uint64_t)(used + len);
            if (s.alloc_word.compare_exchange_weak(w, nw, std::memory_order_acq_rel, std::memory_order_relaxed)) {
              idx = n;
              off = used;
              break;
            }
          }
          s.allocs[idx].off = off;
          s.allocs[idx].len = len;
          reserved = true;
        };
        try {
          const bool low12 = h.bits_stored <= 12;
          if (packable && !low12) {  // take plen of credit if there is that much (lock-free)
            size_t c = s.hole_credit.load(std::memory_order_relaxed);
            while (c >= plen && !s.hole_credit.compare_exchange_weak(c, c - plen, std::memory_order_acq_rel)) {
            }
            credit = c >= plen;
          }
          if (credit) {
            reserve(plen);
            uint8_t* dst = reinterpret_cast<uint8_t*>(reinterpret_cast<uint16_t*>(s.raw_cpu) + off);
            packed = pack12::pack_stream_checked(samples, npix, dst);
            if (packed) {
              s.hole_credit.fetch_add(plen, std::memory_order_acq_rel);
            } else {
              // Grow in place while this is still the last allocation, else leave a hole (uploaded,
              // unused; paid from the credit) and take a 16-bit allocation.
              uint64_t last = ((uint64_t)(idx + 1) << Slot::kAllocShift) | (uint64_t)(off + plen);
              const uint64_t grown = ((uint64_t)(idx + 1) << Slot::kAllocShift) | (uint64_t)(off + ulen);
              if (off + ulen <= cap &&
                  s.alloc_word.compare_exchange_strong(last, grown, std::memory_order_acq_rel, std::memory_order_relaxed)) {
                s.allocs[idx].len = ulen;
                s.hole_credit.fetch_add(plen, std::memory_order_acq_rel);
              } else {
                s.allocs[idx].done.store(true, std::memory_order_release);
                reserve(ulen);
              }
              file.pixels16(reinterpret_cast<uint16_t*>(s.raw_cpu) + off, frame);
            }
          } else {
            packed = packable && (low12 || pack12::fits12(samples, npix));
            reserve(packed ? plen : ulen);
            uint16_t* dst = reinterpret_cast<uint16_t*>(s.raw_cpu) + off;
            if (packed) {
              pack12::pack_stream(samples, npix, reinterpret_cast<uint8_t*>(dst));
            } else {
              file.pixels16(dst, frame);
            }
          }
        } catch (...) {
          if (reserved) s.allocs[idx].done.store(true, std::memory_order_release);  // space stays unused
          throw;
        }
        s.allocs[idx].done.store(true, std::memory_order_release);
        LoadedSlice& L = s.loaded[i];
        L.w = h.cols;
        L.h = h.rows;
        L.type = h.type == kU8 ? kU16 : h.type;
        L.stored_bits = (uint8_t)(h.type == kU8 ? 8 : h.bits_stored);
        L.slope = cfg.pipe.apply_rescale ? h.slope : 1.f;
        L.intercept = cfg.pipe.apply_rescale ? h.intercept : 0.f;
        L.sx = h.spacing_x;
        L.sy = h.spacing_y;
        L.blob_off = (uint32_t)off;
        L.packed = packed;
        L.ok = true;
        st.code = kSliceOk;
        bytes_in += (int64_t)n;
      }
    } catch (const std::exception& e) {
      st.code = kSliceLoadError;
      st.message = e.what();
    }
    load_ns += (int64_t)((now_s() - t0) * 1e9);
  }

  static bool outputs_exist(const WorkItem& w) {
    const std::string base = cohort::with_slash(w.out_dir) + cohort::stem(w.path);
    return access((base + "_original.jpg").c_str(), F_OK) == 0 && access((base + "_processed.jpg").c_str(), F_OK) == 0;
  }

  // ---- descriptor build + GPU enqueue --------------------------------------------------------
  // mode 0: export pair (original, processed); mode 1: test_pipeline (5 canvases, all planes).
  // (seeds_*: per-thread cache of reference_seeds for build_and_run; slot threads run concurrently.)
  static inline thread_local std::vector<Seed> seeds_cache_;
  static inline thread_local int seeds_w_ = 0, seeds_h_ = 0;
  void build_and_run(Slot& s, int mode, StageTimes* acc, BatchMark* mark = nullptr) {
    const int nl = (int)s.live.size();
    uint8_t* hb = s.h_blob;
    auto* stats = reinterpret_cast<SliceStats*>(hb + s.off_stats);
    auto* desc = reinterpret_cast<SliceDesc*>(hb + s.off_desc);
    auto* medt = reinterpret_cast<TileDesc*>(hb + s.off_medt);
    auto* shpt = reinterpret_cast<TileDesc*>(hb + s.off_shpt);
    auto* seeds = reinterpret_cast<SeedXY*>(hb + s.off_seeds);
    auto* rd = reinterpret_cast<RenderDesc*>(hb + s.off_render);
    auto* jd = reinterpret_cast<JpegDesc*>(hb + s.off_jpeg);
    int nmed = 0, nshp = 0, nseed = 0, ncanv = 0;
    s.any_canvas = false;
    uint32_t mask_off = 0;
    s.max_w = s.max_h = 0;
    const int cw = cfg.render.out_width, ch = cfg.render.out_height;
    const uint32_t canvas_bytes = (uint32_t)(cw * ch);
    const uint8_t fill = opacity_u8(cfg.render.label_opacity), bval = opacity_u8(cfg.render.border_opacity);
    uint32_t xoff = 0;  // expanded-sample offsets (K0 output) in batch order
    for (int c = 0; c < nl; ++c) {
      const LoadedSlice& L = s.loaded[s.live[c]];
      stats[c] = SliceStats{0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0u};
      SliceDesc& d = desc[c];
      std::memset(&d, 0, sizeof(d));
      const uint32_t raw_off = xoff;
      xoff += (uint32_t)align_up((size_t)L.w * L.h, 8);
      d.raw_off = raw_off;
      d.blob_off = L.blob_off;
      d.flags = L.packed ? kSliceFlagPacked12 : 0;
      d.w = (uint16_t)L.w;
      d.h = (uint16_t)L.h;
      d.wpr = (uint16_t)((L.w + 63) / 64);
      d.mask_off = mask_off;
      mask_off += (uint32_t)(d.h * d.wpr);
      d.type = L.type;
      d.stored_bits = L.stored_bits;
      d.slope = L.slope;
      d.intercept = L.intercept;
      std::tie(d.lut_off, d.lut_base) = norm_lut(L.type, L.stored_bits, L.slope, L.intercept, s.stream);
      d.f32_off = raw_off;
      // Seeds depend on the slice size only: reuse the last size's list (a batch is nearly always
      // one size) instead of building a vector per slice on the slot thread.
      if (L.w != seeds_w_ || L.h != seeds_h_) {
        seeds_cache_ = reference_seeds(L.w, L.h);
        seeds_w_ = L.w;
        seeds_h_ = L.h;
      }
      const auto& sv = seeds_cache_;
      d.seed_off = (uint32_t)nseed;
      d.seed_count = (uint16_t)std::min<size_t>(sv.size(), kMaxSeeds);
      for (int k = 0; k < d.seed_count; ++k) seeds[nseed++] = SeedXY{(int16_t)sv[k].x, (int16_t)sv[k].y};
      d.med_tile0 = (uint32_t)nmed;
      for (int ty = 0; ty < (L.h + kMedTileH - 1) / kMedTileH; ++ty)
        for (int tx = 0; tx < (L.w + kMedTileW - 1) / kMedTileW; ++tx) medt[nmed++] = TileDesc{(uint32_t)c, (uint16_t)tx, (uint16_t)ty};
      for (int ty = 0; ty < (L.h + kShpTileH - 1) / kShpTileH; ++ty)
        for (int tx = 0; tx < d.wpr; ++tx) shpt[nshp++] = TileDesc{(uint32_t)c, (uint16_t)tx, (uint16_t)ty};
      s.max_w = std::max(s.max_w, L.w);
      s.max_h = std::max(s.max_h, L.h);
      const RenderGeom g = make_render_geom(L.w, L.h, L.sx, L.sy, cw, ch);
      auto base_rd = [&](RenderKind kind) {
        RenderDesc r;
        std::memset(&r, 0, sizeof(r));
        r.kind = kind;
        r.type = L.type;
        r.stored_bits = L.stored_bits;
        r.fill = fill;
        r.border_value = bval;
        r.filter = (uint8_t)(cfg.render.filter == kFilterNearest ? 1 : 0);
        r.slice = (uint32_t)c;
        r.src_w = (uint16_t)L.w;
        r.src_h = (uint16_t)L.h;
        r.wpr = d.wpr;
        r.ox = g.ox;
        r.oy = g.oy;
        r.invx = g.invx;
        r.invy = g.invy;
        r.slope = L.slope;
        r.intercept = L.intercept;
        return r;
      };
      auto labels = [&](Plane lab, Plane brd) {
        RenderDesc r = base_rd(kRenderLabels);
        r.src_off = (uint32_t)(lab * s.plane_words + d.mask_off);
        r.border_off = (uint32_t)(brd * s.plane_words + d.mask_off);
        return r;
      };
      RenderDesc orig = base_rd(kRenderRawGray);
      orig.src_off = raw_off;
      if (mode == 0) {
        rd[ncanv++] = orig;
        rd[ncanv++] = labels(kPDilated, kPBorderD);
      } else {
        rd[ncanv++] = orig;
        RenderDesc pre = base_rd(kRenderF32Gray);
        pre.src_off = d.f32_off;
        rd[ncanv++] = pre;
        rd[ncanv++] = labels(kPRegion, kPBorderR);
        rd[ncanv++] = labels(kPEroded, kPBorderE);
        rd[ncanv++] = labels(kPDilated, kPBorderD);
      }
    }
    for (int k = 0; k < ncanv; ++k) {
      rd[k].canvas_off = (uint32_t)k * canvas_bytes;
      JpegDesc& j = jd[k];
      std::memset(&j, 0, sizeof(j));
      j.canvas_off = (uint32_t)k * canvas_bytes;
      j.out_off = (uint64_t)k * out_cap_;
      j.out_cap = out_cap_;
      // Export runs render straight into the JPEG block kernel when the fit is an exact 2× (the
      // canvas is never materialised; bilinear and nearest gray renders alike); test runs keep
      // canvases for inspection.
      j.render = (mode == 0 && render_is_exact_2x(rd[k], cw, ch) &&
                  (rd[k].kind == kRenderLabels || !rd[k].filter || jpeg_fuses_nearest(cfg.render.jpeg_sampling)))
                     ? k
                     : -1;
      if (j.render < 0) s.any_canvas = true;
    }
    s.ncanvas = ncanv;
    if (nl == 0) return;
    if (host_only_) {
      // The GPU stages' host-visible result: each canvas's segment lands in h_out (the encoder
      // stores over PCIe, so the writers read it from DRAM, not from their caches).
      if (mode != 0) throw DeviceError("host-only engine: export runs only");
      for (int k = 0; k < ncanv; ++k) {
        const auto& t = tmpl_[k & 1];
        dicom::stream_copy_unfenced(s.h_out + (size_t)k * out_cap_, t.data(), t.size());
        s.h_sizes[k] = (int32_t)t.size();
      }
      dicom::stream_copy(s.h_out, tmpl_[0].data(), 0);  // fence
      return;
    }

    uint8_t* db = s.d_blob;
    const auto* d_stats_c = reinterpret_cast<SliceStats*>(db + s.off_stats);
    auto* d_stats = reinterpret_cast<SliceStats*>(db + s.off_stats);
    auto* d_desc = reinterpret_cast<SliceDesc*>(db + s.off_desc);
    auto* d_medt = reinterpret_cast<TileDesc*>(db + s.off_medt);
    auto* d_shpt = reinterpret_cast<TileDesc*>(db + s.off_shpt);
    auto* d_seeds = reinterpret_cast<SeedXY*>(db + s.off_seeds);
    auto* d_rd = reinterpret_cast<RenderDesc*>(db + s.off_render);
    auto* d_jd = reinterpret_cast<JpegDesc*>(db + s.off_jpeg);
    auto* d_raw = s.d_raw_x;
    auto plane = [&](Plane p) { return s.d_bits + p * s.plane_words; };

    const double t_enq = now_s();
    // Tables, then the raw pixels not already queued by upload_progress (all of them without it).
    // The tables sit right before the raw region: with nothing uploaded early (a small batch) both
    // go as one copy — one SDMA command and one completion on the batch's critical path, not two.
    const size_t raw_end = s.raw_used();
    // A small batch (≤ 16 slices) with nothing uploaded early copies on its own stream, without the
    // upload stream's events: on the shared stream every copy sat ≈ 20 µs behind the previous one
    // (SDMA → event marker → SDMA hand-offs) and its first kernel ≈ 16–20 µs behind the copy (the
    // cross-stream wait). 58-slice single pass 0.373–0.399 vs 0.435–0.447 ms median over 200 passes
    // in 3 of 3 rounds (profiles/r3/small_upload/). A shader copy from host-mapped memory instead of
    // SDMA measured no gain (profiles/r3/shader_upload/) and was removed in round 4.
    const bool inline_up = s.uploaded == 0 && !s.upload_started && nl <= 16;
    hipStream_t up = inline_up ? s.stream : s.up;
    if (!s.upload_started && !inline_up) check_hip(hipEventRecord(s.ev0, up), "event");
    if (s.uploaded == 0) {
      check_hip(hipMemcpyAsync(s.d_blob, s.h_blob, s.raw_base + raw_end * 2, hipMemcpyHostToDevice, up),
                "H2D tables + pixels");
    } else {
      check_hip(hipMemcpyAsync(s.d_blob, s.h_blob, s.raw_base, hipMemcpyHostToDevice, up), "H2D tables");
      if (raw_end > s.uploaded)
        check_hip(hipMemcpyAsync(s.d_blob + s.raw_base + s.uploaded * 2, s.h_blob + s.raw_base + s.uploaded * 2,
                                 (raw_end - s.uploaded) * 2, hipMemcpyHostToDevice, up),
                  "H2D pixels");
    }
    s.uploaded = raw_end;
    // ev1: the kernels' wait on a separate upload stream, and the h2d/kernel time split.
    if (!inline_up) check_hip(hipEventRecord(s.ev1, up), "event");
    if (up != s.stream) check_hip(hipStreamWaitEvent(s.stream, s.ev1, 0), "wait upload");
    // The median reads the upload directly (12-bit pairs decoded in its tile load) and writes the
    // expanded samples for the render/JPEG stages. One eager launch per kernel: hipGraph replay of
    // this 5-launch chain cost more host CPU than it saved (85k vs 110k slices/s in round 1; 283–346k
    // eager vs 220–321k replayed in round 2, profiles/r2/graphs_threads/), removed in round 4.
    const auto* blob_raw = reinterpret_cast<const uint16_t*>(db + s.raw_base);
    launch_median(nullptr, s.d_med, d_desc, d_medt, nmed, pc.median_k, d_stats, s.stream, s.d_tile_mm, blob_raw, d_raw);
    launch_sharpen_band(s.d_med, plane(kPBand), mode == 1 ? s.d_f32 : nullptr, d_desc, d_shpt, nshp, pc, d_stats,
                        s.stream, s.d_tile_mm, d_lut_);
    SrgOutputs o;
    o.scratch = s.d_srg_scratch;
    o.dilated = plane(kPDilated);
    o.border_dilated = plane(kPBorderD);
    if (mode == 1) {
      o.region = plane(kPRegion);
      o.eroded = plane(kPEroded);
      o.border_region = plane(kPBorderR);
      o.border_eroded = plane(kPBorderE);
    }
    launch_srg_morph(plane(kPBand), d_desc, nl, d_seeds, pc, o, s.max_w, s.max_h, s.stream);
    if (s.any_canvas) launch_render(d_raw, s.d_f32, s.d_bits, d_stats, d_rd, ncanv, cw, ch, s.d_canvas, s.stream);
    JpegRenderSrc rsrc;
    rsrc.raw = d_raw;
    rsrc.f32 = s.d_f32;
    rsrc.bits = s.d_bits;
    rsrc.stats = d_stats;
    rsrc.rd = d_rd;
    rsrc.nrd = ncanv;
    launch_jpeg(s.d_canvas, d_jd, ncanv, cw, ch, divs, s.jw, s.d_out, s.d_sizes, s.stream, &rsrc,
                cfg.render.jpeg_sampling, cfg.render.filter == kFilterNearest && jpeg_fuses_nearest(cfg.render.jpeg_sampling));
    check_hip(hipEventRecord(s.ev2, s.stream), "event");
    if (mark) mark->enq = now_s();
    wait_batch(s, s.ev2, t_enq, nl);
    if (acc && !inline_up) {  // an inline small upload records no split events
      float a = 0, b = 0;
      (void)hipEventElapsedTime(&a, s.ev0, s.ev1);
      (void)hipEventElapsedTime(&b, s.ev1, s.ev2);
      acc->h2d_s += a * 1e-3;
      acc->kernels_s += b * 1e-3;
    }
  }

  // Host bytes of canvas k's GPU-encoded segment (valid when h_sizes[k] ≥ 0).
  const uint8_t* jpeg_bytes(const Slot& s, int k) const {
    return s.h_out + (size_t)k * out_cap_;
  }

  // Bytes of canvas k's JPEG (header + segment + EOI); falls back to the CPU encoder when the
  // GPU reported a capacity overflow (-1).
  bool jpeg_segment(Slot& s, int k, std::vector<uint8_t>& fallback, int64_t* fallbacks) {
    if (s.h_sizes[k] >= 0) return true;
    const int cw = cfg.render.out_width, ch = cfg.render.out_height;
    if (!s.any_canvas) {
      // Fused batches never materialised canvases: render them now (rare overflow path).
      uint8_t* db = s.d_blob;
      launch_render(s.d_raw_x, s.d_f32, s.d_bits,
                    reinterpret_cast<SliceStats*>(db + s.off_stats), reinterpret_cast<RenderDesc*>(db + s.off_render),
                    s.ncanvas, cw, ch, s.d_canvas, s.stream);
      check_hip(hipStreamSynchronize(s.stream), "fallback render");
      s.any_canvas = true;
    }
    std::vector<uint8_t> canvas((size_t)cw * ch);
    check_hip(hipMemcpy(canvas.data(), s.d_canvas + (size_t)k * cw * ch, canvas.size(), hipMemcpyDeviceToHost),
              "canvas D2H");
    jpeg::Tables t = jpeg::make_tables(cfg.render.jpeg_quality);
    fallback = jpeg::encode_scan_gray(canvas.data(), cw, ch, cw, t, (jpeg::Sampling)cfg.render.jpeg_sampling);
    if (fallbacks) ++*fallbacks;
    return false;
  }

  // A slot thread waiting for a small batch's loads or exports spins up to 200 µs before sleeping:
  // such batches are latency-bound (a strong-scaling shard cut into ⌈shard / streams⌉ batches), and
  // the wake-up is on their critical path. Full batches sleep at once (the spin would take CPU the
  // pool needs: 96-slice batches measured 374–388k with it vs 379–401k without, profiles/r3/wait_spin/).
  static int small_batch_spin(size_t count) { return count <= 16 ? 200 : 0; }
  // `batch`: index within its run (fault injection); `prio`: engine-wide batch sequence number,
  // the host-pool priority (earlier batches first, also across queued runs).
  void process_batch(Slot& s, const std::vector<WorkItem>& items, const IoDirs& dirs, size_t batch, uint64_t prio,
                     size_t first, size_t count, std::vector<SliceStatus>& status, StageTimes& acc,
                     std::mutex& acc_m, const std::function<void(size_t)>& on_start, BatchMark* mark = nullptr) {
    if (mark) mark->claim = now_s();
    s.loaded.assign(count, LoadedSlice{});
    if (!s.allocs) {
      s.max_allocs = 2 * (size_t)s.cap_slices;  // ≤ 2 per slice (a hole)
      s.allocs.reset(new Slot::Alloc[s.max_allocs]);
    }
    for (size_t k = 0; k < s.max_allocs; ++k) s.allocs[k].done.store(false, std::memory_order_relaxed);
    s.alloc_word.store(0, std::memory_order_relaxed);
    s.hole_credit.store(s.hole_slack, std::memory_order_relaxed);
    s.uploaded = 0;
    s.upload_started = false;
    s.loads_finished.store(0, std::memory_order_relaxed);
    s.wake_at.store(0, std::memory_order_relaxed);
    s.progress_quiet.store(false, std::memory_order_relaxed);
    std::atomic<int64_t> load_ns{0}, bytes_in{0}, write_ns{0}, bytes_out{0}, load_cpu_ns{0}, write_cpu_ns{0};
    std::string upload_error;
    {
      TaskGroup tg(*pool);
      tg.for_each(
          count,
          [&](size_t i) {
            if (on_start) on_start(first + i);
            if (cfg.resume && outputs_exist(items[first + i])) {
              status[first + i] = SliceStatus{kSliceOk, "resumed: outputs already present"};
            } else {
              load_into(s, (int)i, first + i, items[first + i].path, status[first + i], load_ns, bytes_in);
            }
            if (upload_chunk_) {
              const size_t lf = s.loads_finished.fetch_add(1, std::memory_order_seq_cst) + 1;
              // The load that reaches the slot thread's wake_at (the next upload chunk's worth; and
              // the last load) wakes it: an upload chunk is ≥ 2 MiB (≥ 20 slices of 256²), so finer
              // wake-ups only cost context switches on the CPUs the loaders run on. The lock is taken
              // only when the slot thread sleeps (or is about to: it then re-checks the count under
              // the lock this waits for).
              if (!s.progress_quiet.load(std::memory_order_relaxed) &&
                  (lf >= s.wake_at.load(std::memory_order_seq_cst) || lf == count) &&
                  s.prog_waiting.load(std::memory_order_seq_cst)) {
                { std::lock_guard<std::mutex> g(s.prog_m); }
                s.prog_cv.notify_one();
              }
            }
          },
          2 * prio, &load_cpu_ns);
      if (upload_chunk_) {
        // A failed early upload fails the batch like any device error (below), not the run; the
        // loads still finish (tg.wait) before the blob is touched again.
        try {
          upload_progress(s, count);
        } catch (const std::exception& e) {
          upload_error = e.what();
        }
      }
      tg.wait(small_batch_spin(count));
    }
    if (mark) mark->loaded = now_s();
    s.live.clear();
    for (size_t i = 0; i < count; ++i)
      if (s.loaded[i].ok) s.live.push_back((int)i);
    // Nothing to run, but early chunks may be in flight: the next batch reuses the pinned blob.
    if (s.live.empty() && s.upload_started) check_hip(hipStreamSynchronize(s.up), "upload drain");
    StageTimes local;
    int64_t fallbacks = 0;
    if (!s.live.empty()) {
      try {
        TraceRange tr("nm03.gpu_batch");
        if (!upload_error.empty()) throw DeviceError(upload_error);
        if (fault_plan().fail_batch == (int64_t)batch)
          throw DeviceError("injected fault: device batch failure");
        build_and_run(s, 0, &local, mark);
        if (mark) mark->gpu = now_s();
      } catch (const std::exception& e) {
        for (int i : s.live) status[first + i] = SliceStatus{kSliceDeviceError, e.what()};
        s.live.clear();
        if (s.upload_started) (void)hipStreamSynchronize(s.up);  // blob is reused next batch
      }
    }
    if (cfg.export_jpeg && !s.live.empty()) {
      // CPU fallbacks (rare) are resolved here, on the slot thread that owns the device context.
      std::vector<std::vector<uint8_t>> fb(s.ncanvas);
      std::vector<char> use_fb(s.ncanvas, 0);
      for (int k = 0; k < s.ncanvas; ++k) {
        try {
          use_fb[k] = !jpeg_segment(s, k, fb[k], &fallbacks);
        } catch (const std::exception& e) {
          const size_t item = first + s.live[k / 2];
          status[item] = SliceStatus{kSliceExportError, e.what()};
        }
      }
      // Export order: round-robin over the batch's output directories, so the pool's concurrent
      // writers spread over several patient directories. Creating a file takes its directory's
      // lock exclusively; in slice order every writer would create in the same directory.
      // Wipe-each-pass figure 145–176k vs 128–139k slices/s (4/4 interleaved pairs,
      // profiles/r2/export_interleave/); headline unchanged.
      std::vector<int> order(s.live.size());
      if (dirs.ndirs > 1) {
        std::vector<std::pair<int32_t, std::vector<int>>> groups;  // (dir, live indices), first-seen order
        for (size_t c = 0; c < s.live.size(); ++c) {
          const int32_t d = dirs.out_dir[first + s.live[c]];
          auto it = std::find_if(groups.rbegin(), groups.rend(), [&](const auto& g) { return g.first == d; });
          if (it == groups.rend()) {
            groups.push_back({d, {}});
            it = groups.rbegin();
          }
          it->second.push_back((int)c);
        }
        size_t o = 0;
        for (size_t r = 0; o < order.size(); ++r)
          for (auto& g : groups)
            if (r < g.second.size()) order[o++] = g.second[r];
      } else {
        for (size_t c = 0; c < order.size(); ++c) order[c] = (int)c;
      }
      // Are the batch's output directories being filled? (cold run: every file is created.) A
      // directory whose state is still unknown is probed once per run with its first file.
      bool creates = false;
      for (int c : s.live) {
        const size_t item = first + (size_t)c;
        std::atomic<uint8_t>& st = dirs.creating[dirs.out_dir[item]];
        uint8_t v = st.load(std::memory_order_relaxed);
        if (v == 0) {
          const std::string f = cohort::with_slash(items[item].out_dir) + cohort::stem(items[item].path) + "_original.jpg";
          const uint8_t probe = ::access(f.c_str(), F_OK) == 0 ? 2 : (errno == ENOENT ? 1 : 2);
          st.compare_exchange_strong(v, probe, std::memory_order_relaxed);
          v = st.load(std::memory_order_relaxed);
        }
        creates = creates || v == 1;
      }
      TaskGroup tg(*pool);
      tg.for_each(
          s.live.size(),
          [&](size_t oc) {
            const size_t c = (size_t)order[oc];
            const size_t item = first + s.live[c];
            if (status[item].code != kSliceOk) return;
            const double t0 = now_s();
            TraceRange tr("nm03.export");
            try {
              if (fault_plan().fail_write == (int64_t)item) throw std::runtime_error("injected fault: export failure");
              const std::string base = cohort::with_slash(items[item].out_dir) + cohort::stem(items[item].path);
              for (int k = 0; k < 2; ++k) {
                const int cv = 2 * (int)c + k;
                const std::string name = base + (k == 0 ? "_original.jpg" : "_processed.jpg");
                const uint8_t* seg = use_fb[cv] ? fb[cv].data() : jpeg_bytes(s, cv);
                const size_t len = use_fb[cv] ? fb[cv].size() : (size_t)s.h_sizes[cv];
                jpeg::write_jpeg_at(AT_FDCWD, std::string(), name, jpeg_header, seg, len,
                                    &dirs.creating[dirs.out_dir[item]]);
                bytes_out += (int64_t)(jpeg_header.size() + len + 2);
              }
            } catch (const std::exception& e) {
              status[item] = SliceStatus{kSliceExportError, std::string("Error in export stage: ") + e.what()};
            }
            write_ns += (int64_t)((now_s() - t0) * 1e9);
          },
          2 * prio + 1, &write_cpu_ns, creates ? cfg.create_writers : 0);
      tg.wait(small_batch_spin(count));
    }
    if (mark) mark->end = now_s();
    std::lock_guard<std::mutex> g(acc_m);
    acc.load_s += load_ns.load() * 1e-9;
    acc.write_s += write_ns.load() * 1e-9;
    acc.load_cpu_s += load_cpu_ns.load() * 1e-9;
    acc.write_cpu_s += write_cpu_ns.load() * 1e-9;
    acc.h2d_s += local.h2d_s;
    acc.kernels_s += local.kernels_s;
    acc.bytes_in += bytes_in.load();
    acc.bytes_out += bytes_out.load();
    acc.jpeg_fallbacks += fallbacks;
    acc.batches += 1;
  }

  // Batch schedule: the fewest batches of at most B slices (⌈n / B⌉), of equal size (±1), larger
  // ones first. Round 6: a strong-scaling shard of 116 slices ran as 96 + 20 — the short batch paid
  // a whole batch's fixed costs for a fifth of the work — and measured 315k vs 350k slices/s per GPU
  // at the driver's 20 steps as 58 + 58 (233 slices: 96 + 96 + 41 → 78 + 78 + 77, 362k vs 373k;
  // profiles/r6/even_batches/). Measured and removed in round 4: a tapered schedule (small first /
  // last batches: 209k vs 220k slices/s) and a spread schedule that split short lists over all the
  // slots (more, smaller batches: slower on the headline, config 2 and strong-scaling shards,
  // profiles/r2/spread/).
  static std::vector<std::pair<size_t, size_t>> plan_batches(size_t n, size_t B) {
    std::vector<std::pair<size_t, size_t>> out;
    if (n == 0 || B == 0) return out;
    const size_t k = (n + B - 1) / B, q = n / k, rem = n % k;
    size_t first = 0;
    for (size_t b = 0; b < k; ++b) {
      const size_t len = q + (b < rem ? 1 : 0);
      out.push_back({first, len});
      first += len;
    }
    return out;
  }

  // ---- persistent slot workers: one host thread per slot --------------------------------------
  // Runs are queued (submit): a slot that finishes a batch takes the next unclaimed batch of the
  // oldest queued run, so consecutive runs pipeline — the slots of run k+1 load, upload and compute
  // while run k's last batches drain — instead of every run paying the ring's fill and drain.
  struct Job {
    std::shared_ptr<const std::vector<WorkItem>> items;
    std::unique_ptr<IoDirs> dirs;
    std::function<void(size_t)> on_start;
    std::vector<SliceStatus> status;
    StageTimes acc;
    std::mutex acc_m;
    std::vector<std::pair<size_t, size_t>> batches;  // (first, count)
    size_t next = 0;     // next unclaimed batch (guarded by job_m)
    uint64_t seq0 = 0;   // engine-wide sequence number of batch 0
    std::atomic<size_t> remaining{0};
    double t0 = 0;
    bool done = false;   // guarded by job_m
    std::exception_ptr err;
    std::mutex err_m;
    std::vector<BatchMark> marks;  // NM03_BATCH_TRACE: one per batch (each written by its slot only)
  };
  std::vector<std::thread> workers;
  std::mutex job_m, single_m;
  std::condition_variable job_cv, done_cv;
  std::deque<std::shared_ptr<Job>> queue;  // runs with unclaimed batches, oldest first
  std::atomic<size_t> queued_jobs_{0};      // queue.size() for the idle slots' spin (no lock)
  // An idle slot spins up to 500 µs for the next run before sleeping on the job queue: +2.5-3%
  // headline in 6/8 A/B pairs (profiles/r3/slot_spin), single pass unchanged.
  static constexpr int kSlotSpinUs = 500;
  uint64_t seq_next = 0;
  size_t inflight = 0;  // submitted runs not finished yet
  bool quit = false;

  void start_workers() {
    for (size_t i = 0; i < slots.size(); ++i) workers.emplace_back([this, i] { worker(i); });
  }
  void stop_workers() {
    {
      std::unique_lock<std::mutex> g(job_m);
      done_cv.wait(g, [&] { return inflight == 0; });  // queued runs finish first
      quit = true;
    }
    job_cv.notify_all();
    for (auto& t : workers) t.join();
    workers.clear();
  }

  void finish(Job& j) {
    for (const auto& st : j.status) (st.code == kSliceOk ? j.acc.slices_ok : j.acc.slices_failed) += 1;
    j.acc.wall_s = now_s() - j.t0;
    if (j.acc.jpeg_fallbacks) log_warn(std::to_string(j.acc.jpeg_fallbacks) + " JPEG(s) exceeded GPU capacity; CPU-encoded");
    log_info("run: " + std::to_string(j.items->size()) + " slices in " + std::to_string(j.acc.batches) + " batches, " +
             std::to_string(j.acc.wall_s * 1e3) + " ms, " + std::to_string(j.acc.slices_failed) + " failed");
    if (!j.marks.empty()) {
      std::string t = "batch trace (ms since submit: claim / loaded / enqueued / gpu done / end):";
      auto ms = [&](double v) { return v > 0 ? std::to_string((int)((v - j.t0) * 1e4) / 10.0).substr(0, 6) : std::string("-"); };
      for (const BatchMark& m : j.marks)
        t += "\n  slot " + std::to_string(m.slot) + " [" + std::to_string(m.first) + "+" + std::to_string(m.count) + "] " +
             ms(m.claim) + " / " + ms(m.loaded) + " / " + ms(m.enq) + " / " + ms(m.gpu) + " / " + ms(m.end);
      log_msg(LogLevel::kError, t);  // printed whenever the trace was asked for
    }
    {
      std::lock_guard<std::mutex> g(job_m);
      j.done = true;
      --inflight;
    }
    done_cv.notify_all();
  }

  // Slots still being built by their own threads (quiesce waits for 0).
  std::mutex build_m_;
  std::condition_variable build_cv_;
  int building_ = 0;
  void quiesce() {
    std::unique_lock<std::mutex> g(build_m_);
    build_cv_.wait(g, [&] { return building_ <= 0; });
  }

  void worker(size_t slot_index) {
    pthread_setname_np(pthread_self(), "nm03-slot");
    place.bind_this_thread();
    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // 1 µs: short poll sleeps stay short
    if (!host_only_) (void)hipSetDevice(cfg.device);
    if (!slots[slot_index] && !cfg.lazy_slots) return;  // could not be built in the constructor
    if (!slots[slot_index]) {  // built lazily (see the constructor); this thread is its only user
      bool ok = true;
      try {
        const double tb = now_s();
        std::string split;
        slots[slot_index] = make_slot(batch_trace() ? &split : nullptr);
        if (batch_trace())
          log_msg(LogLevel::kError, "slot " + std::to_string(slot_index) + " built on its worker: " +
                                        std::to_string((now_s() - tb) * 1e3) + " ms (" + split + ")");
      } catch (const std::exception& e) {
        log_warn("engine slot " + std::to_string(slot_index) + " unavailable, running with fewer streams: " + e.what());
        ok = false;
      }
      {
        std::lock_guard<std::mutex> g(build_m_);
        --building_;
      }
      build_cv_.notify_all();
      if (!ok) return;
    }
    Slot* s = slots[slot_index].get();
    for (;;) {
      std::shared_ptr<Job> j;
      size_t b;
      if (queued_jobs_.load(std::memory_order_acquire) == 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(kSlotSpinUs);
        while (queued_jobs_.load(std::memory_order_acquire) == 0 && std::chrono::steady_clock::now() < until)
          __builtin_ia32_pause();
      }
      {
        std::unique_lock<std::mutex> g(job_m);
        job_cv.wait(g, [&] { return quit || !queue.empty(); });
        if (queue.empty()) return;  // quit
        j = queue.front();
        b = j->next++;
        if (j->next == j->batches.size()) queue.pop_front();
        queued_jobs_.store(queue.size(), std::memory_order_release);
      }
      const int64_t c0 = thread_cpu_ns();
      try {
        const auto [first, count] = j->batches[b];
        BatchMark* mk = j->marks.empty() ? nullptr : &j->marks[b];
        if (mk) {
          mk->slot = (int)slot_index;
          mk->first = first;
          mk->count = count;
        }
        process_batch(*s, *j->items, *j->dirs, b, j->seq0 + b, first, count, j->status, j->acc, j->acc_m,
                      j->on_start, mk);
      } catch (...) {
        std::lock_guard<std::mutex> g(j->err_m);
        if (!j->err) j->err = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> g(j->acc_m);
        j->acc.slot_cpu_s += (thread_cpu_ns() - c0) * 1e-9;
      }
      if (j->remaining.fetch_sub(1) == 1) finish(*j);
    }
  }

  std::shared_ptr<Job> submit(std::shared_ptr<const std::vector<WorkItem>> items, std::function<void(size_t)> on_start,
                              int batch_cap = 0) {
    auto j = std::make_shared<Job>();
    j->t0 = now_s();
    j->items = std::move(items);
    j->dirs = std::make_unique<IoDirs>(*j->items);
    j->on_start = std::move(on_start);
    j->status.resize(j->items->size());
    const size_t B = batch_cap > 0 ? std::min<size_t>((size_t)batch_cap, (size_t)cfg.batch_size) : (size_t)cfg.batch_size;
    j->batches = plan_batches(j->items->size(), B);
    j->remaining = j->batches.size();
    if (batch_trace()) j->marks.resize(j->batches.size());
    {
      std::lock_guard<std::mutex> g(job_m);
      j->seq0 = seq_next;
      seq_next += j->batches.size();
      ++inflight;
      if (!j->batches.empty()) queue.push_back(j);
      queued_jobs_.store(queue.size(), std::memory_order_release);
    }
    if (j->batches.empty())
      finish(*j);
    else
      job_cv.notify_all();
    return j;
  }

  std::vector<SliceStatus> wait(const std::shared_ptr<Job>& j, StageTimes* times) {
    {
      std::unique_lock<std::mutex> g(job_m);
      done_cv.wait(g, [&] { return j->done; });
    }
    if (j->err) std::rethrow_exception(j->err);
    if (times) *times = j->acc;
    return j->status;
  }

  std::vector<SliceStatus> run(const std::vector<WorkItem>& items, StageTimes* times,
                               const std::function<void(size_t)>& on_start, int batch_cap = 0) {
    // Blocking form: the caller's vector outlives the run.
    std::shared_ptr<const std::vector<WorkItem>> view(&items, [](const std::vector<WorkItem>*) {});
    return wait(submit(view, on_start, batch_cap), times);
  }

  SingleResult run_single(const golden::SliceInput& in) {
    std::lock_guard<std::mutex> serial(single_m);
    if (host_only_) throw DeviceError("host-only engine: run_single needs the GPU");
    {
      // Slot 0 is used directly: no queued run may be using it.
      std::unique_lock<std::mutex> g(job_m);
      done_cv.wait(g, [&] { return inflight == 0; });
    }
    check_hip(hipSetDevice(cfg.device), "hipSetDevice");
    Slot& s = *slots[0];
    if (in.w > cfg.max_dim || in.h > cfg.max_dim) throw DeviceError("slice exceeds engine max_dim");
    s.alloc_word.store(align_up((size_t)in.w * in.h, 8), std::memory_order_relaxed);  // one region, no allocation entries
    s.uploaded = 0;
    s.upload_started = false;
    s.loaded.assign(1, LoadedSlice{});
    LoadedSlice& L = s.loaded[0];
    L.ok = true;
    L.w = in.w;
    L.h = in.h;
    L.type = in.type;
    L.stored_bits = (uint8_t)in.stored_bits;
    L.slope = cfg.pipe.apply_rescale ? in.slope : 1.f;
    L.intercept = cfg.pipe.apply_rescale ? in.intercept : 0.f;
    L.sx = in.spacing_x;
    L.sy = in.spacing_y;
    L.blob_off = 0;
    L.packed = false;
    std::memcpy(s.raw_cpu, in.raw.data(), in.raw.size() * sizeof(uint16_t));
    s.live.assign(1, 0);
    build_and_run(s, 1, nullptr);
    SingleResult r;
    r.w = in.w;
    r.h = in.h;
    const size_t npix = (size_t)in.w * in.h;
    const int wpr = (in.w + 63) / 64;
    const size_t pw = (size_t)in.h * wpr;  // words of one plane of this slice
    const int cw = cfg.render.out_width, ch = cfg.render.out_height;
    const size_t cvb = (size_t)cw * ch;
    // Every read-back as an async copy into one pinned area and a single synchronisation (was 14
    // synchronous copies into pageable vectors, each staged by the runtime).
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t o_med = 0, o_f32 = al(npix * 2), o_bits = o_f32 + al(npix * 4),
                 o_cv = o_bits + al(kNumPlanes * pw * 8), need = o_cv + (size_t)s.ncanvas * cvb;
    if (s.single_bytes < need) {
      if (s.h_single) (void)hipHostFree(s.h_single);
      s.h_single = nullptr;
      s.single_bytes = 0;
      check_hip(hipHostMalloc((void**)&s.h_single, need, hipHostMallocDefault), "hipHostMalloc single");
      s.single_bytes = need;
    }
    uint8_t* hs = s.h_single;
    check_hip(hipMemcpyAsync(hs + o_med, s.d_med, npix * 2, hipMemcpyDeviceToHost, s.stream), "D2H median");
    check_hip(hipMemcpyAsync(hs + o_f32, s.d_f32, npix * 4, hipMemcpyDeviceToHost, s.stream), "D2H sharpened");
    for (int p = 0; p < kNumPlanes; ++p)
      check_hip(hipMemcpyAsync(hs + o_bits + (size_t)p * pw * 8, s.d_bits + (size_t)p * s.plane_words, pw * 8,
                               hipMemcpyDeviceToHost, s.stream),
                "D2H plane");
    if (s.ncanvas > 0)
      check_hip(hipMemcpyAsync(hs + o_cv, s.d_canvas, (size_t)s.ncanvas * cvb, hipMemcpyDeviceToHost, s.stream),
                "D2H canvases");
    check_hip(hipStreamSynchronize(s.stream), "single read-back");
    r.median_keys.assign(reinterpret_cast<const uint16_t*>(hs + o_med), reinterpret_cast<const uint16_t*>(hs + o_med) + npix);
    r.sharpened.assign(reinterpret_cast<const float*>(hs + o_f32), reinterpret_cast<const float*>(hs + o_f32) + npix);
    // Bits → bytes eight at a time (x86 little-endian: byte i of the table entry is bit i).
    static const auto expand = [] {
      std::array<uint64_t, 256> t{};
      for (int v = 0; v < 256; ++v)
        for (int i = 0; i < 8; ++i) t[v] |= (uint64_t)((v >> i) & 1) << (8 * i);
      return t;
    }();
    auto unpack = [&](Plane p, std::vector<uint8_t>& dst) {
      const uint64_t* words = reinterpret_cast<const uint64_t*>(hs + o_bits + (size_t)p * pw * 8);
      dst.resize(npix + 8);
      for (int y = 0; y < in.h; ++y) {
        uint8_t* row = dst.data() + (size_t)y * in.w;
        for (int x = 0; x < in.w; x += 8) {
          const uint64_t v = expand[(words[(size_t)y * wpr + x / 64] >> (x % 64)) & 0xFF];
          std::memcpy(row + x, &v, 8);  // the row's last group may spill into the next row: rewritten there
        }
      }
      dst.resize(npix);
    };
    unpack(kPBand, r.band);
    unpack(kPRegion, r.region);
    unpack(kPEroded, r.eroded);
    unpack(kPDilated, r.dilated);
    unpack(kPBorderR, r.border_region);
    unpack(kPBorderE, r.border_eroded);
    unpack(kPBorderD, r.border_dilated);
    for (int k = 0; k < s.ncanvas; ++k) {
      r.canvases.emplace_back(hs + o_cv + (size_t)k * cvb, hs + o_cv + (size_t)(k + 1) * cvb);
      std::vector<uint8_t> fb;
      const bool gpu_ok = jpeg_segment(s, k, fb, nullptr);
      std::vector<uint8_t> f = jpeg_header;
      if (gpu_ok)
        f.insert(f.end(), jpeg_bytes(s, k), jpeg_bytes(s, k) + s.h_sizes[k]);
      else
        f.insert(f.end(), fb.begin(), fb.end());
      f.push_back(0xFF);
      f.push_back(0xD9);
      r.jpegs.push_back(std::move(f));
    }
    return r;
  }
};

Engine::Engine(const EngineConfig& cfg) : impl_(std::make_unique<Impl>(cfg)) {}
void Engine::quiesce() { impl_->quiesce(); }
Engine::~Engine() = default;
std::vector<SliceStatus> Engine::run(const std::vector<WorkItem>& items, StageTimes* times,
                                     const std::function<void(size_t)>& on_start, int batch_cap) {
  return impl_->run(items, times, on_start, batch_cap);
}
struct RunHandle {
  std::shared_ptr<Engine::Impl::Job> job;
};
RunTicket Engine::submit(std::shared_ptr<const std::vector<WorkItem>> items, std::function<void(size_t)> on_start,
                         int batch_cap) {
  return std::make_shared<RunHandle>(RunHandle{impl_->submit(std::move(items), std::move(on_start), batch_cap)});
}
std::vector<SliceStatus> Engine::wait(const RunTicket& t, StageTimes* times) { return impl_->wait(t->job, times); }
SingleResult Engine::run_single(const golden::SliceInput& s) { return impl_->run_single(s); }
const EngineConfig& Engine::config() const { return impl_->cfg; }

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

double reserve_streams(int device, int n) {
  const double t0 = now_s();
  check_hip(hipSetDevice(device), "hipSetDevice");
  for (int i = 0; i < n; ++i) {
    hipStream_t s = nullptr;
    check_hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate (reserve)");
    // The process's first host→device copy brings up the runtime's copy path (≈ 7.5 ms cold): here,
    // not in the first batch's upload, where it held the slot threads (profiles/r5/cold/). (On a
    // second thread, overlapping the other streams' creation, it saved 2 ms of 45: not kept,
    // profiles/r5/cold/variants_cli_wall.jsonl.)
    if (i == 0) warm_copy_once(device, s);
    std::lock_guard<std::mutex> g(g_reserve_m);
    g_reserved.push_back({device, s});
  }
  return now_s() - t0;
}

}  // namespace nm03
