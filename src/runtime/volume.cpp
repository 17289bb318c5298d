// 3D mode: series → volume → per-slice K1 (median, sharpen, band) → K5 3D SRG → cube dilation →
// per-slice K3/K4 export. See include/nm03/volume.h.
#include "nm03/volume.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <iostream>

#include "nm03/cohort.h"
#include "nm03/dicom.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg.h"
#include "nm03/kernels.h"

namespace nm03 {

using namespace nm03::gpu;

VolumeInput load_volume(const std::vector<std::string>& files) {
  VolumeInput v;
  std::vector<uint8_t> buf;
  for (size_t z = 0; z < files.size(); ++z) {
    const size_t n = dicom::read_file_into(files[z], buf);
    dicom::Header h = dicom::parse(buf.data(), n);
    if (z == 0) {
      v.w = h.cols;
      v.h = h.rows;
      v.type = h.type == kU8 ? kU16 : h.type;
      v.stored_bits = h.type == kU8 ? 8 : h.bits_stored;
      v.slope = h.slope;
      v.intercept = h.intercept;
      v.spacing_x = h.spacing_x;
      v.spacing_y = h.spacing_y;
      v.raw.resize((size_t)v.w * v.h * files.size());
    } else if (h.cols != v.w || h.rows != v.h) {
      throw SliceError("volume slices differ in size: " + files[z]);
    }
    dicom::copy_pixels16(h, buf.data(), n, v.raw.data() + z * (size_t)v.w * v.h);
    ++v.d;
  }
  return v;
}

namespace {

struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  explicit DevBuf(size_t bytes) { check_hip(hipMalloc(&p, std::max<size_t>(bytes, 16)), "hipMalloc volume"); }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  template <class T>
  T* as() const {
    return (T*)p;
  }
};

PipeConsts make_consts(const PipelineParams& p, int border_radius) {
  PipeConsts pc{};
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
  pc.connectivity = 4;
  pc.dilation_size = p.dilation_size;
  pc.erosion_size = p.erosion_size;
  pc.border_radius = border_radius;
  return pc;
}

struct VolumeDevice {
  int w, h, d, wpr;
  size_t words, ps;
  hipStream_t stream = nullptr;
  DevBuf raw, med, band, region, dil, tmp, desc, medt, shpt, stats, seeds, flag;
  uint32_t* h_flag = nullptr;
  uint8_t* h_tables = nullptr;  // pinned staging: descriptors, tile lists, stats (reused per run)
  size_t n_medt, n_shpt;
  VolumeDevice(const VolumeInput& v)
      : w(v.w), h(v.h), d(v.d), wpr((v.w + 63) / 64), words((size_t)v.h * ((v.w + 63) / 64)),
        ps(((size_t)v.w * v.h + 7) / 8 * 8),
        raw(ps * v.d * 2), med(ps * v.d * 2), band(words * v.d * 8), region(words * v.d * 8), dil(words * v.d * 8),
        tmp(words * v.d * 8), desc(sizeof(SliceDesc) * v.d),
        medt(sizeof(TileDesc) * v.d * ((v.w + 63) / 64) * ((v.h + 63) / 64)),
        shpt(sizeof(TileDesc) * v.d * ((v.w + 63) / 64) * ((v.h + kShpTileH - 1) / kShpTileH)), stats(sizeof(SliceStats) * v.d),
        seeds(sizeof(int32_t) * 3 * kMaxSeeds), flag(16),
        n_medt((size_t)v.d * ((v.w + 63) / 64) * ((v.h + 63) / 64)),
        n_shpt((size_t)v.d * ((v.w + 63) / 64) * ((v.h + kShpTileH - 1) / kShpTileH)) {
    check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    check_hip(hipHostMalloc((void**)&h_flag, 16, hipHostMallocDefault), "hipHostMalloc flag");
    check_hip(hipHostMalloc((void**)&h_tables, table_bytes(), hipHostMallocDefault), "hipHostMalloc tables");
  }
  size_t table_bytes() const {
    return sizeof(SliceDesc) * d + sizeof(TileDesc) * (n_medt + n_shpt) + sizeof(SliceStats) * d;
  }
  ~VolumeDevice() {
    if (h_tables) (void)hipHostFree(h_tables);
    if (h_flag) (void)hipHostFree(h_flag);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

}  // namespace

static void volume_preprocess(VolumeDevice& V, const VolumeInput& v, const PipelineParams& p, const PipeConsts& pc) {
  // Tables are written into pinned staging (valid until the next run, which starts after this
  // run's final sync), so the uploads stay asynchronous.
  auto* hdesc = reinterpret_cast<SliceDesc*>(V.h_tables);
  auto* mt = reinterpret_cast<TileDesc*>(hdesc + v.d);
  auto* st = mt + V.n_medt;
  auto* stats = reinterpret_cast<SliceStats*>(st + V.n_shpt);
  size_t nm = 0, ns = 0;
  for (int z = 0; z < v.d; ++z) {
    SliceDesc& s = hdesc[z];
    std::memset(&s, 0, sizeof(s));
    s.raw_off = (uint32_t)(z * V.ps);
    s.mask_off = (uint32_t)(z * V.words);
    s.w = (uint16_t)v.w;
    s.h = (uint16_t)v.h;
    s.wpr = (uint16_t)V.wpr;
    s.type = v.type;
    s.stored_bits = (uint8_t)v.stored_bits;
    s.slope = p.apply_rescale ? v.slope : 1.f;
    s.intercept = p.apply_rescale ? v.intercept : 0.f;
    for (int ty = 0; ty < (v.h + 63) / 64; ++ty)
      for (int tx = 0; tx < (v.w + 63) / 64; ++tx) mt[nm++] = {(uint32_t)z, (uint16_t)tx, (uint16_t)ty};
    for (int ty = 0; ty < (v.h + kShpTileH - 1) / kShpTileH; ++ty)
      for (int tx = 0; tx < V.wpr; ++tx) st[ns++] = {(uint32_t)z, (uint16_t)tx, (uint16_t)ty};
    stats[z] = SliceStats{0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0u};
  }
  const size_t plane = (size_t)v.w * v.h;
  if (V.ps == plane) {  // planes are contiguous on both sides: one copy
    check_hip(hipMemcpyAsync(V.raw.p, v.raw.data(), plane * v.d * 2, hipMemcpyHostToDevice, V.stream), "H2D volume");
  } else {
    for (int z = 0; z < v.d; ++z)
      check_hip(hipMemcpyAsync(V.raw.as<uint16_t>() + z * V.ps, v.raw.data() + z * plane, plane * 2,
                               hipMemcpyHostToDevice, V.stream),
                "H2D volume");
  }
  check_hip(hipMemcpyAsync(V.desc.p, hdesc, sizeof(SliceDesc) * v.d, hipMemcpyHostToDevice, V.stream), "H2D");
  check_hip(hipMemcpyAsync(V.medt.p, mt, sizeof(TileDesc) * nm, hipMemcpyHostToDevice, V.stream), "H2D");
  check_hip(hipMemcpyAsync(V.shpt.p, st, sizeof(TileDesc) * ns, hipMemcpyHostToDevice, V.stream), "H2D");
  check_hip(hipMemcpyAsync(V.stats.p, stats, sizeof(SliceStats) * v.d, hipMemcpyHostToDevice, V.stream), "H2D");
  launch_median(V.raw.as<uint16_t>(), V.med.as<uint16_t>(), V.desc.as<SliceDesc>(), V.medt.as<TileDesc>(), (int)nm,
                pc.median_k, V.stats.as<SliceStats>(), V.stream);
  launch_sharpen_band(V.med.as<uint16_t>(), V.band.as<uint64_t>(), nullptr, V.desc.as<SliceDesc>(),
                      V.shpt.as<TileDesc>(), (int)ns, pc, V.stats.as<SliceStats>(), V.stream);
}

static void volume_segment(VolumeDevice& V, const VolumeInput& v, const VolumeParams& p, int* sweeps) {
  std::vector<int32_t> sx;
  std::vector<Seed> seeds = p.seeds;
  if (seeds.empty()) {
    seeds = reference_seeds(v.w, v.h);
    for (auto& s : seeds) s.z = v.d / 2;
  }
  for (size_t i = 0; i < seeds.size() && i < (size_t)kMaxSeeds; ++i) {
    sx.push_back(seeds[i].x);
    sx.push_back(seeds[i].y);
    sx.push_back(seeds[i].z);
  }
  check_hip(hipMemcpyAsync(V.seeds.p, sx.data(), sx.size() * 4, hipMemcpyHostToDevice, V.stream), "H2D seeds");
  *sweeps = srg_volume(V.band.as<uint64_t>(), V.region.as<uint64_t>(), v.w, v.h, v.d, V.seeds.as<int32_t>(),
                       (int)(sx.size() / 3), p.connectivity == 26 ? 26 : 6, V.flag.as<uint32_t>(), V.h_flag, V.stream);
  dilate_volume(V.region.as<uint64_t>(), V.dil.as<uint64_t>(), V.tmp.as<uint64_t>(), v.w, v.h, v.d, p.dilation_size,
                V.stream);
}

static void unpack_volume(const DevBuf& b, const VolumeDevice& V, std::vector<uint8_t>& out) {
  std::vector<uint64_t> words(V.words * V.d);
  check_hip(hipMemcpy(words.data(), b.p, words.size() * 8, hipMemcpyDeviceToHost), "D2H mask");
  out.assign((size_t)V.w * V.h * V.d, 0);
  for (int z = 0; z < V.d; ++z)
    for (int y = 0; y < V.h; ++y)
      for (int x = 0; x < V.w; ++x)
        out[((size_t)z * V.h + y) * V.w + x] = (words[(size_t)z * V.words + (size_t)y * V.wpr + x / 64] >> (x % 64)) & 1;
}

// Device buffers, stream and events are cached across runs (allocation and stream creation cost
// more than the kernels for a 256³ volume); they are rebuilt only when the volume shape changes.
struct VolumeRunner::Impl {
  int device;
  std::unique_ptr<VolumeDevice> V;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  explicit Impl(int dev) : device(dev) {
    check_hip(hipSetDevice(device), "hipSetDevice");
    check_hip(hipEventCreate(&e0), "event");
    check_hip(hipEventCreate(&e1), "event");
  }
  ~Impl() {
    (void)hipSetDevice(device);
    V.reset();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
  }
};

VolumeRunner::VolumeRunner(int device) : impl_(std::make_unique<Impl>(device)) {}
VolumeRunner::~VolumeRunner() = default;

VolumeResult VolumeRunner::run(const VolumeInput& v, const VolumeParams& p, bool want_masks) {
  if (v.d < 1 || v.w < 1 || v.h < 1) throw SliceError("empty volume");
  Impl& I = *impl_;
  check_hip(hipSetDevice(I.device), "hipSetDevice");
  if (!I.V || I.V->w != v.w || I.V->h != v.h || I.V->d != v.d) {
    I.V.reset();
    I.V = std::make_unique<VolumeDevice>(v);
  }
  VolumeDevice& V = *I.V;
  const PipeConsts pc = make_consts(p.pipe, 2);
  check_hip(hipEventRecord(I.e0, V.stream), "event");
  VolumeResult r;
  r.w = v.w;
  r.h = v.h;
  r.d = v.d;
  volume_preprocess(V, v, p.pipe, pc);
  volume_segment(V, v, p, &r.sweeps);
  check_hip(hipEventRecord(I.e1, V.stream), "event");
  check_hip(hipEventSynchronize(I.e1), "sync");
  float ms = 0;
  (void)hipEventElapsedTime(&ms, I.e0, I.e1);
  r.kernels_s = ms * 1e-3;
  if (want_masks) {
    unpack_volume(V.band, V, r.band);
    unpack_volume(V.region, V, r.region);
    unpack_volume(V.dil, V, r.dilated);
  }
  return r;
}

VolumeResult run_volume(const VolumeInput& v, const VolumeParams& p, int device, bool want_masks) {
  VolumeRunner runner(device);
  return runner.run(v, p, want_masks);
}

namespace app {

int run_volume_cohort(const AppConfig& cfg) {
  // 3D variant of the cohort run: each patient's series becomes one volume; the exported images
  // are the per-slice renders of the original and of the 3D dilated segmentation.
  const std::string base = cohort::cohort_dir(cfg.data_root);
  std::cout << "\n=== Starting 3D Volume Processing for All Patients ===\n" << std::endl;
  std::vector<std::string> pids = cohort::find_patient_dirs(base);
  std::cout << "Found " << pids.size() << " patient directories." << std::endl;
  if (pids.empty()) {
    std::cout << "No patient directories found. Exiting." << std::endl;
    return 0;
  }
  const RenderParams& rp = cfg.engine.render;
  jpeg::Tables t = jpeg::make_tables(rp.jpeg_quality);
  int successful = 0;
  VolumeRunner runner(cfg.engine.device);
  for (const auto& pid : pids) {
    try {
      std::cout << "\n=== Processing Patient: " << pid << " as a 3D volume ===\n" << std::endl;
      const std::string out = cfg.out_dir + "/" + pid;
      cohort::setup_output_dir(out);
      std::cout << "Created output directory: " + out << std::endl;
      cohort::Series s = cohort::list_patient_series(base, pid);
      std::cout << "Using series directory: " << s.series_dir << std::endl;
      std::cout << "Found " << s.files.size() << " DICOM files for patient " << pid << std::endl;
      VolumeInput v = load_volume(s.files);
      VolumeParams vp;
      vp.pipe = cfg.engine.pipe;
      vp.connectivity = cfg.engine.pipe.srg_connectivity == 26 ? 26 : 6;
      vp.dilation_size = cfg.engine.pipe.dilation_size;
      VolumeResult r = runner.run(v, vp, true);
      // Export per slice (golden renderer + encoder on the host; the 3D path is not the headline).
      PipelineParams pp = cfg.engine.pipe;
      for (int z = 0; z < v.d; ++z) {
        golden::SliceInput si;
        si.w = v.w;
        si.h = v.h;
        si.type = v.type;
        si.stored_bits = v.stored_bits;
        si.slope = v.slope;
        si.intercept = v.intercept;
        si.spacing_x = v.spacing_x;
        si.spacing_y = v.spacing_y;
        si.raw.assign(v.raw.begin() + (size_t)z * v.w * v.h, v.raw.begin() + (size_t)(z + 1) * v.w * v.h);
        std::vector<float> val = golden::rescaled(si, pp);
        auto mm = std::minmax_element(val.begin(), val.end());
        const RenderGeom g = make_render_geom(v.w, v.h, v.spacing_x, v.spacing_y, rp.out_width, rp.out_height);
        std::vector<uint8_t> lab(r.dilated.begin() + (size_t)z * v.w * v.h, r.dilated.begin() + (size_t)(z + 1) * v.w * v.h);
        auto c0 = golden::render_gray(val, g, *mm.first, *mm.second);
        auto c1 = golden::render_labels(lab, golden::border(lab, v.w, v.h, rp.border_radius), g,
                                        opacity_u8(rp.label_opacity), opacity_u8(rp.border_opacity));
        const std::string stem = out + "/" + cohort::stem(s.files[z]);
        auto j0 = jpeg::encode_scan_gray420(c0.data(), rp.out_width, rp.out_height, rp.out_width, t);
        auto j1 = jpeg::encode_scan_gray420(c1.data(), rp.out_width, rp.out_height, rp.out_width, t);
        auto hdr = jpeg::make_header(rp.out_width, rp.out_height, t);
        jpeg::write_jpeg_file(stem + "_original.jpg", hdr, j0.data(), j0.size());
        jpeg::write_jpeg_file(stem + "_processed.jpg", hdr, j1.data(), j1.size());
      }
      std::cout << "\nPatient " << pid << " completed. 3D region growing converged in " << r.sweeps
                << " sweeps; GPU time " << r.kernels_s * 1e3 << " ms." << std::endl;
      ++successful;
    } catch (const std::exception& e) {
      std::cerr << "Error processing patient " << pid << ": " << e.what() << std::endl;
    }
  }
  std::cout << "\n=== All Processing Completed ===\n" << std::endl;
  std::cout << "Successfully processed " << successful << "/" << pids.size() << " patients." << std::endl;
  return 0;
}

}  // namespace app
}  // namespace nm03
