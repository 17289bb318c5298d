// 3D mode: series → volume → per-slice K1 (median, sharpen, band) → K5 3D SRG → cube dilation →
// per-slice K3/K4 export. See include/nm03/volume.h.
#include "nm03/volume.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <fstream>
#include <iostream>
#include <sstream>

#include "nm03/cohort.h"
#include "nm03/comm.h"
#include "nm03/golden.h"
#include "nm03/thread_pool.h"
#include "nm03/volume_slabs.h"
#include "nm03/dicom.h"
#include "nm03/gpu_types.h"
#include "nm03/jpeg.h"
#include "nm03/kernels.h"

namespace nm03 {

using namespace nm03::gpu;

// Every frame of every file, stacked in file order: a series of single-frame slices, or a
// multi-frame file (one file = one volume), or a mix of both.
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
      v.raw.reserve((size_t)v.w * v.h * files.size());
    } else if (h.cols != v.w || h.rows != v.h) {
      throw SliceError("volume slices differ in size: " + files[z]);
    }
    const size_t plane = (size_t)v.w * v.h;
    for (int f = 0; f < h.frames; ++f) {
      v.raw.resize(plane * (size_t)(v.d + 1));
      dicom::copy_pixels16(h, buf.data(), n, v.raw.data() + (size_t)v.d * plane, f);
      ++v.d;
    }
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
  pc.se_disc = p.se_shape == kSeDisc ? 1 : 0;
  return pc;
}

struct VolumeDevice {
  int w, h, d, wpr;
  size_t words, ps;
  hipStream_t stream = nullptr;
  DevBuf raw, med, band, region, dil, tmp, desc, medt, shpt, stats, seeds, flag;
  DevBuf srg_scratch, morph_scratch;  // bit planes too large for LDS (a side > 512), else unused
  uint32_t* h_flag = nullptr;         // the region growing's control words (sweep count, error)
  uint8_t* h_tables = nullptr;  // pinned staging: descriptors, tile lists, stats (reused per run)
  size_t n_medt, n_shpt;
  // z-slab decomposition (run_slab): the two neighbour boundary planes, the added-voxel counter
  // and the halo-extended dilation buffers, allocated on first use and kept.
  std::unique_ptr<DevBuf> slab_nb, slab_added, ext, ext_dil, ext_tmp, ext_scr;
  int ext_planes = 0;
  VolumeDevice(const VolumeInput& v)
      : w(v.w), h(v.h), d(v.d), wpr((v.w + 63) / 64), words((size_t)v.h * ((v.w + 63) / 64)),
        ps(((size_t)v.w * v.h + 7) / 8 * 8),
        raw(ps * v.d * 2), med(ps * v.d * 2), band(words * v.d * 8), region(words * v.d * 8), dil(words * v.d * 8),
        tmp(words * v.d * 8), desc(sizeof(SliceDesc) * v.d),
        medt(sizeof(TileDesc) * v.d * ((v.w + 63) / 64) * ((v.h + 63) / 64)),
        shpt(sizeof(TileDesc) * v.d * ((v.w + 63) / 64) * ((v.h + kShpTileH - 1) / kShpTileH)), stats(sizeof(SliceStats) * v.d),
        seeds(sizeof(int32_t) * 3 * kMaxSeeds), flag(sizeof(uint32_t) * kSrg3dCtlWords),
        srg_scratch(8 * srg3d_scratch_words(v.w, v.h, v.d)), morph_scratch(8 * morph3d_scratch_words(v.w, v.h, v.d)),
        n_medt((size_t)v.d * ((v.w + 63) / 64) * ((v.h + 63) / 64)),
        n_shpt((size_t)v.d * ((v.w + 63) / 64) * ((v.h + kShpTileH - 1) / kShpTileH)) {
    check_hip(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "stream");
    check_hip(hipHostMalloc((void**)&h_flag, sizeof(uint32_t) * kSrg3dCtlWords, hipHostMallocDefault),
              "hipHostMalloc flag");
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

// Enqueues seeding, region growing (convergence decided on the device) and the cube dilation; no
// host synchronisation. The sweep count is read from V.h_flag after the caller's sync.
static void volume_segment(VolumeDevice& V, const VolumeInput& v, const VolumeParams& p) {
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
  srg_volume(V.band.as<uint64_t>(), V.region.as<uint64_t>(), v.w, v.h, v.d, V.seeds.as<int32_t>(),
             (int)(sx.size() / 3), p.connectivity == 26 ? 26 : 6, V.flag.as<uint32_t>(), V.h_flag,
             V.srg_scratch.as<uint64_t>(), V.stream);
  dilate_volume(V.region.as<uint64_t>(), V.dil.as<uint64_t>(), V.tmp.as<uint64_t>(), v.w, v.h, v.d, p.dilation_size,
                V.stream, V.morph_scratch.as<uint64_t>(), p.pipe.se_shape == kSeDisc);
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

// GPU export of a processed volume (K3/K4, like the 2D engine): per plane the original (gray render
// of the raw plane, windowed by the median kernel's per-plane stats) and the processed image (the
// 3D dilated mask with its per-plane renderer border), rendered — fused into the encoder for an
// exact 2× fit — and JPEG-encoded in chunks of kExportSlices planes. Images the GPU encoder cannot
// hold (capacity overflow, rare) are re-encoded on the host from their rendered canvas.
constexpr int kExportSlices = 32;
constexpr uint32_t kVolOutCap = 512 * 1024 + 64;  // per image, as the 2D engine

struct ExportBufs {
  int cap = 2 * kExportSlices;  // canvases per launch
  int cw = 0, ch = 0;
  DevBuf bits, canvas, tables, look, ticket, spill;
  JpegWork jw;
  uint8_t* h_tables = nullptr;
  uint8_t* h_out = nullptr;
  uint8_t* d_out = nullptr;
  int32_t* h_sizes = nullptr;
  int32_t* d_sizes = nullptr;
  size_t bits_words = 0;
  ExportBufs(int cw_, int ch_, size_t vol_words)
      : cw(cw_), ch(ch_),
        bits(2 * vol_words * 8),
        canvas((size_t)cw_ * ch_ * 2 * kExportSlices),
        tables(2 * kExportSlices * (sizeof(RenderDesc) + sizeof(JpegDesc)) + 256),
        look(6 * 8 * (size_t)2 * kExportSlices * (((size_t)cw_ * ch_ / 64 + 255) / 256)),
        ticket(4 * 2 * kExportSlices),
        spill(4 * (size_t)2 * kExportSlices * (((size_t)cw_ * ch_ / 64 + 255) / 256) * 256 * 56),
        bits_words(vol_words) {
    const size_t blocks = (size_t)cw * ch / 64;
    jw.look = look.as<uint64_t>();
    jw.look_cap = (size_t)cap * ((blocks + 255) / 256);
    jw.ticket = ticket.as<uint32_t>();
    jw.spill = spill.as<uint32_t>();
    check_hip(hipMemset(jw.ticket, 0, 4 * (size_t)cap), "memset tickets");
    check_hip(hipMemset(jw.look, 0, 6 * jw.look_cap * 8), "memset look-back");
    check_hip(hipHostMalloc((void**)&h_tables, cap * (sizeof(RenderDesc) + sizeof(JpegDesc)) + 256, hipHostMallocDefault),
              "hipHostMalloc export tables");
    check_hip(hipHostMalloc((void**)&h_out, (size_t)kVolOutCap * cap, hipHostMallocMapped), "hipHostMalloc out");
    check_hip(hipHostGetDevicePointer((void**)&d_out, h_out, 0), "device pointer out");
    check_hip(hipHostMalloc((void**)&h_sizes, 4 * (size_t)cap, hipHostMallocMapped), "hipHostMalloc sizes");
    check_hip(hipHostGetDevicePointer((void**)&d_sizes, h_sizes, 0), "device pointer sizes");
  }
  ~ExportBufs() {
    if (h_tables) (void)hipHostFree(h_tables);
    if (h_out) (void)hipHostFree(h_out);
    if (h_sizes) (void)hipHostFree(h_sizes);
  }
};

// Device buffers, stream and events are cached across runs (allocation and stream creation cost
// more than the kernels for a 256³ volume); they are rebuilt only when the volume shape changes.
struct VolumeRunner::Impl {
  int device;
  std::unique_ptr<VolumeDevice> V;
  std::unique_ptr<ExportBufs> X;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  explicit Impl(int dev) : device(dev) {
    check_hip(hipSetDevice(device), "hipSetDevice");
    preload_kernels();  // every code object, before the first launch (kernels.h)
    check_hip(hipEventCreate(&e0), "event");
    check_hip(hipEventCreate(&e1), "event");
  }
  ~Impl() {
    (void)hipSetDevice(device);
    X.reset();
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
    I.X.reset();
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
  volume_segment(V, v, p);
  check_hip(hipEventRecord(I.e1, V.stream), "event");
  check_hip(hipEventSynchronize(I.e1), "sync");
  r.sweeps = srg_volume_result(V.h_flag);
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

namespace {

// GPU backend of the z-slab decomposition: the slab's planes on the device (VolumeDevice); plane
// reads/writes are small synchronous copies (a boundary plane is 8 KiB for 256²).
class GpuSlabGrower final : public SlabGrower {
 public:
  GpuSlabGrower(VolumeDevice& V, int nseeds, int connectivity) : V_(V), nseeds_(nseeds), conn_(connectivity) {}
  int grow(bool first) override {
    srg_volume(V_.band.as<uint64_t>(), V_.region.as<uint64_t>(), V_.w, V_.h, V_.d, V_.seeds.as<int32_t>(),
               first ? nseeds_ : 0, conn_, V_.flag.as<uint32_t>(), V_.h_flag, V_.srg_scratch.as<uint64_t>(), V_.stream,
               first);
    check_hip(hipStreamSynchronize(V_.stream), "slab grow");
    return srg_volume_result(V_.h_flag);
  }
  std::vector<uint64_t> band_plane(int zl) override { return plane(V_.band, zl); }
  std::vector<uint64_t> region_plane(int zl) override { return plane(V_.region, zl); }
  void or_region_plane(int zl, const std::vector<uint64_t>& bits) override {
    std::vector<uint64_t> cur = plane(V_.region, zl);
    for (size_t i = 0; i < cur.size(); ++i) cur[i] |= bits[i];
    check_hip(hipMemcpy(V_.region.as<uint64_t>() + (size_t)zl * V_.words, cur.data(), V_.words * 8,
                        hipMemcpyHostToDevice),
              "H2D slab plane");
  }
  void dilate(int size, const std::vector<std::vector<uint64_t>>& below,
              const std::vector<std::vector<uint64_t>>& above) override {
    const int nb = (int)below.size(), na = (int)above.size(), de = nb + V_.d + na;
    const size_t wds = V_.words;
    DevBuf ext(wds * de * 8), dil(wds * de * 8), tmp(wds * de * 8), scr(8 * morph3d_scratch_words(V_.w, V_.h, de));
    for (int k = 0; k < nb; ++k)
      check_hip(hipMemcpy(ext.as<uint64_t>() + (size_t)k * wds, below[(size_t)k].data(), wds * 8, hipMemcpyHostToDevice),
                "H2D halo");
    for (int k = 0; k < na; ++k)
      check_hip(hipMemcpy(ext.as<uint64_t>() + (size_t)(nb + V_.d + k) * wds, above[(size_t)k].data(), wds * 8,
                          hipMemcpyHostToDevice),
                "H2D halo");
    check_hip(hipMemcpyAsync(ext.as<uint64_t>() + (size_t)nb * wds, V_.region.p, wds * V_.d * 8, hipMemcpyDeviceToDevice,
                             V_.stream),
              "D2D slab region");
    dilate_volume(ext.as<uint64_t>(), dil.as<uint64_t>(), tmp.as<uint64_t>(), V_.w, V_.h, de, size, V_.stream,
                  scr.as<uint64_t>(), ball);
    check_hip(hipMemcpyAsync(V_.dil.p, dil.as<uint64_t>() + (size_t)nb * wds, wds * V_.d * 8, hipMemcpyDeviceToDevice,
                             V_.stream),
              "D2D slab dilation");
    check_hip(hipStreamSynchronize(V_.stream), "slab dilation");
  }

 private:
  std::vector<uint64_t> plane(const DevBuf& b, int zl) {
    std::vector<uint64_t> v(V_.words);
    check_hip(hipMemcpy(v.data(), b.as<uint64_t>() + (size_t)zl * V_.words, V_.words * 8, hipMemcpyDeviceToHost),
              "D2H slab plane");
    return v;
  }
  VolumeDevice& V_;
  int nseeds_, conn_;
};

}  // namespace

// Device-resident z-slab growth and dilation (volume_slabs.h steps 2 and 3 on the GPU): the slab's
// boundary region planes go from V.region straight into the neighbours' device buffers
// (Comm::sendrecv_device — RCCL over xGMI, or staged through pinned memory by the host comms), the
// boundary seeding is a kernel, and the added-voxel count is all-reduced from device memory: one
// host synchronisation per round, no pageable copies. The dilation halo is received straight into
// the extended buffer around a device copy of the slab. Slabs thinner than the halo fall back to the
// generic algorithm (grow_and_dilate_slabs with GpuSlabGrower).
static SlabStats slab_grow_dilate_gpu(Comm& comm, VolumeDevice& V, int nseeds, int conn, int depth, int z0, int z1,
                                      int dilation, bool ball) {
  const int rank = comm.rank(), n = comm.size();
  const int d = z1 - z0, r = dilation / 2;
  const size_t pw = V.words, pbytes = pw * 8;
  const int below = rank > 0 ? rank - 1 : -1, above = rank + 1 < n ? rank + 1 : -1;
  SlabStats st;
  if (!V.slab_nb) {
    V.slab_nb = std::make_unique<DevBuf>(2 * pbytes);
    V.slab_added = std::make_unique<DevBuf>(8);
  }
  uint64_t* nb_below = V.slab_nb->as<uint64_t>();
  uint64_t* nb_above = nb_below + pw;
  auto* added = V.slab_added->as<int64_t>();
  uint64_t* band = V.band.as<uint64_t>();
  uint64_t* region = V.region.as<uint64_t>();
  for (bool first = true;; first = false) {
    srg_volume(band, region, V.w, V.h, d, V.seeds.as<int32_t>(), first ? nseeds : 0, conn, V.flag.as<uint32_t>(),
               V.h_flag, V.srg_scratch.as<uint64_t>(), V.stream, first);
    // My top plane goes up while the plane below my slab comes up from rank − 1; then the reverse.
    comm.sendrecv_device(region + (size_t)(d - 1) * pw, pbytes, above, nb_below, pbytes, below, V.stream);
    comm.sendrecv_device(region, pbytes, below, nb_above, pbytes, above, V.stream);
    st.exchanged_bytes += (int64_t)((above >= 0) + (below >= 0)) * (int64_t)pbytes;
    check_hip(hipMemsetAsync(added, 0, 8, V.stream), "memset added");
    auto* acc = reinterpret_cast<unsigned long long*>(added);
    if (below >= 0) launch_slab_seed(band, region, nb_below, V.w, V.h, conn == 26, acc, V.stream);
    if (above >= 0)
      launch_slab_seed(band + (size_t)(d - 1) * pw, region + (size_t)(d - 1) * pw, nb_above, V.w, V.h, conn == 26, acc,
                       V.stream);
    const int64_t total = comm.allreduce_sum_i64_device(added, V.stream);  // waits for the round
    st.sweeps += srg_volume_result(V.h_flag);
    ++st.rounds;
    if (total == 0) break;
  }
  const int rb = std::min(r, z0), ra = std::min(r, depth - z1), de = rb + d + ra;
  if (!V.ext || V.ext_planes < de) {
    const size_t bytes = pbytes * (size_t)de;
    V.ext = std::make_unique<DevBuf>(bytes);
    V.ext_dil = std::make_unique<DevBuf>(bytes);
    V.ext_tmp = std::make_unique<DevBuf>(bytes);
    V.ext_scr = std::make_unique<DevBuf>(8 * std::max<size_t>(1, morph3d_scratch_words(V.w, V.h, de)));
    V.ext_planes = de;
  }
  uint64_t* ext = V.ext->as<uint64_t>();
  if (r > 0) {
    // Top r planes up into the successor's lower halo; bottom r planes down into the predecessor's
    // upper halo (every slab holds ≥ r planes here).
    comm.sendrecv_device(region + (size_t)(d - r) * pw, above >= 0 ? (size_t)r * pbytes : 0, above, ext,
                         (size_t)rb * pbytes, below, V.stream);
    comm.sendrecv_device(region, below >= 0 ? (size_t)r * pbytes : 0, below, ext + (size_t)(rb + d) * pw,
                         (size_t)ra * pbytes, above, V.stream);
    st.exchanged_bytes += (int64_t)((above >= 0) + (below >= 0)) * r * (int64_t)pbytes;
  }
  check_hip(hipMemcpyAsync(ext + (size_t)rb * pw, region, pbytes * d, hipMemcpyDeviceToDevice, V.stream), "D2D slab");
  dilate_volume(ext, V.ext_dil->as<uint64_t>(), V.ext_tmp->as<uint64_t>(), V.w, V.h, de, dilation, V.stream,
                V.ext_scr->as<uint64_t>(), ball);
  check_hip(hipMemcpyAsync(V.dil.p, V.ext_dil->as<uint64_t>() + (size_t)rb * pw, pbytes * d, hipMemcpyDeviceToDevice,
                           V.stream),
            "D2D slab dilation");
  return st;
}

VolumeResult VolumeRunner::run_slab(Comm& comm, const VolumeInput& slab, int z0, int depth, const VolumeParams& p,
                                    bool want_masks, SlabStats* stats) {
  if (slab.d < 1 || slab.w < 1 || slab.h < 1) throw SliceError("empty slab");
  Impl& I = *impl_;
  check_hip(hipSetDevice(I.device), "hipSetDevice");
  if (!I.V || I.V->w != slab.w || I.V->h != slab.h || I.V->d != slab.d) {
    I.X.reset();
    I.V.reset();
    I.V = std::make_unique<VolumeDevice>(slab);
  }
  VolumeDevice& V = *I.V;
  const PipeConsts pc = make_consts(p.pipe, 2);
  check_hip(hipEventRecord(I.e0, V.stream), "event");
  volume_preprocess(V, slab, p.pipe, pc);
  // Seeds in volume coordinates → this slab's (the rest belong to other ranks).
  std::vector<int32_t> sx;
  for (const Seed& s : slab_seeds(p.seeds, slab.w, slab.h, depth, z0, slab.d))
    if (sx.size() / 3 < (size_t)kMaxSeeds) {
      sx.push_back(s.x);
      sx.push_back(s.y);
      sx.push_back(s.z);
    }
  if (!sx.empty())
    check_hip(hipMemcpyAsync(V.seeds.p, sx.data(), sx.size() * 4, hipMemcpyHostToDevice, V.stream), "H2D seeds");
  const int conn = p.connectivity == 26 ? 26 : 6;
  if (depth < comm.size())
    throw std::runtime_error("z-slabs: volume depth " + std::to_string(depth) + " < " + std::to_string(comm.size()) +
                             " ranks leaves empty slabs");
  SlabStats st;
  if (depth / comm.size() >= p.dilation_size / 2) {
    st = slab_grow_dilate_gpu(comm, V, (int)(sx.size() / 3), conn, depth, z0, z0 + slab.d, p.dilation_size,
                              p.pipe.se_shape == kSeDisc);
  } else {  // slabs thinner than the dilation halo: the generic exchange (all-gather of slab ends)
    GpuSlabGrower g(V, (int)(sx.size() / 3), conn);
    g.ball = p.pipe.se_shape == kSeDisc;
    st = grow_and_dilate_slabs(comm, g, slab.w, slab.h, depth, z0, z0 + slab.d, conn, p.dilation_size);
  }
  check_hip(hipEventRecord(I.e1, V.stream), "event");
  check_hip(hipEventSynchronize(I.e1), "sync");
  VolumeResult r;
  r.w = slab.w;
  r.h = slab.h;
  r.d = slab.d;
  r.sweeps = st.sweeps;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, I.e0, I.e1);
  r.kernels_s = ms * 1e-3;
  if (stats) *stats = st;
  if (want_masks) {
    unpack_volume(V.band, V, r.band);
    unpack_volume(V.region, V, r.region);
    unpack_volume(V.dil, V, r.dilated);
  }
  return r;
}

std::vector<std::vector<uint8_t>> VolumeRunner::export_jpegs(const VolumeInput& v, const VolumeParams& p,
                                                             const RenderParams& rp, VolumeExportStats* st) {
  Impl& I = *impl_;
  if (!I.V || I.V->w != v.w || I.V->h != v.h || I.V->d != v.d) throw DeviceError("export_jpegs: run() this volume first");
  check_hip(hipSetDevice(I.device), "hipSetDevice");
  VolumeDevice& V = *I.V;
  const int cw = rp.out_width, ch = rp.out_height;
  if (cw % 16 || ch % 16) throw DeviceError("canvas size must be a multiple of 16");
  if (!I.X || I.X->cw != cw || I.X->ch != ch) {
    I.X.reset();
    I.X = std::make_unique<ExportBufs>(cw, ch, V.words * V.d);
  }
  ExportBufs& X = *I.X;
  const double t0 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  // Label planes = the dilated mask, border planes right behind them in one bit buffer.
  uint64_t* bits = X.bits.as<uint64_t>();
  const size_t vol_words = V.words * V.d;
  check_hip(hipMemcpyAsync(bits, V.dil.p, vol_words * 8, hipMemcpyDeviceToDevice, V.stream), "D2D labels");
  border_volume(bits, bits + vol_words, v.w, v.h, v.d, rp.border_radius, V.stream, V.morph_scratch.as<uint64_t>());
  const jpeg::Tables tables = jpeg::make_tables(rp.jpeg_quality);
  const jpeg::Sampling samp = (jpeg::Sampling)rp.jpeg_sampling;
  const std::vector<uint8_t> header = jpeg::make_header(cw, ch, tables, samp);
  const RenderGeom g = make_render_geom(v.w, v.h, v.spacing_x, v.spacing_y, cw, ch);
  const uint8_t fill = opacity_u8(rp.label_opacity), bval = opacity_u8(rp.border_opacity);
  const size_t canvas_bytes = (size_t)cw * ch;
  std::vector<std::vector<uint8_t>> files((size_t)2 * v.d);
  for (int z0 = 0; z0 < v.d; z0 += kExportSlices) {
    const int nz = std::min(kExportSlices, v.d - z0), nc = 2 * nz;
    auto* rd = reinterpret_cast<RenderDesc*>(X.h_tables);
    auto* jd = reinterpret_cast<JpegDesc*>(X.h_tables + (size_t)X.cap * sizeof(RenderDesc));
    bool any_canvas = false;
    for (int k = 0; k < nc; ++k) {
      const int z = z0 + k / 2;
      RenderDesc& r = rd[k];
      std::memset(&r, 0, sizeof(r));
      r.kind = (k & 1) ? kRenderLabels : kRenderRawGray;
      r.filter = (uint8_t)(rp.filter == kFilterNearest ? 1 : 0);
      r.type = (uint8_t)v.type;
      r.stored_bits = (uint8_t)v.stored_bits;
      r.fill = fill;
      r.border_value = bval;
      r.slice = (uint32_t)z;  // the median kernel's per-plane stats
      r.src_w = (uint16_t)v.w;
      r.src_h = (uint16_t)v.h;
      r.wpr = (uint16_t)V.wpr;
      r.ox = g.ox;
      r.oy = g.oy;
      r.invx = g.invx;
      r.invy = g.invy;
      r.slope = p.pipe.apply_rescale ? v.slope : 1.f;
      r.intercept = p.pipe.apply_rescale ? v.intercept : 0.f;
      r.src_off = (k & 1) ? (uint32_t)(z * V.words) : (uint32_t)(z * V.ps);
      r.border_off = (uint32_t)(vol_words + z * V.words);
      r.canvas_off = (uint32_t)(k * canvas_bytes);
      JpegDesc& j = jd[k];
      std::memset(&j, 0, sizeof(j));
      j.canvas_off = (uint32_t)(k * canvas_bytes);
      j.out_off = (uint64_t)k * kVolOutCap;
      j.out_cap = kVolOutCap;
      j.render = render_is_exact_2x(r, cw, ch) && (r.kind == kRenderLabels || !r.filter || jpeg_fuses_nearest(samp)) ? k : -1;
      any_canvas |= j.render < 0;
    }
    auto* d_rd = X.tables.as<uint8_t>();
    auto* d_jd = d_rd + (size_t)X.cap * sizeof(RenderDesc);
    check_hip(hipMemcpyAsync(d_rd, X.h_tables, (size_t)X.cap * (sizeof(RenderDesc) + sizeof(JpegDesc)),
                             hipMemcpyHostToDevice, V.stream),
              "H2D export tables");
    const auto* drd = reinterpret_cast<const RenderDesc*>(d_rd);
    if (any_canvas)
      launch_render(V.raw.as<uint16_t>(), nullptr, bits, V.stats.as<SliceStats>(), drd, nc, cw, ch,
                    X.canvas.as<uint8_t>(), V.stream);
    JpegRenderSrc rs;
    rs.raw = V.raw.as<uint16_t>();
    rs.bits = bits;
    rs.stats = V.stats.as<SliceStats>();
    rs.rd = drd;
    rs.nrd = nc;
    launch_jpeg(X.canvas.as<uint8_t>(), reinterpret_cast<const JpegDesc*>(d_jd), nc, cw, ch, tables.div_luma, X.jw,
                X.d_out, X.d_sizes, V.stream, &rs, samp, rp.filter == kFilterNearest && jpeg_fuses_nearest(samp));
    check_hip(hipStreamSynchronize(V.stream), "export sync");
    bool rendered = any_canvas;
    for (int k = 0; k < nc; ++k) {
      std::vector<uint8_t>& f = files[(size_t)2 * z0 + k];
      f = header;
      if (X.h_sizes[k] >= 0) {
        f.insert(f.end(), X.h_out + (size_t)k * kVolOutCap, X.h_out + (size_t)k * kVolOutCap + X.h_sizes[k]);
      } else {  // capacity overflow: host encoder on the rendered canvas
        if (!rendered) {
          launch_render(V.raw.as<uint16_t>(), nullptr, bits, V.stats.as<SliceStats>(), drd, nc, cw, ch,
                        X.canvas.as<uint8_t>(), V.stream);
          check_hip(hipStreamSynchronize(V.stream), "fallback render");
          rendered = true;
        }
        std::vector<uint8_t> canvas(canvas_bytes);
        check_hip(hipMemcpy(canvas.data(), X.canvas.as<uint8_t>() + (size_t)k * canvas_bytes, canvas_bytes,
                            hipMemcpyDeviceToHost),
                  "canvas D2H");
        const auto scan = jpeg::encode_scan_gray(canvas.data(), cw, ch, cw, tables, samp);
        f.insert(f.end(), scan.begin(), scan.end());
        if (st) ++st->jpeg_fallbacks;
      }
      f.push_back(0xFF);
      f.push_back(0xD9);
    }
  }
  if (st)
    st->export_s += std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() - t0;
  return files;
}

VolumeResult run_volume(const VolumeInput& v, const VolumeParams& p, int device, bool want_masks) {
  VolumeRunner runner(device);
  return runner.run(v, p, want_masks);
}

namespace app {

namespace {

double wall_now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

struct VolPatient {
  std::string id, out_dir, series_dir, error;
  bool setup_ok = false, listed = false;
  std::vector<std::string> files;
};

struct VolOutcome {
  int32_t ok = 0;
  std::string message;
  int32_t sweeps = 0;
  double gpu_s = 0, export_s = 0, wall_s = 0;
  int64_t slices = 0, fallbacks = 0;
  int32_t rounds = 0;         // --split-volume: grow/exchange rounds
  int64_t exchanged = 0;      // --split-volume: boundary + halo bytes sent
};

std::vector<uint8_t> encode(const std::vector<VolPatient>& pl) {
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

std::vector<VolPatient> decode(const std::vector<uint8_t>& b) {
  ByteReader r(b.data(), b.size());
  std::vector<VolPatient> pl(r.u32());
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

void write_file(const std::string& path, const std::vector<uint8_t>& jpg) {
  // complete JPEG file (header + scan + EOI): write_jpeg_file appends the EOI itself
  jpeg::write_jpeg_file(path, {}, jpg.data(), jpg.size() - 2);
}

// Golden 3D path (--cpu): per-plane preprocessing on a thread pool, 3D SRG + cube dilation, host
// render + encoder — the oracle the GPU 3D export is checked against.
struct GoldenPlanes {
  std::vector<uint8_t> band;               // 0/1 voxels of every plane
  std::vector<std::vector<float>> vals;    // rescaled values per plane (original render)
};

GoldenPlanes golden_preprocess(const VolumeInput& v, const VolumeParams& vp) {
  const size_t plane = (size_t)v.w * v.h;
  GoldenPlanes g;
  g.band.assign(plane * v.d, 0);
  g.vals.resize((size_t)v.d);
  ThreadPool pool(16);
  TaskGroup tg(pool);
  for (int z = 0; z < v.d; ++z)
    tg.run([&, z] {
      golden::SliceInput si;
      si.w = v.w;
      si.h = v.h;
      si.type = v.type;
      si.stored_bits = v.stored_bits;
      si.slope = v.slope;
      si.intercept = v.intercept;
      si.spacing_x = v.spacing_x;
      si.spacing_y = v.spacing_y;
      si.raw.assign(v.raw.begin() + z * plane, v.raw.begin() + (z + 1) * plane);
      golden::SliceResult r = golden::run(si, vp.pipe, false);
      std::copy(r.band.begin(), r.band.end(), g.band.begin() + z * plane);
      g.vals[z] = golden::rescaled(si, vp.pipe);
    });
  tg.wait();
  return g;
}

// The 2·d files (original, processed per plane) of the dilated mask `dil` of volume `v`.
std::vector<std::vector<uint8_t>> golden_export(const VolumeInput& v, const std::vector<std::vector<float>>& vals,
                                                const std::vector<uint8_t>& dil, const RenderParams& rp) {
  const size_t plane = (size_t)v.w * v.h;
  const RenderGeom g = make_render_geom(v.w, v.h, v.spacing_x, v.spacing_y, rp.out_width, rp.out_height);
  std::vector<std::vector<uint8_t>> files((size_t)2 * v.d);
  for (int z = 0; z < v.d; ++z) {
    const auto mm = std::minmax_element(vals[z].begin(), vals[z].end());
    std::vector<uint8_t> lab(dil.begin() + z * plane, dil.begin() + (z + 1) * plane);
    const auto c0 = golden::render_gray(vals[z], g, *mm.first, *mm.second, rp.filter == kFilterNearest);
    const auto c1 = golden::render_labels(lab, golden::border(lab, v.w, v.h, rp.border_radius), g,
                                          opacity_u8(rp.label_opacity), opacity_u8(rp.border_opacity));
    files[2 * z] = jpeg::encode_gray(c0.data(), rp.out_width, rp.out_height, rp.out_width, rp.jpeg_quality,
                                     (jpeg::Sampling)rp.jpeg_sampling);
    files[2 * z + 1] = jpeg::encode_gray(c1.data(), rp.out_width, rp.out_height, rp.out_width, rp.jpeg_quality,
                                     (jpeg::Sampling)rp.jpeg_sampling);
  }
  return files;
}

std::vector<std::vector<uint8_t>> golden_volume_jpegs(const VolumeInput& v, const VolumeParams& vp,
                                                      const RenderParams& rp) {
  const GoldenPlanes gp = golden_preprocess(v, vp);
  std::vector<Seed> seeds = vp.seeds;
  if (seeds.empty()) {
    seeds = reference_seeds(v.w, v.h);
    for (auto& sd : seeds) sd.z = v.d / 2;
  }
  const auto region = golden::region_grow3d(gp.band, v.w, v.h, v.d, seeds, vp.connectivity);
  const auto dil = golden::dilate3d(region, v.w, v.h, v.d, vp.dilation_size, vp.pipe.se_shape == kSeDisc);
  return golden_export(v, gp.vals, dil, rp);
}

// One rank's z-slab of a volume on the golden model (--cpu --split-volume): the same
// decomposition and exchanges as the GPU slab path (volume_slabs.h), host arithmetic.
std::vector<std::vector<uint8_t>> golden_slab_jpegs(Comm& comm, const VolumeInput& slab, int z0, int depth,
                                                    const VolumeParams& vp, const RenderParams& rp, SlabStats* st) {
  GoldenPlanes gp = golden_preprocess(slab, vp);
  GoldenSlabGrower g(std::move(gp.band), slab.w, slab.h, slab.d, slab_seeds(vp.seeds, slab.w, slab.h, depth, z0, slab.d),
                     vp.connectivity);
  g.ball = vp.pipe.se_shape == kSeDisc;
  *st = grow_and_dilate_slabs(comm, g, slab.w, slab.h, depth, z0, z0 + slab.d, vp.connectivity, vp.dilation_size);
  return golden_export(slab, gp.vals, g.dilated(), rp);
}

int volume_rank(const AppConfig& cfg, int rank, int size, Comm& comm, int device) {
  const std::string base = cohort::cohort_dir(cfg.data_root);
  VolumeParams vp;
  vp.pipe = cfg.engine.pipe;
  vp.connectivity = cfg.engine.pipe.srg_connectivity == 26 ? 26 : 6;
  // BASELINE config 5: 7×7×7 cube dilation unless --dilation-size was given.
  vp.dilation_size = cfg.dilation_set ? cfg.engine.pipe.dilation_size : 7;
  const RenderParams& rp = cfg.engine.render;
  const double t_start = wall_now();
  // ---- plan on rank 0 -----------------------------------------------------------------------
  std::vector<uint8_t> plan_bytes;
  int64_t fatal = 0;
  std::string fatal_msg;
  if (rank == 0) {
    std::cout << "\n=== Starting 3D Volume Processing for All Patients ===\n" << std::endl;
    try {
      std::vector<VolPatient> plan;
      std::vector<std::string> pids = cohort::find_patient_dirs(base);
      std::cout << "Found " << pids.size() << " patient directories." << std::endl;
      for (const auto& pid : pids) {
        VolPatient p;
        p.id = pid;
        p.out_dir = cfg.out_dir + "/" + pid;
        try {
          cohort::setup_output_dir(p.out_dir);
          p.setup_ok = true;
          cohort::Series s = cohort::list_patient_series(base, pid);
          p.series_dir = s.series_dir;
          p.files = std::move(s.files);
          p.listed = true;
        } catch (const std::exception& e) {
          p.error = e.what();
        }
        plan.push_back(std::move(p));
      }
      plan_bytes = encode(plan);
    } catch (const std::exception& e) {
      fatal = 1;
      fatal_msg = e.what();
    }
  }
  comm.allreduce_sum_i64(&fatal, 1);
  if (fatal) {
    if (rank == 0) std::cerr << "Error finding patient directories: " << fatal_msg << std::endl;
    return 1;
  }
  comm.broadcast_bytes(plan_bytes, 0);
  const std::vector<VolPatient> plan = decode(plan_bytes);
  // ---- this rank's patients (contiguous blocks; one volume per patient) ----------------------
  const size_t lo = plan.size() * rank / size, hi = plan.size() * (rank + 1) / size;
  std::unique_ptr<VolumeRunner> runner;
  std::string setup_error;
  if (!cfg.cpu) {
    try {
      runner = std::make_unique<VolumeRunner>(device);
    } catch (const std::exception& e) {
      setup_error = e.what();
    }
  }
  std::vector<VolOutcome> mine;
  double my_wall = 0;
  auto write_planes = [&](const VolPatient& pp, int z0, int d, const std::vector<std::vector<uint8_t>>& files) {
    for (int z = 0; z < d; ++z) {
      const std::string stem = pp.out_dir + "/" + cohort::stem(pp.files[(size_t)(z0 + z)]);
      write_file(stem + "_original.jpg", files[2 * z]);
      write_file(stem + "_processed.jpg", files[2 * z + 1]);
    }
  };
  if (cfg.split_volume) {
    // Every patient's volume over ALL ranks, one z-slab each (volume_slabs.h). Failures before the
    // collective part are agreed on first; a failure inside it is fatal for the rank, and the
    // launcher's abort flag then ends the others' collectives.
    for (const VolPatient& pp : plan) {
      VolOutcome o;
      const double t0 = wall_now();
      const int depth = (int)pp.files.size();
      int z0 = 0, z1 = 0;
      VolumeInput slab;
      int64_t bad = 0;
      try {
        if (!setup_error.empty()) throw std::runtime_error(setup_error);
        if (!pp.listed) throw std::runtime_error(pp.error);
        if (depth < size)
          throw std::runtime_error("--split-volume: " + std::to_string(depth) + " planes cannot be split over " +
                                   std::to_string(size) + " ranks");
        std::tie(z0, z1) = slab_bounds(depth, rank, size);
        slab = load_volume(std::vector<std::string>(pp.files.begin() + z0, pp.files.begin() + z1));
      } catch (const std::exception& e) {
        o.message = e.what();
        bad = 1;
      }
      // Agree on failures and on the plane shape before any exchange.
      double shape[2] = {bad ? -1.0 : (double)slab.w, bad ? -1.0 : (double)slab.h};
      double nshape[2] = {-shape[0], -shape[1]};
      comm.allreduce_sum_i64(&bad, 1);
      comm.allreduce_max_f64(shape, 2);
      comm.allreduce_max_f64(nshape, 2);
      if (!bad && (shape[0] != -nshape[0] || shape[1] != -nshape[1])) {
        bad = 1;
        o.message = "volume slices differ in size across slabs";
      }
      if (!bad) {
        SlabStats st;
        std::vector<std::vector<uint8_t>> files;
        if (cfg.cpu) {
          files = golden_slab_jpegs(comm, slab, z0, depth, vp, rp, &st);
        } else {
          VolumeResult r = runner->run_slab(comm, slab, z0, depth, vp, false, &st);
          o.gpu_s = r.kernels_s;
          VolumeExportStats xs;
          files = runner->export_jpegs(slab, vp, rp, &xs);
          o.export_s = xs.export_s;
          o.fallbacks = xs.jpeg_fallbacks;
        }
        o.sweeps = st.sweeps;
        o.rounds = st.rounds;
        o.exchanged = st.exchanged_bytes;
        o.slices = slab.d;
        write_planes(pp, z0, slab.d, files);
        o.ok = 1;
      } else if (o.message.empty()) {
        o.message = "failed on another rank";
      }
      o.wall_s = wall_now() - t0;
      my_wall += o.wall_s;
      mine.push_back(std::move(o));
    }
  }
  for (size_t i = lo; i < hi && !cfg.split_volume; ++i) {
    const VolPatient& pp = plan[i];
    VolOutcome o;
    const double t0 = wall_now();
    try {
      if (!setup_error.empty()) throw std::runtime_error(setup_error);
      if (!pp.listed) throw std::runtime_error(pp.error);
      VolumeInput v = load_volume(pp.files);
      o.slices = v.d;
      std::vector<std::vector<uint8_t>> files;
      if (cfg.cpu) {
        files = golden_volume_jpegs(v, vp, rp);
      } else {
        VolumeResult r = runner->run(v, vp, false);
        o.sweeps = r.sweeps;
        o.gpu_s = r.kernels_s;
        VolumeExportStats xs;
        files = runner->export_jpegs(v, vp, rp, &xs);
        o.export_s = xs.export_s;
        o.fallbacks = xs.jpeg_fallbacks;
      }
      write_planes(pp, 0, v.d, files);
      o.ok = 1;
    } catch (const std::exception& e) {
      o.message = e.what();
    }
    o.wall_s = wall_now() - t0;
    my_wall += o.wall_s;
    mine.push_back(std::move(o));
  }
  // ---- gather outcomes, rank 0 prints in patient order ---------------------------------------
  ByteWriter w;
  w.u32((uint32_t)mine.size());
  for (const auto& o : mine) {
    w.i32(o.ok);
    w.str(o.message);
    w.i32(o.sweeps);
    w.f64(o.gpu_s);
    w.f64(o.export_s);
    w.f64(o.wall_s);
    w.u64((uint64_t)o.slices);
    w.u64((uint64_t)o.fallbacks);
    w.i32(o.rounds);
    w.u64((uint64_t)o.exchanged);
  }
  auto all = comm.allgather_bytes(w.b);
  double tot = wall_now() - t_start;
  comm.allreduce_max_f64(&tot, 1);
  std::vector<double> walls((size_t)size);
  comm.allgather(&my_wall, sizeof(double), walls.data());
  if (rank != 0) return 0;
  std::vector<VolOutcome> outs;
  for (auto& b : all) {
    ByteReader r(b.data(), b.size());
    const uint32_t k = r.u32();
    for (uint32_t i = 0; i < k; ++i) {
      VolOutcome o;
      o.ok = r.i32();
      o.message = r.str();
      o.sweeps = r.i32();
      o.gpu_s = r.f64();
      o.export_s = r.f64();
      o.wall_s = r.f64();
      o.slices = (int64_t)r.u64();
      o.fallbacks = (int64_t)r.u64();
      o.rounds = r.i32();
      o.exchanged = (int64_t)r.u64();
      outs.push_back(std::move(o));
    }
  }
  if (cfg.split_volume) {
    // Rank-major per-patient outcomes → one per patient: ok if every slab was, the first failure's
    // message, the slowest slab's times, the sum of planes and exchanged bytes.
    std::vector<VolOutcome> merged(plan.size());
    for (size_t i = 0; i < plan.size(); ++i) {
      VolOutcome& m = merged[i];
      m.ok = 1;
      for (int q = 0; q < size; ++q) {
        const VolOutcome& o = outs[(size_t)q * plan.size() + i];
        if (!o.ok) {
          if (m.ok || m.message == "failed on another rank") m.message = o.message;
          m.ok = 0;
        }
        m.sweeps = std::max(m.sweeps, o.sweeps);
        m.rounds = std::max(m.rounds, o.rounds);
        m.gpu_s = std::max(m.gpu_s, o.gpu_s);
        m.export_s = std::max(m.export_s, o.export_s);
        m.wall_s = std::max(m.wall_s, o.wall_s);
        m.slices += o.slices;
        m.fallbacks += o.fallbacks;
        m.exchanged += o.exchanged;
      }
    }
    outs = std::move(merged);
  }
  int successful = 0;
  int64_t slices = 0, fallbacks = 0;
  std::ostringstream pj;
  for (size_t i = 0; i < plan.size(); ++i) {
    const VolPatient& pp = plan[i];
    const VolOutcome& o = outs[i];
    std::cout << "\n=== Processing Patient: " << pp.id << " as a 3D volume ===\n" << std::endl;
    if (pp.setup_ok) std::cout << "Created output directory: " + pp.out_dir << std::endl;
    if (pp.listed) {
      std::cout << "Using series directory: " << pp.series_dir << std::endl;
      std::cout << "Found " << pp.files.size() << " DICOM files for patient " << pp.id << std::endl;
    }
    if (o.ok) {
      ++successful;
      slices += o.slices;
      fallbacks += o.fallbacks;
      if (cfg.cpu)
        std::cout << "\nPatient " << pp.id << " completed on the CPU golden model." << std::endl;
      else
        std::cout << "\nPatient " << pp.id << " completed. 3D region growing converged in " << o.sweeps
                  << " sweeps; GPU time " << o.gpu_s * 1e3 << " ms." << std::endl;
      if (cfg.split_volume)
        std::cout << "Split over " << size << " ranks: " << o.rounds << " exchange rounds, " << o.exchanged
                  << " bytes exchanged." << std::endl;
    } else {
      std::cerr << "Error processing patient " << pp.id << ": " << o.message << std::endl;
    }
    pj << (i ? ", " : "") << "{\"id\": \"" << pp.id << "\", \"ok\": " << (o.ok ? "true" : "false")
       << ", \"slices\": " << o.slices << ", \"sweeps\": " << o.sweeps << ", \"gpu_s\": " << o.gpu_s
       << ", \"export_s\": " << o.export_s << ", \"wall_s\": " << o.wall_s << ", \"rounds\": " << o.rounds
       << ", \"exchanged_bytes\": " << o.exchanged << "}";
  }
  std::cout << "\n=== All Processing Completed ===\n" << std::endl;
  std::cout << "Successfully processed " << successful << "/" << plan.size() << " patients." << std::endl;
  if (!cfg.json.empty()) {
    std::ofstream f(cfg.json, std::ios::trunc);
    f << "{\"mode\": \"3d\", \"backend\": \"" << (cfg.cpu ? "cpu" : "gpu") << "\", \"gpus\": " << size
      << ", \"comm\": \"" << comm.backend() << "\", \"dilation_size\": " << vp.dilation_size
      << ", \"connectivity\": " << vp.connectivity << ", \"split_volume\": " << (cfg.split_volume ? "true" : "false")
      << ", \"wall_s\": " << tot << ", \"slices\": " << slices
      << ", \"jpeg_fallbacks\": " << fallbacks << ", \"per_rank_wall_s\": [";
    for (int r = 0; r < size; ++r) f << (r ? ", " : "") << walls[r];
    f << "], \"patients\": [" << pj.str() << "]}\n";
  }
  return 0;
}

}  // namespace

int run_volume_cohort(const AppConfig& cfg) {
  // 3D variant of the cohort run (BASELINE config 5): each patient's series becomes one volume
  // (3D SRG + cube dilation on the GPU), exported per plane like the 2D run; patients are sharded
  // over the ranks (one process per MI355X) like the 2D work list.
  LaunchOptions lo = LaunchOptions::from_env();
  int n = 1;
  if (cfg.cpu) {  // golden model: the ranks are CPU processes over the host comm (default 1)
    n = std::max(1, cfg.gpus);  // auto / all: 1
    lo.comm = "host";
  } else {
    n = resolve_gpus(cfg, lo);
  }
  return launch_ranks(n, [&](int rank, int size, Comm& comm) {
    const int dev = size > 1 ? lo.device_of(rank) : lo.device_override >= 0 ? lo.device_override : cfg.engine.device;
    return volume_rank(cfg, rank, size, comm, dev);
  }, lo);
}

}  // namespace app
}  // namespace nm03
