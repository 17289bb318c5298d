// pybind11 module `_nm03` — Python surface of the native engine (package nm03_capstone_project_amd).
// Host codecs, golden model, engine, 3D mode, comm self-tests, and raw-pointer kernel entry points
// that the torch-tensor wrappers in nm03_capstone_project_amd/ops use (device pointers + stream).
#include <hip/hip_runtime_api.h>
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <thread>

#include "nm03/app.h"
#include "nm03/cohort.h"
#include "nm03/comm.h"
#include "nm03/cpu_sampler.h"
#include "nm03/dicom.h"
#include "nm03/engine.h"
#include "nm03/metaimage.h"
#include "nm03/numa.h"
#include "nm03/golden.h"
#include "nm03/jpeg.h"
#include "nm03/jpeg_dct.h"
#include "nm03/jpeg_lossless.h"
#include "nm03/kernels.h"
#include "nm03/synth.h"
#include "nm03/volume.h"
#include "nm03/volume_slabs.h"

namespace py = pybind11;
using namespace nm03;

namespace {

template <class T>
py::array_t<T> to_np(const std::vector<T>& v, std::vector<py::ssize_t> shape) {
  py::array_t<T> a(shape);
  std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

template <class T>
std::vector<T> from_np(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
  return std::vector<T>(a.data(), a.data() + a.size());
}

PixelType parse_type(const std::string& t) {
  if (t == "u16") return kU16;
  if (t == "i16") return kI16;
  if (t == "u8") return kU8;
  throw std::invalid_argument("pixel type must be u16, i16 or u8");
}

golden::SliceInput slice_from(py::array_t<uint16_t, py::array::c_style | py::array::forcecast> raw, const std::string& type,
                              int stored_bits, float slope, float intercept, float sx, float sy) {
  if (raw.ndim() != 2) throw std::invalid_argument("raw must be a 2D uint16 array");
  golden::SliceInput s;
  s.h = (int)raw.shape(0);
  s.w = (int)raw.shape(1);
  s.type = parse_type(type);
  if (s.type == kU8) s.type = kU16;
  s.stored_bits = stored_bits;
  s.slope = slope;
  s.intercept = intercept;
  s.spacing_x = sx;
  s.spacing_y = sy;
  s.raw = from_np<uint16_t>(raw);
  return s;
}

py::dict header_dict(const dicom::Header& h) {
  py::dict d;
  d["rows"] = h.rows;
  d["cols"] = h.cols;
  d["bits_allocated"] = h.bits_allocated;
  d["bits_stored"] = h.bits_stored;
  d["pixel_representation"] = h.pixel_rep;
  d["type"] = h.type == kU16 ? "u16" : h.type == kI16 ? "i16" : "u8";
  d["has_rescale"] = h.has_rescale;
  d["slope"] = h.slope;
  d["intercept"] = h.intercept;
  d["spacing_x"] = h.spacing_x;
  d["spacing_y"] = h.spacing_y;
  d["instance_number"] = h.instance_number;
  d["transfer_syntax"] = h.transfer_syntax;
  d["photometric"] = h.photometric;
  d["patient_id"] = h.patient_id;
  d["modality"] = h.modality;
  d["sop_instance_uid"] = h.sop_instance_uid;
  d["series_uid"] = h.series_uid;
  d["pixel_offset"] = h.pixel_offset;
  d["pixel_length"] = h.pixel_length;
  d["frames"] = h.frames;
  d["invert"] = h.invert;
  d["syntax"] = dicom::syntax_name(h.syntax);
  return d;
}

std::vector<Seed> seeds_from(const std::vector<std::tuple<int, int, int>>& s) {
  std::vector<Seed> v;
  for (auto& t : s) v.push_back({std::get<0>(t), std::get<1>(t), std::get<2>(t)});
  return v;
}

py::array_t<uint8_t> mask2d(const std::vector<uint8_t>& v, int h, int w) { return to_np<uint8_t>(v, {h, w}); }

// ---- device scratch for the raw-pointer kernel entry points --------------------------------
struct Scratch {
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t bytes) {
    if (bytes > cap) {
      if (p) (void)hipFree(p);
      cap = std::max<size_t>(bytes, 1 << 20);
      gpu::check_hip(hipMalloc(&p, cap), "hipMalloc scratch");
    }
    return p;
  }
};
Scratch& scratch() {
  static Scratch s;
  return s;
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Builds SliceDesc/TileDesc tables for n equally sized slices laid out contiguously
// (raw/med: n×h×w u16; masks: n×h×wpr words) and uploads them (synchronously) to scratch.
struct BatchTables {
  gpu::SliceDesc* desc;
  gpu::TileDesc* medt;
  gpu::TileDesc* shpt;
  gpu::SeedXY* seeds;
  gpu::SliceStats* stats;
  int nmed, nshp;
};

BatchTables upload_tables(int n, int h, int w, PixelType type, int stored_bits, float slope, float intercept,
                          const std::vector<Seed>& seeds, hipStream_t st) {
  std::vector<gpu::SliceDesc> d(n);
  std::vector<gpu::TileDesc> mt, sh;
  std::vector<gpu::SeedXY> sd;
  const int wpr = (w + 63) / 64;
  for (int i = 0; i < n; ++i) {
    gpu::SliceDesc& s = d[i];
    std::memset(&s, 0, sizeof(s));
    s.raw_off = (uint32_t)((size_t)i * h * w);
    s.mask_off = (uint32_t)((size_t)i * h * wpr);
    s.f32_off = s.raw_off;
    s.w = (uint16_t)w;
    s.h = (uint16_t)h;
    s.wpr = (uint16_t)wpr;
    s.type = type == kU8 ? kU16 : type;
    s.stored_bits = (uint8_t)stored_bits;
    s.slope = slope;
    s.intercept = intercept;
    s.seed_off = (uint32_t)sd.size();
    s.seed_count = (uint16_t)seeds.size();
    for (auto& q : seeds) sd.push_back({(int16_t)q.x, (int16_t)q.y});
    for (int ty = 0; ty < (h + 63) / 64; ++ty)
      for (int tx = 0; tx < (w + 63) / 64; ++tx) mt.push_back({(uint32_t)i, (uint16_t)tx, (uint16_t)ty});
    for (int ty = 0; ty < (h + gpu::kShpTileH - 1) / gpu::kShpTileH; ++ty)
      for (int tx = 0; tx < wpr; ++tx) sh.push_back({(uint32_t)i, (uint16_t)tx, (uint16_t)ty});
  }
  if (sd.empty()) sd.push_back({0, 0});
  std::vector<gpu::SliceStats> stats(n, gpu::SliceStats{0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0u});
  const size_t o1 = 0, o2 = o1 + d.size() * sizeof(gpu::SliceDesc), o3 = (o2 + mt.size() * 8 + 255) / 256 * 256,
               o4 = (o3 + sh.size() * 8 + 255) / 256 * 256, o5 = (o4 + sd.size() * 4 + 255) / 256 * 256,
               total = o5 + stats.size() * sizeof(gpu::SliceStats);
  std::vector<uint8_t> blob(total);
  std::memcpy(blob.data() + o1, d.data(), d.size() * sizeof(gpu::SliceDesc));
  std::memcpy(blob.data() + o2, mt.data(), mt.size() * 8);
  std::memcpy(blob.data() + o3, sh.data(), sh.size() * 8);
  std::memcpy(blob.data() + o4, sd.data(), sd.size() * 4);
  std::memcpy(blob.data() + o5, stats.data(), stats.size() * sizeof(gpu::SliceStats));
  uint8_t* dev = (uint8_t*)scratch().get(total);
  gpu::check_hip(hipMemcpyAsync(dev, blob.data(), total, hipMemcpyHostToDevice, st), "H2D tables");
  gpu::check_hip(hipStreamSynchronize(st), "sync tables");
  return BatchTables{(gpu::SliceDesc*)(dev + o1), (gpu::TileDesc*)(dev + o2), (gpu::TileDesc*)(dev + o3),
                     (gpu::SeedXY*)(dev + o4), (gpu::SliceStats*)(dev + o5), (int)mt.size(), (int)sh.size()};
}

gpu::PipeConsts consts_from(const PipelineParams& p, int border_radius) {
  gpu::PipeConsts pc{};
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
  pc.border_radius = border_radius;
  pc.se_disc = p.se_shape == kSeDisc ? 1 : 0;
  return pc;
}

}  // namespace

template <class Fn>
py::dict volume_call(py::array_t<uint16_t, py::array::c_style | py::array::forcecast> vol, const PipelineParams& p,
                     int connectivity, int dilation, const std::vector<std::tuple<int, int, int>>& seeds, Fn&& fn) {
  if (vol.ndim() != 3) throw std::invalid_argument("volume must be (depth, height, width)");
  VolumeInput v;
  v.d = (int)vol.shape(0);
  v.h = (int)vol.shape(1);
  v.w = (int)vol.shape(2);
  v.raw = from_np<uint16_t>(vol);
  VolumeParams vp;
  vp.pipe = p;
  vp.connectivity = connectivity;
  vp.dilation_size = dilation;
  vp.seeds = seeds_from(seeds);
  VolumeResult r;
  {
    py::gil_scoped_release nogil;
    r = fn(v, vp);
  }
  py::dict d;
  d["band"] = to_np<uint8_t>(r.band, {v.d, v.h, v.w});
  d["region"] = to_np<uint8_t>(r.region, {v.d, v.h, v.w});
  d["dilated"] = to_np<uint8_t>(r.dilated, {v.d, v.h, v.w});
  d["sweeps"] = r.sweeps;
  d["kernels_s"] = r.kernels_s;
  return d;
}

PYBIND11_MODULE(_nm03, m) {
  m.doc() = "NM03 MI355X-native DICOM batch engine (native core)";

  // ---- parameters -----------------------------------------------------------------------------
  py::class_<PipelineParams>(m, "PipelineParams")
      .def(py::init<>())
      .def_readwrite("norm_low", &PipelineParams::norm_low)
      .def_readwrite("norm_high", &PipelineParams::norm_high)
      .def_readwrite("norm_min", &PipelineParams::norm_min)
      .def_readwrite("norm_max", &PipelineParams::norm_max)
      .def_readwrite("clip_min", &PipelineParams::clip_min)
      .def_readwrite("clip_max", &PipelineParams::clip_max)
      .def_readwrite("median_window", &PipelineParams::median_window)
      .def_readwrite("sharpen_gain", &PipelineParams::sharpen_gain)
      .def_readwrite("sharpen_sigma", &PipelineParams::sharpen_sigma)
      .def_readwrite("sharpen_mask", &PipelineParams::sharpen_mask)
      .def_readwrite("srg_min", &PipelineParams::srg_min)
      .def_readwrite("srg_max", &PipelineParams::srg_max)
      .def_readwrite("srg_connectivity", &PipelineParams::srg_connectivity)
      .def_readwrite("dilation_size", &PipelineParams::dilation_size)
      .def_readwrite("erosion_size", &PipelineParams::erosion_size)
      .def_readwrite("min_dim", &PipelineParams::min_dim)
      .def_readwrite("apply_rescale", &PipelineParams::apply_rescale)
      .def_readwrite("frame", &PipelineParams::frame)
      .def_readwrite("se_shape", &PipelineParams::se_shape);
  py::class_<RenderParams>(m, "RenderParams")
      .def(py::init<>())
      .def_readwrite("out_width", &RenderParams::out_width)
      .def_readwrite("out_height", &RenderParams::out_height)
      .def_readwrite("label_opacity", &RenderParams::label_opacity)
      .def_readwrite("border_opacity", &RenderParams::border_opacity)
      .def_readwrite("border_radius", &RenderParams::border_radius)
      .def_readwrite("jpeg_quality", &RenderParams::jpeg_quality)
      .def_readwrite("filter", &RenderParams::filter)
      .def_readwrite("jpeg_sampling", &RenderParams::jpeg_sampling);
  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("device", &EngineConfig::device)
      .def_readwrite("batch_size", &EngineConfig::batch_size)
      .def_readwrite("streams", &EngineConfig::streams)
      .def_readwrite("threads", &EngineConfig::threads)
      .def_readwrite("cpus", &EngineConfig::cpus)
      .def_readwrite("max_dim", &EngineConfig::max_dim)
      .def_readwrite("pipe", &EngineConfig::pipe)
      .def_readwrite("render", &EngineConfig::render)
      .def_readwrite("export_jpeg", &EngineConfig::export_jpeg)
      .def_readwrite("resume", &EngineConfig::resume)
      .def_readwrite("jpeg_out_cap", &EngineConfig::jpeg_out_cap)
      .def_readwrite("upload_chunk_kb", &EngineConfig::upload_chunk_kb)
      .def_readwrite("create_writers", &EngineConfig::create_writers)
      .def_readwrite("lazy_slots", &EngineConfig::lazy_slots)
      .def_readwrite("host_only", &EngineConfig::host_only);

  m.def("reference_seeds", [](int w, int h) {
    std::vector<std::pair<int, int>> v;
    for (auto& s : reference_seeds(w, h)) v.push_back({s.x, s.y});
    return v;
  });
  m.def("gaussian_taps", [](float sigma, int mask) {
    std::vector<float> t(mask);
    gaussian_taps(sigma, mask, t.data());
    return t;
  });

  // ---- DICOM -----------------------------------------------------------------------------------
  m.def("dicom_parse", [](py::bytes b) {
    std::string s = b;
    return header_dict(dicom::parse((const uint8_t*)s.data(), s.size()));
  });
  m.def(
      "dicom_pixels",
      [](py::bytes b, int frame) {
        std::string s = b;
        dicom::Header h = dicom::parse((const uint8_t*)s.data(), s.size());
        std::vector<uint16_t> px((size_t)h.rows * h.cols);
        dicom::copy_pixels16(h, (const uint8_t*)s.data(), s.size(), px.data(), frame);
        return to_np<uint16_t>(px, {h.rows, h.cols});
      },
      py::arg("data"), py::arg("frame") = 0);
  m.def("dicom_select_frame", [](py::bytes b, int policy) {
    std::string s = b;
    return dicom::select_frame(dicom::parse((const uint8_t*)s.data(), s.size()), policy);
  });
  m.def(
      "dicom_bytes",
      [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> px, const std::string& type, int bits_stored,
         bool write_rescale, float slope, float intercept, float sx, float sy, int instance, const std::string& patient_id,
         const std::string& syntax, bool preamble, const std::string& photometric, int jpeg_predictor,
         int jpeg_restart_rows, int jpeg_fragments, int jpeg_quality) {
        dicom::WriteSpec w;
        w.jpeg_quality = jpeg_quality;
        w.jpeg_predictor = jpeg_predictor;
        w.jpeg_restart_rows = jpeg_restart_rows;
        w.jpeg_fragments = jpeg_fragments;
        // (rows, cols) or (frames, rows, cols)
        if (px.ndim() != 2 && px.ndim() != 3) throw std::invalid_argument("pixels must be 2D or 3D (frames, rows, cols)");
        w.frames = px.ndim() == 3 ? (int)px.shape(0) : 1;
        w.rows = (int)px.shape(px.ndim() - 2);
        w.cols = (int)px.shape(px.ndim() - 1);
        w.photometric = photometric;
        w.type = parse_type(type);
        w.bits_stored = bits_stored;
        std::vector<uint16_t> v = from_np<uint16_t>(px);
        w.pixels = v.data();
        w.write_rescale = write_rescale;
        w.slope = slope;
        w.intercept = intercept;
        w.spacing_x = sx;
        w.spacing_y = sy;
        w.instance_number = instance;
        w.patient_id = patient_id;
        w.syntax = syntax == "implicit"   ? dicom::Syntax::kImplicitLE
                   : syntax == "big"      ? dicom::Syntax::kExplicitBE
                   : syntax == "deflated" ? dicom::Syntax::kDeflatedLE
                   : syntax == "rle"      ? dicom::Syntax::kRleLossless
                   : syntax == "jpeg-lossless" ? dicom::Syntax::kJpegLossless
                   : syntax == "jpeg-baseline" ? dicom::Syntax::kJpegBaseline
                   : syntax == "jpeg-extended" ? dicom::Syntax::kJpegExtended
                   : syntax == "explicit" ? dicom::Syntax::kExplicitLE
                                          : throw std::invalid_argument("syntax: implicit|explicit|big|deflated|rle|jpeg-lossless|jpeg-baseline|jpeg-extended");
        w.preamble = preamble;
        auto b = dicom::write(w);
        return py::bytes((const char*)b.data(), b.size());
      },
      py::arg("pixels"), py::arg("type") = "u16", py::arg("bits_stored") = 16, py::arg("write_rescale") = false,
      py::arg("slope") = 1.f, py::arg("intercept") = 0.f, py::arg("spacing_x") = 1.f, py::arg("spacing_y") = 1.f,
      py::arg("instance") = 1, py::arg("patient_id") = "PGBM-000", py::arg("syntax") = "explicit",
      py::arg("preamble") = true, py::arg("photometric") = "MONOCHROME2", py::arg("jpeg_predictor") = 1,
      py::arg("jpeg_restart_rows") = 0, py::arg("jpeg_fragments") = 1, py::arg("jpeg_quality") = 90);
  m.def("jpeg_dct_decode", [](py::bytes b) {
    const std::string s = b;
    std::vector<uint16_t> px;
    const jpegdct::Info i = jpegdct::decode((const uint8_t*)s.data(), s.size(), px);
    py::dict d;
    d["precision"] = i.precision;
    d["sof"] = i.sof;
    d["restart_interval"] = i.restart_interval;
    d["pixels"] = to_np(px, {(py::ssize_t)i.rows, (py::ssize_t)i.cols});
    return d;
  });
  m.def("jpeg_dct_encode", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> px, int precision,
                              int quality, int restart_blocks) {
    if (px.ndim() != 2) throw std::invalid_argument("pixels must be 2D");
    std::vector<uint16_t> v = from_np<uint16_t>(px);
    auto j = jpegdct::encode(v.data(), (int)px.shape(0), (int)px.shape(1), precision, quality, restart_blocks);
    return py::bytes((const char*)j.data(), j.size());
  }, py::arg("pixels"), py::arg("precision") = 8, py::arg("quality") = 90, py::arg("restart_blocks") = 0);
  m.def("jpeg_lossless_decode", [](py::bytes b) {
    const std::string s = b;
    std::vector<uint16_t> px;
    const jpegll::Info i = jpegll::decode((const uint8_t*)s.data(), s.size(), px);
    py::dict d;
    d["precision"] = i.precision;
    d["predictor"] = i.predictor;
    d["point_transform"] = i.point_transform;
    d["restart_interval"] = i.restart_interval;
    d["pixels"] = to_np(px, {(py::ssize_t)i.rows, (py::ssize_t)i.cols});
    return d;
  });
  m.def("jpeg_lossless_encode", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> px, int precision,
                                   int predictor, int pt, int restart_rows) {
    if (px.ndim() != 2) throw std::invalid_argument("pixels must be 2D");
    std::vector<uint16_t> v = from_np<uint16_t>(px);
    auto j = jpegll::encode(v.data(), (int)px.shape(0), (int)px.shape(1), precision, predictor, pt, restart_rows);
    return py::bytes((const char*)j.data(), j.size());
  }, py::arg("pixels"), py::arg("precision") = 16, py::arg("predictor") = 1, py::arg("pt") = 0, py::arg("restart_rows") = 0);
  m.def("numa_parse_cpulist", &numa::parse_cpulist);
  m.def(
      "mhd_write",
      [](const std::string& base, py::array arr, float sx, float sy, float sz) {
        py::buffer_info bi = arr.request();
        if (!(py::array::c_style & arr.flags())) throw std::invalid_argument("array must be C-contiguous");
        mhd::MetType t;
        const std::string f = bi.format;
        if (bi.itemsize == 1) t = mhd::MetType::kUChar;
        else if (bi.itemsize == 2 && (f == "H")) t = mhd::MetType::kUShort;
        else if (bi.itemsize == 2 && (f == "h")) t = mhd::MetType::kShort;
        else if (bi.itemsize == 4 && f == "f") t = mhd::MetType::kFloat;
        else throw std::invalid_argument("mhd_write: uint8, uint16, int16 or float32 arrays only");
        int w = 1, h = 1, d = 1;
        if (bi.ndim == 2) { h = (int)bi.shape[0]; w = (int)bi.shape[1]; }
        else if (bi.ndim == 3) { d = (int)bi.shape[0]; h = (int)bi.shape[1]; w = (int)bi.shape[2]; }
        else throw std::invalid_argument("mhd_write: 2D or 3D arrays only");
        mhd::write(base, bi.ptr, w, h, d, t, sx, sy, sz);
      },
      py::arg("base"), py::arg("array"), py::arg("sx") = 1.f, py::arg("sy") = 1.f, py::arg("sz") = 1.f);
  m.def("mhd_read", [](const std::string& path) {
    mhd::Image im = mhd::read(path);
    std::vector<py::ssize_t> shape = im.d > 1 ? std::vector<py::ssize_t>{im.d, im.h, im.w}
                                               : std::vector<py::ssize_t>{im.h, im.w};
    py::array a;
    switch (im.type) {
      case mhd::MetType::kUChar: a = py::array_t<uint8_t>(shape); break;
      case mhd::MetType::kUShort: a = py::array_t<uint16_t>(shape); break;
      case mhd::MetType::kShort: a = py::array_t<int16_t>(shape); break;
      case mhd::MetType::kFloat: a = py::array_t<float>(shape); break;
    }
    std::memcpy(a.mutable_data(), im.bytes.data(), im.bytes.size());
    return py::make_tuple(a, py::make_tuple(im.spacing[0], im.spacing[1], im.spacing[2]));
  });
  m.def("numa_node_cpus", &numa::node_cpus);
  m.def("numa_device_node", &numa::device_node, py::arg("device"));
  m.def("device_bus_id", &numa::device_bus_id, py::arg("device"));
  m.def("cpu_budget", &numa::cpu_budget, py::arg("cgroup_root") = "/sys/fs/cgroup");
  m.def("allowed_cpus", &numa::allowed_cpus);
  m.def("format_cpulist", &numa::format_cpulist);
  // Per-rank CPU partition (numa.h): {node, index, count, cpus, threads}. `sysfs` / `allowed` let
  // tests describe a fake host.
  m.def(
      "rank_partition",
      [](const std::vector<int>& rank_nodes, int local_rank, int budget, int cap, const std::string& sysfs,
         const std::vector<int>& allowed) {
        const numa::Topology t = numa::read_topology(sysfs, allowed);
        const numa::RankCpus r = numa::rank_partition(t, rank_nodes, local_rank, budget, cap);
        py::dict d;
        d["node"] = r.node;
        d["index"] = r.index;
        d["count"] = r.count;
        d["cpus"] = r.cpus;
        d["threads"] = r.threads;
        return d;
      },
      py::arg("rank_nodes"), py::arg("local_rank"), py::arg("budget"), py::arg("cap") = 16,
      py::arg("sysfs") = "/sys", py::arg("allowed") = std::vector<int>{});
  m.def(
      "read_pixels_direct",
      [](const std::string& path, const std::string& mode, size_t prefix, int frame) {
        dicom::SliceFile f(path, mode == "staged" ? dicom::ReadMode::kStaged : dicom::ReadMode::kDirect, prefix);
        std::vector<uint8_t> scratch;
        const dicom::Header& h = f.header(scratch);
        std::vector<uint16_t> px((size_t)h.rows * h.cols + 1);  // +1: misaligned destination below
        uint16_t* dst = px.data() + 1;
        f.pixels16(dst, frame);
        std::vector<uint16_t> out(dst, dst + (size_t)h.rows * h.cols);
        // The staged fast path's view of the same frame (None when pixels16 must convert).
        const uint16_t* ss = f.staged_samples(frame);
        py::object staged = py::none();
        if (ss) staged = to_np<uint16_t>(std::vector<uint16_t>(ss, ss + (size_t)h.rows * h.cols), {h.rows, h.cols});
        return py::make_tuple(to_np<uint16_t>(out, {h.rows, h.cols}), f.direct(), staged);
      },
      py::arg("path"), py::arg("mode") = "direct", py::arg("prefix") = 16384, py::arg("frame") = 0);
  m.def(
      "read_slice",
      [](const std::string& path, int min_dim, int frame) {
        golden::SliceInput s = golden::load_slice(path, min_dim, frame);
        py::dict meta;
        meta["type"] = s.type == kI16 ? "i16" : "u16";
        meta["stored_bits"] = s.stored_bits;
        meta["slope"] = s.slope;
        meta["intercept"] = s.intercept;
        meta["spacing_x"] = s.spacing_x;
        meta["spacing_y"] = s.spacing_y;
        return py::make_tuple(to_np<uint16_t>(s.raw, {s.h, s.w}), meta);
      },
      py::arg("path"), py::arg("min_dim") = 0, py::arg("frame") = -1);

  // ---- cohort / synthetic data -------------------------------------------------------------------
  m.def("extract_file_number", &cohort::extract_file_number);
  // img_processing_parallel's default rank count (app.h): policy and the listing-only slice count.
  m.def("auto_gpus", &app::auto_gpus, py::arg("slices"), py::arg("visible"));
  m.def("auto_slices_per_rank", [] { return app::kAutoSlicesPerRank; });
  m.def("count_cohort_slices", [](const std::string& data_root) {
    app::AppConfig c;
    c.data_root = cohort::with_slash(data_root);
    return app::count_cohort_slices(c);
  });
  m.def("default_data_root", &cohort::default_data_root);
  m.def("cohort_dir", &cohort::cohort_dir);
  m.def("test_slice_path", &cohort::test_slice_path);
  m.def("find_patient_dirs", &cohort::find_patient_dirs);
  m.def("list_patient_series", [](const std::string& root, const std::string& pid) {
    auto s = cohort::list_patient_series(root, pid);
    return py::make_tuple(s.series_dir, s.files);
  });
  m.def("setup_output_dir", &cohort::setup_output_dir);
  m.def("setup_output_dirs", [](const std::vector<std::string>& dirs, int threads) {
    py::gil_scoped_release nogil;
    cohort::setup_output_dirs(dirs, threads);
  }, py::arg("dirs"), py::arg("threads") = 8);
  py::class_<cohort::OutputReaper>(m, "OutputReaper")
      .def(py::init<int>(), py::arg("threads") = 4)
      .def("wipe", [](cohort::OutputReaper& r, const std::vector<std::string>& dirs) {
        py::gil_scoped_release nogil;
        r.wipe(dirs);
      })
      .def("drain", [](cohort::OutputReaper& r) {
        py::gil_scoped_release nogil;
        r.drain();
      })
      .def_property_readonly("files_reaped", &cohort::OutputReaper::files_reaped);
  m.def(
      "synth_cohort",
      [](const std::string& root, int patients, int min_slices, int max_slices, int rows, int cols, uint64_t seed,
         int threads, bool test_slice, bool decoy, bool signed_px) {
        synth::CohortSpec s;
        s.data_root = cohort::with_slash(root);
        s.patients = patients;
        s.min_slices = min_slices;
        s.max_slices = max_slices;
        s.rows = rows;
        s.cols = cols;
        s.seed = seed;
        s.threads = threads;
        s.test_slice = test_slice;
        s.decoy_series = decoy;
        s.type = signed_px ? kI16 : kU16;
        py::gil_scoped_release nogil;
        return synth::generate_cohort(s);
      },
      py::arg("data_root"), py::arg("patients") = 20, py::arg("min_slices") = 21, py::arg("max_slices") = 25,
      py::arg("rows") = 256, py::arg("cols") = 256, py::arg("seed") = 20250404, py::arg("threads") = 8,
      py::arg("test_slice") = true, py::arg("decoy") = false, py::arg("signed") = false);
  m.def("synth_flat", [](const std::string& root, int count, int rows, int cols, uint64_t seed, int threads) {
    py::gil_scoped_release nogil;
    return synth::generate_flat(root, count, rows, cols, seed, threads);
  });
  m.def("phantom_slice", [](int rows, int cols, int patient, int slice, int nslices, uint64_t seed) {
    std::vector<uint16_t> v((size_t)rows * cols);
    synth::phantom_slice(rows, cols, patient, slice, nslices, seed, v.data());
    return to_np<uint16_t>(v, {rows, cols});
  });

  // ---- golden model ----------------------------------------------------------------------------
  m.def(
      "golden_run",
      [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> raw, const std::string& type, int stored_bits,
         float slope, float intercept, const PipelineParams& p, const RenderParams& rp, float sx, float sy) {
        golden::SliceInput s = slice_from(raw, type, stored_bits, slope, intercept, sx, sy);
        golden::SliceResult r = golden::run(s, p, true);
        py::dict d;
        d["clipped"] = to_np<float>(r.clipped, {s.h, s.w});
        d["median"] = to_np<float>(r.median, {s.h, s.w});
        d["sharpened"] = to_np<float>(r.sharpened, {s.h, s.w});
        d["band"] = mask2d(r.band, s.h, s.w);
        d["region"] = mask2d(r.region, s.h, s.w);
        d["eroded"] = mask2d(r.eroded, s.h, s.w);
        d["dilated"] = mask2d(r.dilated, s.h, s.w);
        d["window"] = py::make_tuple(r.window_lo, r.window_hi);
        golden::SliceJpegs j = golden::export_jpegs(s, r, p, rp);
        d["jpeg_original"] = py::bytes((const char*)j.original.data(), j.original.size());
        d["jpeg_processed"] = py::bytes((const char*)j.processed.data(), j.processed.size());
        return d;
      },
      py::arg("raw"), py::arg("type") = "u16", py::arg("stored_bits") = 16, py::arg("slope") = 1.f,
      py::arg("intercept") = 0.f, py::arg("params") = PipelineParams(), py::arg("render") = RenderParams(),
      py::arg("spacing_x") = 1.f, py::arg("spacing_y") = 1.f);
  m.def("golden_norm_clip", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> raw, const std::string& type,
                               int stored_bits, float slope, float intercept, const PipelineParams& p) {
    golden::SliceInput s = slice_from(raw, type, stored_bits, slope, intercept, 1, 1);
    return to_np<float>(golden::norm_clip(s, p), {s.h, s.w});
  });
  m.def("golden_median", [](py::array_t<float, py::array::c_style | py::array::forcecast> img, int k) {
    const int h = (int)img.shape(0), w = (int)img.shape(1);
    return to_np<float>(golden::median(from_np<float>(img), w, h, k), {h, w});
  });
  m.def("golden_median_u16", [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> img, int k) {
    const int h = (int)img.shape(0), w = (int)img.shape(1);
    return to_np<uint16_t>(golden::median_u16(from_np<uint16_t>(img), w, h, k), {h, w});
  });
  m.def("golden_vector_median", [](py::array_t<float, py::array::c_style | py::array::forcecast> img, int k) {
    const int h = (int)img.shape(0), w = (int)img.shape(1);
    return to_np<float>(golden::vector_median(from_np<float>(img), w, h, k), {h, w});
  });
  m.def("golden_sharpen", [](py::array_t<float, py::array::c_style | py::array::forcecast> img, float gain, float sigma,
                             int mask, bool direct) {
    const int h = (int)img.shape(0), w = (int)img.shape(1);
    auto v = from_np<float>(img);
    return to_np<float>(direct ? golden::sharpen_direct(v, w, h, gain, sigma, mask) : golden::sharpen(v, w, h, gain, sigma, mask),
                        {h, w});
  }, py::arg("img"), py::arg("gain") = 2.0f, py::arg("sigma") = 0.5f, py::arg("mask") = 9, py::arg("direct") = false);
  m.def("golden_region_grow", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> band,
                                 const std::vector<std::tuple<int, int, int>>& seeds, int conn) {
    const int h = (int)band.shape(0), w = (int)band.shape(1);
    return mask2d(golden::region_grow(from_np<uint8_t>(band), w, h, seeds_from(seeds), conn), h, w);
  });
  m.def(
      "golden_morph",
      [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> mk, int size, bool dilate, bool disc) {
        const int h = (int)mk.shape(0), w = (int)mk.shape(1);
        auto v = from_np<uint8_t>(mk);
        return mask2d(dilate ? golden::dilate(v, w, h, size, disc) : golden::erode(v, w, h, size, disc), h, w);
      },
      py::arg("mask"), py::arg("size"), py::arg("dilate"), py::arg("disc") = false);
  m.def("golden_border", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> mk, int radius) {
    const int h = (int)mk.shape(0), w = (int)mk.shape(1);
    return mask2d(golden::border(from_np<uint8_t>(mk), w, h, radius), h, w);
  });
  m.def("golden_region_grow3d", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> band,
                                   const std::vector<std::tuple<int, int, int>>& seeds, int conn) {
    const int d = (int)band.shape(0), h = (int)band.shape(1), w = (int)band.shape(2);
    return to_np<uint8_t>(golden::region_grow3d(from_np<uint8_t>(band), w, h, d, seeds_from(seeds), conn), {d, h, w});
  });
  m.def(
      "golden_dilate3d",
      [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> mk, int size, bool ball) {
        const int d = (int)mk.shape(0), h = (int)mk.shape(1), w = (int)mk.shape(2);
        return to_np<uint8_t>(golden::dilate3d(from_np<uint8_t>(mk), w, h, d, size, ball), {d, h, w});
      },
      py::arg("mask"), py::arg("size"), py::arg("ball") = false);
  m.def(
      "golden_render_gray",
      [](py::array_t<float, py::array::c_style | py::array::forcecast> v, float lo, float hi, float sx, float sy, int out_w,
         int out_h, bool nearest) {
        const int h = (int)v.shape(0), w = (int)v.shape(1);
        RenderGeom g = make_render_geom(w, h, sx, sy, out_w, out_h);
        return to_np<uint8_t>(golden::render_gray(from_np<float>(v), g, lo, hi, nearest), {out_h, out_w});
      },
      py::arg("values"), py::arg("lo"), py::arg("hi"), py::arg("sx"), py::arg("sy"), py::arg("out_w"), py::arg("out_h"),
      py::arg("nearest") = false);
  m.def("golden_render_labels", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> lab,
                                   py::array_t<uint8_t, py::array::c_style | py::array::forcecast> brd, float sx, float sy,
                                   int out_w, int out_h, int fill, int bv) {
    const int h = (int)lab.shape(0), w = (int)lab.shape(1);
    RenderGeom g = make_render_geom(w, h, sx, sy, out_w, out_h);
    return to_np<uint8_t>(golden::render_labels(from_np<uint8_t>(lab), from_np<uint8_t>(brd), g, (uint8_t)fill, (uint8_t)bv),
                          {out_h, out_w});
  });
  m.def("opacity_u8", &opacity_u8);

  // ---- JPEG --------------------------------------------------------------------------------------
  m.def("jpeg_encode_gray420", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> g, int quality) {
    const int h = (int)g.shape(0), w = (int)g.shape(1);
    auto b = jpeg::encode_gray(g.data(), w, h, w, quality);
    return py::bytes((const char*)b.data(), b.size());
  }, py::arg("gray"), py::arg("quality") = 75);
  // sampling: jpeg::Sampling (0 YCbCr 4:2:0, 1 YCbCr 4:4:4, 2 one gray component).
  m.def("jpeg_encode_gray", [](py::array_t<uint8_t, py::array::c_style | py::array::forcecast> g, int quality,
                               int sampling) {
    if (sampling < 0 || sampling > 2) throw std::invalid_argument("sampling must be 0, 1 or 2");
    const int h = (int)g.shape(0), w = (int)g.shape(1);
    auto b = jpeg::encode_gray(g.data(), w, h, w, quality, (jpeg::Sampling)sampling);
    return py::bytes((const char*)b.data(), b.size());
  }, py::arg("gray"), py::arg("quality") = 75, py::arg("sampling") = 0);
  m.def("jpeg_header", [](int w, int h, int quality, int sampling) {
    if (sampling < 0 || sampling > 2) throw std::invalid_argument("sampling must be 0, 1 or 2");
    auto b = jpeg::make_header(w, h, jpeg::make_tables(quality), (jpeg::Sampling)sampling);
    return py::bytes((const char*)b.data(), b.size());
  }, py::arg("w"), py::arg("h"), py::arg("quality") = 75, py::arg("sampling") = 0);
  m.def("jpeg_quant_tables", [](int quality) {
    auto t = jpeg::make_tables(quality);
    return py::make_tuple(std::vector<int>(t.qluma, t.qluma + 64), std::vector<int>(t.qchroma, t.qchroma + 64));
  });

  // ---- engine --------------------------------------------------------------------------------------
  // A work list converted once to its native form (the cohort plan), reusable across runs and
  // shared with the engine while a submitted run is in flight.
  struct WorkList {
    std::shared_ptr<std::vector<WorkItem>> items = std::make_shared<std::vector<WorkItem>>();
  };
  py::class_<WorkList>(m, "WorkList")
      .def(py::init([](const std::vector<std::pair<std::string, std::string>>& items) {
        WorkList w;
        w.items->reserve(items.size());
        for (auto& p : items) w.items->push_back({p.first, p.second});
        return w;
      }))
      .def("__len__", [](const WorkList& w) { return w.items->size(); })
      .def("items", [](const WorkList& w) {
        std::vector<std::pair<std::string, std::string>> v;
        v.reserve(w.items->size());
        for (auto& it : *w.items) v.push_back({it.path, it.out_dir});
        return v;
      })
      // A reference run's set-up in one native call (main_sequential.cpp:93-168, 32-47): discover
      // the PGBM-* patients under data_root's cohort directory, per patient wipe (through `reaper`:
      // rename aside + background deletion) or create <out_root>/<pid>, list its first series in
      // reference order, and build the work list.
      .def_static(
          "discover",
          [](const std::string& data_root, const std::string& out_root, cohort::OutputReaper* reaper) {
            py::gil_scoped_release nogil;
            WorkList w;
            const std::string base = cohort::cohort_dir(data_root);
            for (const auto& pid : cohort::find_patient_dirs(base)) {
              const std::string out = out_root + "/" + pid;
              if (reaper)
                reaper->wipe(out);
              else
                cohort::make_dirs(out);
              cohort::Series s = cohort::list_patient_series(base, pid);
              for (auto& f : s.files) w.items->push_back({std::move(f), out});
            }
            return w;
          },
          py::arg("data_root"), py::arg("out_root"), py::arg("reaper") = nullptr);
  struct Ticket {
    RunTicket t;
  };
  py::class_<Ticket>(m, "RunTicket");
  auto times_dict = [](const StageTimes& t) {
    py::dict td;
    td["load_s"] = t.load_s;
    td["h2d_s"] = t.h2d_s;
    td["kernels_s"] = t.kernels_s;
    td["write_s"] = t.write_s;
    td["load_cpu_s"] = t.load_cpu_s;
    td["write_cpu_s"] = t.write_cpu_s;
    td["slot_cpu_s"] = t.slot_cpu_s;
    td["wall_s"] = t.wall_s;
    td["batches"] = t.batches;
    td["slices_ok"] = t.slices_ok;
    td["slices_failed"] = t.slices_failed;
    td["bytes_in"] = t.bytes_in;
    td["bytes_out"] = t.bytes_out;
    td["jpeg_fallbacks"] = t.jpeg_fallbacks;
    return td;
  };
  auto compact = [times_dict](const std::vector<SliceStatus>& st, const StageTimes& t) {
    py::array_t<int32_t> codes((py::ssize_t)st.size());
    auto c = codes.mutable_unchecked<1>();
    py::dict msgs;
    for (size_t i = 0; i < st.size(); ++i) {
      c((py::ssize_t)i) = st[i].code;
      if (st[i].code != kSliceOk) msgs[py::int_(i)] = st[i].message;
    }
    return py::make_tuple(codes, msgs, times_dict(t));
  };
  py::class_<Engine>(m, "Engine")
      .def(py::init<const EngineConfig&>())
      .def(
          "run",
          [times_dict](Engine& e, const std::vector<std::pair<std::string, std::string>>& items) {
            std::vector<WorkItem> wi;
            for (auto& p : items) wi.push_back({p.first, p.second});
            StageTimes t;
            std::vector<SliceStatus> st;
            {
              py::gil_scoped_release nogil;
              st = e.run(wi, &t);
            }
            std::vector<std::pair<int, std::string>> out;
            for (auto& s : st) out.push_back({s.code, s.message});
            return py::make_tuple(out, times_dict(t));
          })
      .def(
          "run_list",
          // Compact form for hot loops: (codes int32[n], {index: message} for non-OK slices, times).
          [compact](Engine& e, const WorkList& wl, int batch_cap) {
            StageTimes t;
            std::vector<SliceStatus> st;
            {
              py::gil_scoped_release nogil;
              st = e.run(*wl.items, &t, {}, batch_cap);
            }
            return compact(st, t);
          },
          py::arg("work"), py::arg("batch_cap") = 0)
      .def(
          "submit",
          // Queue a run and return at once (Engine::submit); the next run can be submitted before
          // this one finished — the engine pipelines across them.
          [](Engine& e, const WorkList& wl, int batch_cap) {
            py::gil_scoped_release nogil;
            return Ticket{e.submit(wl.items, {}, batch_cap)};
          },
          py::arg("work"), py::arg("batch_cap") = 0)
      .def(
          "wait",
          // Result of a submitted run, in run_list's compact form.
          [compact](Engine& e, const Ticket& t) {
            StageTimes tm;
            std::vector<SliceStatus> st;
            {
              py::gil_scoped_release nogil;
              st = e.wait(t.t, &tm);
            }
            return compact(st, tm);
          })
      .def("run_single",
           [](Engine& e, py::array_t<uint16_t, py::array::c_style | py::array::forcecast> raw, const std::string& type,
              int stored_bits, float slope, float intercept, float sx, float sy) {
             golden::SliceInput s = slice_from(raw, type, stored_bits, slope, intercept, sx, sy);
             SingleResult r;
             {
               py::gil_scoped_release nogil;
               r = e.run_single(s);
             }
             py::dict d;
             d["median_keys"] = to_np<uint16_t>(r.median_keys, {r.h, r.w});
             d["sharpened"] = to_np<float>(r.sharpened, {r.h, r.w});
             d["band"] = mask2d(r.band, r.h, r.w);
             d["region"] = mask2d(r.region, r.h, r.w);
             d["eroded"] = mask2d(r.eroded, r.h, r.w);
             d["dilated"] = mask2d(r.dilated, r.h, r.w);
             d["border_region"] = mask2d(r.border_region, r.h, r.w);
             d["border_eroded"] = mask2d(r.border_eroded, r.h, r.w);
             d["border_dilated"] = mask2d(r.border_dilated, r.h, r.w);
             py::list cv, jp;
             const int cw = e.config().render.out_width, ch = e.config().render.out_height;
             for (auto& c : r.canvases) cv.append(to_np<uint8_t>(c, {ch, cw}));
             for (auto& j : r.jpegs) jp.append(py::bytes((const char*)j.data(), j.size()));
             d["canvases"] = cv;
             d["jpegs"] = jp;
             return d;
           },
           py::arg("raw"), py::arg("type") = "u16", py::arg("stored_bits") = 16, py::arg("slope") = 1.f,
           py::arg("intercept") = 0.f, py::arg("spacing_x") = 1.f, py::arg("spacing_y") = 1.f);
  m.def("device_count", &device_count);
  // CPU sampling profiler (cpu_sampler.h; bench.py --cpu-profile, tools/cpu_profile.py).
  m.def("cpu_profile_start", &prof::sampler_start, py::arg("period_us") = 250, py::arg("max_samples") = 1 << 20,
        py::arg("depth") = 24);
  m.def("cpu_profile_stop", &prof::sampler_stop, py::arg("path"), py::call_guard<py::gil_scoped_release>());

  // ---- 3D ---------------------------------------------------------------------------------------------
  m.def(
      "run_volume",
      [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> vol, const PipelineParams& p, int connectivity,
         int dilation, const std::vector<std::tuple<int, int, int>>& seeds, int device) {
        return volume_call(vol, p, connectivity, dilation, seeds, [device](const VolumeInput& v, const VolumeParams& vp) {
          return run_volume(v, vp, device, true);
        });
      },
      py::arg("volume"), py::arg("params") = PipelineParams(), py::arg("connectivity") = 6, py::arg("dilation") = 7,
      py::arg("seeds") = std::vector<std::tuple<int, int, int>>{}, py::arg("device") = 0);
  // Persistent runner: device buffers, stream, events and pinned staging are kept across volumes
  // (0.94 ms per 256^3 volume vs ~8.7 ms for the one-shot run_volume).
  py::class_<VolumeRunner>(m, "VolumeRunner")
      .def(py::init<int>(), py::arg("device") = 0)
      .def(
          "run",
          [](VolumeRunner& self, py::array_t<uint16_t, py::array::c_style | py::array::forcecast> vol,
             const PipelineParams& p, int connectivity, int dilation,
             const std::vector<std::tuple<int, int, int>>& seeds) {
            return volume_call(vol, p, connectivity, dilation, seeds,
                               [&self](const VolumeInput& v, const VolumeParams& vp) { return self.run(v, vp, true); });
          },
          py::arg("volume"), py::arg("params") = PipelineParams(), py::arg("connectivity") = 6,
          py::arg("dilation") = 7, py::arg("seeds") = std::vector<std::tuple<int, int, int>>{})
      .def(
          "run_slab",
          // One rank's z-slab (planes [z0, z0 + slab depth) of a `depth`-deep volume) through the
          // distributed 3D pipeline over `comm` (collective; volume_slabs.h). Seeds in volume
          // coordinates. Returns the slab's masks plus rounds / exchanged bytes.
          [](VolumeRunner& self, Comm& comm, py::array_t<uint16_t, py::array::c_style | py::array::forcecast> slab,
             int z0, int depth, const PipelineParams& p, int connectivity, int dilation,
             const std::vector<std::tuple<int, int, int>>& seeds) {
            SlabStats st;
            py::dict d = volume_call(slab, p, connectivity, dilation, seeds,
                                     [&](const VolumeInput& v, const VolumeParams& vp) {
                                       return self.run_slab(comm, v, z0, depth, vp, true, &st);
                                     });
            d["rounds"] = st.rounds;
            d["exchanged_bytes"] = st.exchanged_bytes;
            return d;
          },
          py::arg("comm"), py::arg("slab"), py::arg("z0"), py::arg("depth"), py::arg("params") = PipelineParams(),
          py::arg("connectivity") = 6, py::arg("dilation") = 7,
          py::arg("seeds") = std::vector<std::tuple<int, int, int>>{});

  // One-process rehearsal of the z-slab decomposition: `nranks` threads, each with its own
  // VolumeRunner (stream) on `device`, talking over loopback comms — the device-resident exchange
  // (Comm::sendrecv_device staged through pinned memory here) without the inter-process GPU
  // time-slicing that several rank processes on one GPU add. Runs `repeats` timed splits after one
  // warm-up; returns the wall times (max over ranks per split, seconds), the last split's rounds /
  // exchanged bytes per rank and its gathered masks.
  m.def(
      "run_volume_slabs_threads",
      [](py::array_t<uint16_t, py::array::c_style | py::array::forcecast> vol, int nranks, const PipelineParams& p,
         int connectivity, int dilation, int device, int repeats) {
        if (vol.ndim() != 3) throw std::invalid_argument("volume must be (depth, height, width)");
        const int D = (int)vol.shape(0), H = (int)vol.shape(1), W = (int)vol.shape(2);
        if (nranks < 1 || nranks > D) throw std::invalid_argument("1 <= nranks <= depth");
        const std::vector<uint16_t> raw = from_np<uint16_t>(vol);
        std::vector<VolumeInput> slabs((size_t)nranks);
        for (int r = 0; r < nranks; ++r) {
          const auto [z0, z1] = slab_bounds(D, r, nranks);
          VolumeInput& v = slabs[(size_t)r];
          v.w = W;
          v.h = H;
          v.d = z1 - z0;
          v.raw.assign(raw.begin() + (size_t)z0 * W * H, raw.begin() + (size_t)z1 * W * H);
        }
        VolumeParams vp;
        vp.pipe = p;
        vp.connectivity = connectivity;
        vp.dilation_size = dilation;
        std::vector<double> walls;
        std::vector<VolumeResult> res((size_t)nranks);
        std::vector<SlabStats> st((size_t)nranks);
        {
          py::gil_scoped_release nogil;
          std::vector<std::unique_ptr<VolumeRunner>> runners;
          for (int r = 0; r < nranks; ++r) runners.push_back(std::make_unique<VolumeRunner>(device));
          auto group = make_loopback_group(nranks);
          for (int rep = 0; rep <= repeats; ++rep) {
            const bool last = rep == repeats;
            std::vector<double> t((size_t)nranks);
            std::vector<std::string> err((size_t)nranks);
            std::vector<std::thread> th;
            for (int r = 0; r < nranks; ++r)
              th.emplace_back([&, r] {
                try {
                  const auto zz = slab_bounds(D, r, nranks);
                  group[(size_t)r]->barrier();
                  const auto t0 = std::chrono::steady_clock::now();
                  res[(size_t)r] = runners[(size_t)r]->run_slab(*group[(size_t)r], slabs[(size_t)r], zz.first, D, vp,
                                                                last, &st[(size_t)r]);
                  t[(size_t)r] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                } catch (const std::exception& e) {
                  err[(size_t)r] = e.what();
                }
              });
            for (auto& x : th) x.join();
            for (auto& e : err)
              if (!e.empty()) throw std::runtime_error("run_volume_slabs_threads: " + e);
            if (rep > 0) walls.push_back(*std::max_element(t.begin(), t.end()));
          }
        }
        py::dict d;
        d["walls_s"] = walls;
        std::vector<int> rounds;
        std::vector<int64_t> bytes;
        std::vector<uint8_t> region, dilated;
        for (int r = 0; r < nranks; ++r) {
          rounds.push_back(st[(size_t)r].rounds);
          bytes.push_back(st[(size_t)r].exchanged_bytes);
          region.insert(region.end(), res[(size_t)r].region.begin(), res[(size_t)r].region.end());
          dilated.insert(dilated.end(), res[(size_t)r].dilated.begin(), res[(size_t)r].dilated.end());
        }
        d["rounds"] = rounds;
        d["exchanged_bytes"] = bytes;
        d["region"] = to_np<uint8_t>(region, {D, H, W});
        d["dilated"] = to_np<uint8_t>(dilated, {D, H, W});
        return d;
      },
      py::arg("volume"), py::arg("nranks"), py::arg("params") = PipelineParams(), py::arg("connectivity") = 6,
      py::arg("dilation") = 7, py::arg("device") = 0, py::arg("repeats") = 5);

  // The same decomposition on the golden model: this rank's slab of a band volume (0/1 uint8,
  // planes [z0, z0 + d) of `depth`), seeds in volume coordinates. Collective over `comm`.
  m.def(
      "golden_volume_slab",
      [](Comm& comm, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> band, int z0, int depth,
         const std::vector<std::tuple<int, int, int>>& seeds, int connectivity, int dilation) {
        if (band.ndim() != 3) throw std::invalid_argument("band must be (depth, height, width)");
        const int d = (int)band.shape(0), h = (int)band.shape(1), w = (int)band.shape(2);
        GoldenSlabGrower g(from_np<uint8_t>(band), w, h, d, slab_seeds(seeds_from(seeds), w, h, depth, z0, d),
                           connectivity);
        SlabStats st;
        {
          py::gil_scoped_release nogil;
          st = grow_and_dilate_slabs(comm, g, w, h, depth, z0, z0 + d, connectivity, dilation);
        }
        py::dict r;
        r["region"] = to_np<uint8_t>(g.region(), {d, h, w});
        r["dilated"] = to_np<uint8_t>(g.dilated(), {d, h, w});
        r["rounds"] = st.rounds;
        r["exchanged_bytes"] = st.exchanged_bytes;
        return r;
      },
      py::arg("comm"), py::arg("band"), py::arg("z0"), py::arg("depth"), py::arg("seeds"), py::arg("connectivity") = 6,
      py::arg("dilation") = 7);
  // CPU self-test of the decomposition: `ranks` forked rank processes over the host comm (no HIP),
  // each growing its slab of `band` on the golden model; returns the reassembled (region,
  // dilated, rounds) — to compare with the single-volume golden result.
  m.def(
      "golden_slabs_selftest",
      [](int ranks, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> band,
         const std::vector<std::tuple<int, int, int>>& seeds, int connectivity, int dilation) {
        if (band.ndim() != 3) throw std::invalid_argument("band must be (depth, height, width)");
        const int D = (int)band.shape(0), h = (int)band.shape(1), w = (int)band.shape(2);
        const size_t vox = (size_t)D * h * w;
        const std::vector<uint8_t> b = from_np<uint8_t>(band);
        const std::vector<Seed> sd = seeds_from(seeds);
        // Results come back through a shared anonymous mapping made before the fork.
        void* map = mmap(nullptr, 2 * vox + 64, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
        if (map == MAP_FAILED) throw std::runtime_error("mmap failed");
        auto* out = static_cast<uint8_t*>(map);
        LaunchOptions o;
        o.comm = "host";
        o.timeout_s = 60;
        int rc;
        {
          py::gil_scoped_release nogil;
          rc = launch_ranks(ranks, [&](int rank, int size, Comm& c) {
            const auto [z0, z1] = slab_bounds(D, rank, size);
            const size_t plane = (size_t)w * h;
            GoldenSlabGrower g(std::vector<uint8_t>(b.begin() + (long)(z0 * plane), b.begin() + (long)(z1 * plane)), w, h,
                               z1 - z0, slab_seeds(sd, w, h, D, z0, z1 - z0), connectivity);
            const SlabStats st = grow_and_dilate_slabs(c, g, w, h, D, z0, z1, connectivity, dilation);
            std::memcpy(out + z0 * plane, g.region().data(), g.region().size());
            std::memcpy(out + vox + z0 * plane, g.dilated().data(), g.dilated().size());
            if (rank == 0) std::memcpy(out + 2 * vox, &st.rounds, sizeof(int));
            return 0;
          }, o);
        }
        std::vector<uint8_t> reg(out, out + vox), dil(out + vox, out + 2 * vox);
        int rounds = 0;
        std::memcpy(&rounds, out + 2 * vox, sizeof(int));
        munmap(map, 2 * vox + 64);
        if (rc != 0) throw std::runtime_error("golden_slabs_selftest: a rank failed with status " + std::to_string(rc));
        return py::make_tuple(to_np<uint8_t>(reg, {D, h, w}), to_np<uint8_t>(dil, {D, h, w}), rounds);
      },
      py::arg("ranks"), py::arg("band"), py::arg("seeds"), py::arg("connectivity") = 6, py::arg("dilation") = 7);

  // ---- raw-pointer kernel entry points (torch interop; all synchronous on `stream`) ----------------
  m.def("k_threshold", [](uintptr_t in, uintptr_t out, size_t n, float lo, float hi, uintptr_t stream) {
    hipStream_t st = as_stream(stream);
    gpu::launch_threshold((const float*)in, (uint8_t*)out, n, lo, hi, st);
    gpu::check_hip(hipStreamSynchronize(st), "k_threshold");
  });
  m.def("k_median", [](uintptr_t raw, uintptr_t out, int n, int h, int w, int k, const std::string& type, int stored_bits,
                       uintptr_t stream) {
    hipStream_t st = as_stream(stream);
    BatchTables t = upload_tables(n, h, w, parse_type(type), stored_bits, 1.f, 0.f, {}, st);
    gpu::launch_median((const uint16_t*)raw, (uint16_t*)out, t.desc, t.medt, t.nmed, k, t.stats, st);
    gpu::check_hip(hipStreamSynchronize(st), "k_median");
  });
  m.def("k_sharpen_band", [](uintptr_t med, uintptr_t band, uintptr_t sharp, int n, int h, int w, const std::string& type,
                             int stored_bits, float slope, float intercept, const PipelineParams& p, uintptr_t stream) {
    hipStream_t st = as_stream(stream);
    BatchTables t = upload_tables(n, h, w, parse_type(type), stored_bits, slope, intercept, {}, st);
    gpu::launch_sharpen_band((const uint16_t*)med, (uint64_t*)band, (float*)sharp, t.desc, t.shpt, t.nshp,
                             consts_from(p, 2), t.stats, st);
    gpu::check_hip(hipStreamSynchronize(st), "k_sharpen_band");
  });
  m.def("k_srg_morph", [](uintptr_t band, uintptr_t region, uintptr_t dilated, uintptr_t eroded, uintptr_t border_region,
                          int n, int h, int w, const std::vector<std::tuple<int, int, int>>& seeds, const PipelineParams& p,
                          int border_radius, uintptr_t stream) {
    hipStream_t st = as_stream(stream);
    BatchTables t = upload_tables(n, h, w, kU16, 16, 1.f, 0.f, seeds_from(seeds), st);
    gpu::SrgOutputs o;
    o.region = (uint64_t*)region;
    o.dilated = (uint64_t*)dilated;
    o.eroded = (uint64_t*)eroded;
    o.border_region = (uint64_t*)border_region;
    void* scr = nullptr;  // bit planes of slices above the LDS limit
    if (w > gpu::kSrgMaxDim || h > gpu::kSrgMaxDim) {
      gpu::check_hip(hipMalloc(&scr, (size_t)n * 4 * gpu::srg_plane_words(w, h) * 8), "hipMalloc srg scratch");
      o.scratch = (uint64_t*)scr;
    }
    try {
      gpu::launch_srg_morph((const uint64_t*)band, t.desc, n, t.seeds, consts_from(p, border_radius), o, w, h, st);
      gpu::check_hip(hipStreamSynchronize(st), "k_srg_morph");
    } catch (...) {
      if (scr) {
        (void)hipStreamSynchronize(st);
        (void)hipFree(scr);
      }
      throw;
    }
    if (scr) (void)hipFree(scr);
  });
  // 3D region growing on bit volumes [d][h][ceil(w/64)] (int64 words), continuing from the region
  // already present when reset is false; returns the sweep count. Synchronous on `stream`.
  m.def("k_srg3d", [](uintptr_t band, uintptr_t region, int w, int h, int d,
                      const std::vector<std::tuple<int, int, int>>& seeds, int connectivity, bool reset,
                      uintptr_t stream) {
    hipStream_t st = as_stream(stream);
    if (connectivity != 6 && connectivity != 26) throw std::invalid_argument("connectivity must be 6 or 26");
    std::vector<int32_t> sx;
    for (const auto& [x, y, z] : seeds) {
      sx.push_back(x);
      sx.push_back(y);
      sx.push_back(z);
    }
    int32_t* d_seeds = nullptr;
    uint32_t* d_flag = nullptr;
    uint32_t* h_flag = nullptr;
    uint64_t* scratch = nullptr;
    auto release = [&] {
      if (d_seeds) (void)hipFree(d_seeds);
      if (d_flag) (void)hipFree(d_flag);
      if (h_flag) (void)hipHostFree(h_flag);
      if (scratch) (void)hipFree(scratch);
    };
    try {
      gpu::check_hip(hipMalloc((void**)&d_flag, gpu::kSrg3dCtlWords * sizeof(uint32_t)), "hipMalloc flag");
      gpu::check_hip(hipHostMalloc((void**)&h_flag, gpu::kSrg3dCtlWords * sizeof(uint32_t), hipHostMallocDefault),
                     "hipHostMalloc flag");
      if (const size_t sw = gpu::srg3d_scratch_words(w, h, d))
        gpu::check_hip(hipMalloc((void**)&scratch, sw * 8), "hipMalloc srg3d scratch");
      if (!sx.empty()) {
        gpu::check_hip(hipMalloc((void**)&d_seeds, sx.size() * sizeof(int32_t)), "hipMalloc seeds");
        gpu::check_hip(hipMemcpyAsync(d_seeds, sx.data(), sx.size() * sizeof(int32_t), hipMemcpyHostToDevice, st),
                       "H2D seeds");
      }
      gpu::srg_volume((const uint64_t*)band, (uint64_t*)region, w, h, d, d_seeds, (int)(sx.size() / 3), connectivity,
                      d_flag, h_flag, scratch, st, reset);
      gpu::check_hip(hipStreamSynchronize(st), "k_srg3d");
      const int sweeps = gpu::srg_volume_result(h_flag);
      release();
      return sweeps;
    } catch (...) {
      (void)hipStreamSynchronize(st);
      release();
      throw;
    }
  });
  m.def("k_dilate3d", [](uintptr_t src, uintptr_t dst, uintptr_t tmp, int w, int h, int d, int size, uintptr_t stream,
                         bool ball) {
    hipStream_t st = as_stream(stream);
    if (size < 1 || !(size & 1)) throw std::invalid_argument("dilation size must be odd and >= 1");
    void* scr = nullptr;
    if (const size_t sw = gpu::morph3d_scratch_words(w, h, d))
      gpu::check_hip(hipMalloc(&scr, sw * 8), "hipMalloc morph scratch");
    try {
      gpu::dilate_volume((const uint64_t*)src, (uint64_t*)dst, (uint64_t*)tmp, w, h, d, size, st, (uint64_t*)scr, ball);
      gpu::check_hip(hipStreamSynchronize(st), "k_dilate3d");
    } catch (...) {
      (void)hipStreamSynchronize(st);
      if (scr) (void)hipFree(scr);
      throw;
    }
    if (scr) (void)hipFree(scr);
  }, py::arg("src"), py::arg("dst"), py::arg("tmp"), py::arg("w"), py::arg("h"), py::arg("d"), py::arg("size"),
     py::arg("stream"), py::arg("ball") = false);
  m.def("k_jpeg", [](uintptr_t canvas, int n, int h, int w, int quality, uintptr_t stream, int sampling) {
    hipStream_t st = as_stream(stream);
    const int blocks = (w / 8) * (h / 8);
    const uint32_t out_cap = 512 * 1024 + 64;
    std::vector<gpu::JpegDesc> jd(n);
    for (int i = 0; i < n; ++i) {
      std::memset(&jd[i], 0, sizeof(jd[i]));
      jd[i].canvas_off = (uint32_t)((size_t)i * w * h);
      jd[i].out_off = (uint64_t)i * out_cap;
      jd[i].out_cap = out_cap;
      jd[i].render = -1;
    }
    size_t off = 0;
    auto take = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) / 256 * 256;
      return o;
    };
    const size_t look_cap = (size_t)n * ((blocks + 255) / 256);
    const size_t o_jd = take(sizeof(gpu::JpegDesc) * n), o_look = take(6 * look_cap * 8), o_ticket = take(4 * (size_t)n),
                 o_spill = take(look_cap * 256 * 56 * 4), o_out = take((size_t)n * out_cap), o_sz = take((size_t)n * 4);
    uint8_t* dev = (uint8_t*)scratch().get(off);
    gpu::check_hip(hipMemcpyAsync(dev + o_jd, jd.data(), sizeof(gpu::JpegDesc) * n, hipMemcpyHostToDevice, st), "H2D");
    gpu::check_hip(hipMemsetAsync(dev + o_ticket, 0, 4 * (size_t)n, st), "memset tickets");
    gpu::check_hip(hipMemsetAsync(dev + o_look, 0, 6 * look_cap * 8, st), "memset look-back");
    gpu::JpegWork wk;
    wk.look = (uint64_t*)(dev + o_look);
    wk.look_cap = look_cap;
    wk.ticket = (uint32_t*)(dev + o_ticket);
    wk.spill = (uint32_t*)(dev + o_spill);
    int32_t divs[64];
    gpu::jpeg_divisors(quality, divs);
    gpu::launch_jpeg((const uint8_t*)canvas, (const gpu::JpegDesc*)(dev + o_jd), n, w, h, divs, wk, dev + o_out,
                     (int32_t*)(dev + o_sz), st, nullptr, sampling);
    std::vector<int32_t> sizes(n);
    gpu::check_hip(hipMemcpyAsync(sizes.data(), dev + o_sz, 4 * n, hipMemcpyDeviceToHost, st), "D2H");
    gpu::check_hip(hipStreamSynchronize(st), "k_jpeg");
    py::list res;
    for (int i = 0; i < n; ++i) {
      if (sizes[i] < 0) {
        res.append(py::none());
        continue;
      }
      std::string b((size_t)sizes[i], '\0');
      gpu::check_hip(hipMemcpy(b.data(), dev + o_out + (size_t)i * out_cap, sizes[i], hipMemcpyDeviceToHost), "D2H");
      res.append(py::bytes(b));
    }
    return res;
  }, py::arg("canvas"), py::arg("n"), py::arg("h"), py::arg("w"), py::arg("quality"), py::arg("stream"),
     py::arg("sampling") = 0);

  // ---- comm self-tests (CPU) ------------------------------------------------------------------------
  m.def("loopback_selftest", [](int n) {
    // Every rank contributes rank-dependent data; returns what rank 0 observed.
    auto group = make_loopback_group(n);
    std::vector<std::string> errors(n);
    std::vector<std::thread> th;
    for (int r = 0; r < n; ++r)
      th.emplace_back([&, r] {
        Comm& c = *group[r];
        try {
          std::vector<uint8_t> b;
          if (r == 0) b = {1, 2, 3, 4, 5};
          c.broadcast_bytes(b, 0);
          if (b != std::vector<uint8_t>{1, 2, 3, 4, 5}) errors[r] = "broadcast";
          std::vector<uint8_t> mine(r + 1, (uint8_t)r);
          auto all = c.allgather_bytes(mine);
          for (int q = 0; q < n; ++q)
            if (all[q] != std::vector<uint8_t>(q + 1, (uint8_t)q)) errors[r] = "allgather";
          int64_t v[2] = {r, 1};
          c.allreduce_sum_i64(v, 2);
          if (v[0] != (int64_t)n * (n - 1) / 2 || v[1] != n) errors[r] = "allreduce_sum";
          double f = r * 1.5;
          c.allreduce_max_f64(&f, 1);
          if (f != (n - 1) * 1.5) errors[r] = "allreduce_max";
          // ring neighbour exchange: send r+1 bytes up, receive r bytes from below (none at the ends)
          std::vector<uint8_t> up((size_t)r + 1, (uint8_t)(10 + r)), got((size_t)std::max(r, 0));
          c.sendrecv(up.data(), up.size(), r + 1 < n ? r + 1 : -1, got.data(), got.size(), r > 0 ? r - 1 : -1);
          if (r > 0 && got != std::vector<uint8_t>((size_t)r, (uint8_t)(9 + r))) errors[r] = "sendrecv";
          c.barrier();
        } catch (const std::exception& e) {
          errors[r] = e.what();
        }
      });
    for (auto& t : th) t.join();
    return errors;
  });
  m.def(
      "launcher_selftest",
      // Forks n rank processes over the host comm (no RCCL, no HIP): every rank checks the
      // collectives, then `mode` decides the ending — "ok": all succeed; "exit": the last rank
      // (n > 2) returns 7 after the collectives; "die": the last rank exits 3 while the others
      // block in a barrier (abort flag); "hang": the last rank sleeps while the others wait in
      // a barrier (deadline, then SIGTERM from the supervisor). Returns the job's exit status.
      // comm "rccl": the ranks get launch_ranks' deferred RCCL communicator; after the collectives each
      // starts RCCL and promotes — without a GPU every rank fails to bring RCCL up, they agree on it
      // and the last collectives run on the control plane.
      [](int n, const std::string& mode, double timeout_s, double grace_s, const std::string& comm) {
        LaunchOptions o;
        o.comm = comm;
        o.timeout_s = timeout_s;
        o.grace_s = grace_s;
        py::gil_scoped_release nogil;
        return launch_ranks(
            n,
            [mode](int rank, int size, Comm& c) {
              std::vector<uint8_t> b;
              if (rank == 0) b.assign(3 << 20, 0);  // larger than a slot: chunked broadcast
              for (size_t i = 0; i < b.size(); ++i) b[i] = (uint8_t)(i * 7 + 1);
              c.broadcast_bytes(b, 0);
              for (size_t i = 0; i < b.size(); i += 4099)
                if (b[i] != (uint8_t)(i * 7 + 1)) return 11;
              if (b.size() != (3u << 20)) return 12;
              auto all = c.allgather_bytes(std::vector<uint8_t>(rank + 1, (uint8_t)rank));
              for (int q = 0; q < size; ++q)
                if (all[q] != std::vector<uint8_t>(q + 1, (uint8_t)q)) return 13;
              int64_t v[2] = {rank, 1};
              c.allreduce_sum_i64(v, 2);
              if (v[0] != (int64_t)size * (size - 1) / 2 || v[1] != size) return 14;
              double f = rank * 1.5;
              c.allreduce_max_f64(&f, 1);
              if (f != (size - 1) * 1.5) return 15;
              // neighbour exchange larger than a slot (chunked): rank r sends to r + 1
              const size_t big = (2u << 20) + 777;
              std::vector<uint8_t> snd(big), rcv(rank > 0 ? big : 0);
              for (size_t i = 0; i < big; ++i) snd[i] = (uint8_t)(i * 13 + rank);
              c.sendrecv(snd.data(), big, rank + 1 < size ? rank + 1 : -1, rcv.data(), rcv.size(), rank > 0 ? rank - 1 : -1);
              for (size_t i = 0; i < rcv.size(); i += 4097)
                if (rcv[i] != (uint8_t)(i * 13 + rank - 1)) return 16;
              const bool last = rank == size - 1;
              if (mode == "exit" && last && size > 2) return 7;
              if (mode == "die" && last) _exit(3);
              if (mode == "hang" && last) {
                std::this_thread::sleep_for(std::chrono::seconds(600));
                return 0;
              }
              c.start_data_plane();
              c.promote();  // ranks on different planes afterwards would hang the next collective
              int64_t one = 1;
              c.allreduce_sum_i64(&one, 1);
              if (one != size) return 18;
              c.barrier();
              return 0;
            },
            o);
      },
      py::arg("n"), py::arg("mode") = "exit", py::arg("timeout_s") = -1.0, py::arg("grace_s") = 5.0,
      py::arg("comm") = "host");

  // ---- native communicators (bench.py and other Python drivers) ------------------------------------
  // Host/RCCL comms for ranks started by torchrun or bench.py's own launcher; the rendezvous
  // (segment name or RCCL unique id) travels through the caller's store.
  py::class_<ShmSegment, std::shared_ptr<ShmSegment>>(m, "ShmSegment")
      .def_property_readonly("size", &ShmSegment::size)
      .def("wait_attached_and_unlink", [](ShmSegment& s, double t) {
        py::gil_scoped_release nogil;
        s.wait_attached_and_unlink(t);
      }, py::arg("timeout_s") = 120.0)
      .def("raise_abort", &ShmSegment::raise_abort)
      .def_property_readonly("aborted", &ShmSegment::aborted);
  m.def("shm_create", [](int n, std::string name) {
    auto s = ShmSegment::create_named(n, &name);
    return py::make_tuple(s, name);
  }, py::arg("n"), py::arg("name") = std::string());
  m.def("shm_attach", [](const std::string& name, int n, double t) {
    py::gil_scoped_release nogil;
    return ShmSegment::attach_named(name, n, t);
  }, py::arg("name"), py::arg("n"), py::arg("timeout_s") = 120.0);
  py::class_<Comm, std::unique_ptr<Comm>>(m, "Comm")
      .def_property_readonly("rank", &Comm::rank)
      .def_property_readonly("size", &Comm::size)
      .def_property_readonly("backend", [](const Comm& c) { return std::string(c.backend()); })
      .def("barrier", [](Comm& c) {
        py::gil_scoped_release nogil;
        c.barrier();
      })
      .def("broadcast_bytes", [](Comm& c, py::bytes data, int root) {
        std::string s = data;
        std::vector<uint8_t> v(s.begin(), s.end());
        {
          py::gil_scoped_release nogil;
          c.broadcast_bytes(v, root);
        }
        return py::bytes((const char*)v.data(), v.size());
      }, py::arg("data"), py::arg("root") = 0)
      .def("allgather_bytes", [](Comm& c, py::bytes data) {
        std::string s = data;
        std::vector<std::vector<uint8_t>> all;
        {
          py::gil_scoped_release nogil;
          all = c.allgather_bytes(std::vector<uint8_t>(s.begin(), s.end()));
        }
        py::list out;
        for (auto& v : all) out.append(py::bytes((const char*)v.data(), v.size()));
        return out;
      })
      .def("allreduce_sum", [](Comm& c, std::vector<int64_t> v) {
        py::gil_scoped_release nogil;
        c.allreduce_sum_i64(v.data(), v.size());
        return v;
      })
      .def("allreduce_max", [](Comm& c, std::vector<double> v) {
        py::gil_scoped_release nogil;
        c.allreduce_max_f64(v.data(), v.size());
        return v;
      })
      .def("start_data_plane", [](Comm& c) {
        py::gil_scoped_release nogil;
        c.start_data_plane();
      })
      .def("settle_data_plane", [](Comm& c) {
        py::gil_scoped_release nogil;
        c.settle_data_plane(nullptr);
      })
      .def("fail_data_plane", [](Comm& c, const std::string& why) { c.fail_data_plane(why); }, py::arg("why"))
      .def("promote", [](Comm& c) {
        py::gil_scoped_release nogil;
        c.promote();
      })
      .def_property_readonly("data_plane_times", [](const Comm& c) {
        const Comm::DataPlaneTimes t = c.data_plane_times();
        py::dict d;
        d["start_s"] = t.start_s;
        d["settle_s"] = t.settle_s;
        d["wait_s"] = t.wait_s;
        d["init_upper_s"] = t.init_upper_s;
        return d;
      })
      .def_property_readonly("fallback_error", &Comm::fallback_error)
      .def_property_readonly("transport_size", &Comm::transport_size)
      .def_property_readonly("transport_rank", &Comm::transport_rank)
      .def_property_readonly("transport_device", &Comm::transport_device)
      .def("set_abort_segment", &Comm::set_abort_segment, py::arg("segment"))
      .def("sendrecv", [](Comm& c, py::bytes data, int dst, size_t rbytes, int src) {
        std::string s = data;
        std::string out(rbytes, '\0');
        {
          py::gil_scoped_release nogil;
          c.sendrecv(s.data(), s.size(), dst, out.data(), rbytes, src);
        }
        return py::bytes(out);
      }, py::arg("data"), py::arg("dst"), py::arg("rbytes"), py::arg("src"))
      .def("gather_rank_devices", [](Comm& c, int device, const std::string& bus_id, int node, const std::string& cpus,
                                     int threads, const std::string& error) {
        RankDevice me;
        me.device = device;
        me.bus_id = bus_id;
        me.node = node;
        me.cpus = cpus;
        me.threads = threads;
        me.transport_size = c.transport_size();
        me.transport_device = c.transport_device();
        me.error = error;
        std::vector<RankDevice> all;
        {
          py::gil_scoped_release nogil;
          all = gather_rank_devices(c, me);
        }
        py::list out;
        for (const auto& d : all) {
          py::dict x;
          x["device"] = d.device;
          x["bus_id"] = d.bus_id;
          x["numa_node"] = d.node;
          x["cpus"] = d.cpus;
          x["threads"] = d.threads;
          x["transport_size"] = d.transport_size;
          x["transport_device"] = d.transport_device;
          x["error"] = d.error;
          out.append(x);
        }
        return out;
      }, py::arg("device"), py::arg("bus_id"), py::arg("node"), py::arg("cpus"), py::arg("threads"),
         py::arg("error") = "")
      .def("allgather_f64", [](Comm& c, std::vector<double> v) {
        std::vector<double> all(v.size() * (size_t)c.size());
        {
          py::gil_scoped_release nogil;
          c.allgather(v.data(), v.size() * sizeof(double), all.data());
        }
        return all;
      });
  m.def("self_comm", &make_self_comm);
  m.def("host_comm", [](std::shared_ptr<ShmSegment> seg, int rank, double t) { return make_host_comm(seg, rank, t); },
        py::arg("segment"), py::arg("rank"), py::arg("timeout_s") = -1.0);
  m.def("rccl_unique_id", [] {
    auto v = rccl_unique_id();
    return py::bytes((const char*)v.data(), v.size());
  });
  m.def("rccl_comm", [](int rank, int size, py::bytes uid, int device, std::shared_ptr<ShmSegment> seg, double t) {
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    py::gil_scoped_release nogil;
    return make_rccl_comm(rank, size, v, device, seg, t);
  }, py::arg("rank"), py::arg("size"), py::arg("unique_id"), py::arg("device"), py::arg("segment") = nullptr,
     py::arg("timeout_s") = -1.0);
  m.def("deferred_rccl_comm", [](int rank, int size, int device, std::shared_ptr<ShmSegment> seg, double t) {
    return make_deferred_rccl_comm(rank, size, device, std::move(seg), t);
  }, py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("segment"), py::arg("timeout_s") = -1.0);
  m.def("comm_timeout_s", &comm_timeout_s);
  py::register_exception<CommError>(m, "CommError", PyExc_RuntimeError);
}
