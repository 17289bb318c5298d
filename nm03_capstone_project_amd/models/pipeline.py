"""The per-slice pipeline of the reference as a model object.

Stages (reference main_sequential.cpp:175-262 / test_pipeline.cpp:33-125):
  import → IntensityNormalization(0.5, 2.5, 0, 10000) → IntensityClipping(0.68, 4000)
  → VectorMedianFilter(7) → ImageSharpening(2.0, 0.5, 9) → SeededRegionGrowing(0.74, 0.91, 41 seeds)
  → ImageCaster(UINT8) → Dilation(3) [+ Erosion(3) in test_pipeline]
  → RenderToImage 512² (ImageRenderer / SegmentationRenderer(0.6, 1.0, 2)) → JPEG q75.

`SlicePipeline.run_*` executes every stage on the MI355X through the native engine (K1..K4);
`SlicePipeline.golden` runs the single-threaded CPU golden model of the same contract.
"""
from dataclasses import asdict, dataclass, fields

from .._native import native


@dataclass
class PipelineConfig:
    # pipeline literals
    norm_low: float = 0.5
    norm_high: float = 2.5
    norm_min: float = 0.0
    norm_max: float = 10000.0
    clip_min: float = 0.68
    clip_max: float = 4000.0
    median_window: int = 7
    sharpen_gain: float = 2.0
    sharpen_sigma: float = 0.5
    sharpen_mask: int = 9
    srg_min: float = 0.74
    srg_max: float = 0.91
    srg_connectivity: int = 4
    dilation_size: int = 3
    erosion_size: int = 3
    min_dim: int = 100
    apply_rescale: bool = True
    se_shape: int = 0  # structuring element of dilation/erosion: 0 square (default), 1 disc (params.h SeShape)
    frame: int = -1  # multi-frame DICOM: -1 rejects such files, k >= 0 imports frame k (dicom.h select_frame)
    # render / export
    out_width: int = 512
    out_height: int = 512
    label_opacity: float = 0.6
    border_opacity: float = 1.0
    border_radius: int = 2
    jpeg_quality: int = 75
    render_filter: int = 0  # gray renders: 0 bilinear (default), 1 nearest (params.h RenderFilter)
    jpeg_sampling: int = 0  # JPEG files: 0 YCbCr 4:2:0 (default), 1 YCbCr 4:4:4, 2 one gray component
    # engine
    batch_size: int = 25
    streams: int = 3
    threads: int = 16
    max_dim: int = 512
    device: int = 0
    export_jpeg: bool = True
    resume: bool = False
    host_only: bool = False  # host path only, no GPU (loads + JPEG writes with fixed segments, engine.h)

    _PIPE = ("norm_low", "norm_high", "norm_min", "norm_max", "clip_min", "clip_max", "median_window",
             "sharpen_gain", "sharpen_sigma", "sharpen_mask", "srg_min", "srg_max", "srg_connectivity",
             "dilation_size", "erosion_size", "min_dim", "apply_rescale", "frame", "se_shape")
    _RENDER = ("out_width", "out_height", "label_opacity", "border_opacity", "border_radius", "jpeg_quality",
               "jpeg_sampling")

    def pipeline_params(self):
        p = native().PipelineParams()
        for k in self._PIPE:
            setattr(p, k, getattr(self, k))
        return p

    def render_params(self):
        r = native().RenderParams()
        for k in self._RENDER:
            setattr(r, k, getattr(self, k))
        r.filter = self.render_filter
        return r

    def engine_config(self):
        c = native().EngineConfig()
        c.device = self.device
        c.batch_size = self.batch_size
        c.streams = self.streams
        c.threads = self.threads
        c.max_dim = self.max_dim
        c.pipe = self.pipeline_params()
        c.render = self.render_params()
        c.export_jpeg = self.export_jpeg
        c.resume = self.resume
        c.host_only = self.host_only
        return c

    def replace(self, **kw):
        d = {f.name: getattr(self, f.name) for f in fields(self)}
        d.update(kw)
        return PipelineConfig(**d)

    def to_dict(self):
        return asdict(self)


STATUS_NAMES = {0: "ok", 1: "load_error", 2: "too_small", 3: "device_error", 4: "export_error", 5: "not_run"}


class SlicePipeline:
    """2D pipeline bound to one GPU (lazily creates the native Engine)."""

    def __init__(self, config: PipelineConfig = None):
        self.config = config or PipelineConfig()
        self._engine = None

    @property
    def engine(self):
        if self._engine is None:
            self._engine = native().Engine(self.config.engine_config())
        return self._engine

    # -- GPU ---------------------------------------------------------------------------------------
    def run_array(self, raw, meta=None):
        """All stage outputs of one slice (uint16 raw [H, W]) computed on the GPU."""
        meta = meta or {}
        return self.engine.run_single(raw, meta.get("type", "u16"), int(meta.get("stored_bits", 16)),
                                      float(meta.get("slope", 1.0)), float(meta.get("intercept", 0.0)),
                                      float(meta.get("spacing_x", 1.0)), float(meta.get("spacing_y", 1.0)))

    def run_file(self, path):
        raw, meta = native().read_slice(path, 0)
        return self.run_array(raw, meta)

    def process(self, items):
        """Batch-process [(dicom_path, out_dir), ...] → (statuses, stage_times)."""
        return self.engine.run(list(items))

    # -- CPU golden model ------------------------------------------------------------------------
    def golden(self, raw, meta=None):
        meta = meta or {}
        return native().golden_run(raw, meta.get("type", "u16"), int(meta.get("stored_bits", 16)),
                                   float(meta.get("slope", 1.0)), float(meta.get("intercept", 0.0)),
                                   self.config.pipeline_params(), self.config.render_params(),
                                   float(meta.get("spacing_x", 1.0)), float(meta.get("spacing_y", 1.0)))

    def seeds(self, width, height):
        return native().reference_seeds(width, height)
