"""3D mode (BASELINE config 5): a series as one volume, per-slice median/sharpen/band, 6- or
26-connected seeded region growing by LDS plane sweeps, and separable cube dilation."""
import numpy as np

from .._native import native
from .pipeline import PipelineConfig


class VolumePipeline:
    def __init__(self, config: PipelineConfig = None, connectivity: int = 6, dilation: int = 7):
        self.config = config or PipelineConfig()
        self.connectivity = connectivity
        self.dilation = dilation
        self._runners = {}  # device -> native VolumeRunner (buffers/stream reused across volumes)

    def default_seeds(self, volume):
        d, h, w = volume.shape
        return [(x, y, d // 2) for (x, y) in native().reference_seeds(w, h)]

    def run(self, volume, seeds=None, device=None):
        vol = np.ascontiguousarray(volume, dtype=np.uint16)
        s = list(seeds) if seeds is not None else self.default_seeds(vol)
        dev = self.config.device if device is None else device
        runner = self._runners.get(dev)
        if runner is None:
            runner = self._runners[dev] = native().VolumeRunner(dev)
        return runner.run(vol, self.config.pipeline_params(), self.connectivity, self.dilation, s)

    def run_series(self, series_dir, seeds=None, device=None):
        """A DICOM series directory as one volume (utils.read_series: the reference's file-number
        order, every slice of one shape) through `run`."""
        from ..utils.dicom import read_series
        vol, _ = read_series(series_dir)
        return self.run(vol, seeds=seeds, device=device)

    def run_slabs(self, volume=None, comm=None, seeds=None, band=None, backend="gpu", gather=True, device=None):
        """The same pipeline on a volume split into z-slabs over the ranks of the native `comm` (one
        process per GPU; parallel/volume_slabs.py). Returns the whole volume's masks on every rank
        with gather=True, else this rank's slab."""
        from ..parallel.volume_slabs import run_volume_slabs
        dev = self.config.device if device is None else device
        runner = None
        if backend == "gpu":
            runner = self._runners.get(dev)
            if runner is None:
                runner = self._runners[dev] = native().VolumeRunner(dev)
        return run_volume_slabs(volume=volume, comm=comm, config=self.config, connectivity=self.connectivity,
                                dilation=self.dilation, seeds=seeds, band=band, backend=backend, gather=gather,
                                device=dev, runner=runner)

    def golden(self, band, seeds):
        n = native()
        region = n.golden_region_grow3d(band, list(seeds), self.connectivity)
        return region, n.golden_dilate3d(region, self.dilation, self.config.se_shape == 1)
