"""Pipelines ("models") of the framework: the reference's per-slice 2D pipeline and the 3D mode."""
from .pipeline import PipelineConfig, SlicePipeline  # noqa: F401
from .volume import VolumePipeline  # noqa: F401
