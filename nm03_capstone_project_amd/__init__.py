"""NM03 on MI355X — a brand-new MI355X-native DICOM batch-processing engine with the capabilities
of calebhabesh/NM03-Capstone-Project (reference @ /root/reference).

Layers:
  native core (C++/HIP, gfx950): DICOM + JPEG codecs, golden CPU model, fused HIP kernels K1–K5,
      batch engine (pinned blob uploads, per-slot streams, host-mapped JPEG output), RCCL comm,
      the three reference CLIs (build/bin/test_pipeline, img_processing_sequential,
      img_processing_parallel)
  models/    the per-slice pipeline (2D) and the volume pipeline (3D) as Python objects
  ops/       torch-tensor entry points of every HIP kernel + plain-PyTorch fp32 references
  parallel/  native communicators (RCCL over xGMI / host), sharding, cohort plans, z-slab volumes
  utils/     DICOM/JPEG/cohort helpers and the synthetic T1+C cohort generator
"""
from ._native import native, available  # noqa: F401
from .models.pipeline import SlicePipeline, PipelineConfig  # noqa: F401
from .models.volume import VolumePipeline  # noqa: F401
from . import ops, parallel, utils  # noqa: F401,E402

__version__ = "0.1.0"
