"""Z-slab domain decomposition of ONE 3D volume across ranks — the spatial analogue of context
parallelism for this workload. The reference has no 3D path at all (it forces 2D with
`setLoadSeries(false)`, test_pipeline.cpp:38-41) and no multi-process anything.

Everything runs in native code (include/nm03/volume_slabs.h, src/runtime/volume_slabs.cpp) over a
native `Comm` (parallel/native_comm.py: RCCL over xGMI, or the host comm when ranks share a GPU):

1. per-plane preprocessing (median → sharpen → band) is in-plane only: no halo;
2. seeded region growing is a global fixpoint — local fixpoints on each slab (K5: one cooperative
   launch, convergence on the device), then the two bit-packed boundary region planes go to the
   neighbours (Comm.sendrecv = grouped ncclSend/ncclRecv) and the in-band voxels touching the
   neighbour's region are added; an all-reduce of the additions decides another round;
3. cube dilation of size s takes r = s // 2 halo planes from each side (sendrecv; all-gather when a
   slab is thinner than r), dilates slab + halo and drops the halo.

The CLI form is `img_processing_parallel --mode 3d --split-volume --gpus N`."""
import numpy as np

from .._native import native
from .dist import shard_bounds


def slab_bounds(depth, rank, world):
    """Planes [z0, z1) of `rank`: contiguous, ±1 plane."""
    return shard_bounds(depth, rank, world)


def _self():
    return native().self_comm()


def _gather(comm, arr, depth):
    """All-gather every rank's slab of a [d, H, W] uint8 mask into the [depth, H, W] volume."""
    parts = comm.allgather_bytes(np.ascontiguousarray(arr, dtype=np.uint8).tobytes())
    h, w = arr.shape[1:]
    return np.concatenate([np.frombuffer(p, np.uint8).reshape(-1, h, w) for p in parts])[:depth]


def run_volume_slabs(volume=None, comm=None, config=None, connectivity=6, dilation=7, seeds=None, band=None,
                     backend="gpu", gather=False, device=0, runner=None):
    """This rank's slab of the 3D pipeline, collectively over `comm` (None: a single rank).

    backend "gpu": `volume` (uint16 [D, H, W], the whole volume or only this rank's slab with
    `depth`-sized first axis… pass the whole volume) through VolumeRunner.run_slab on `device`.
    backend "cpu": `band` (0/1 uint8 [D, H, W]) through the golden model (hosts without a GPU).
    Seeds are in volume coordinates (default: the reference pattern on plane D // 2). Returns a dict
    with this rank's "z0", "z1", "region", "dilated" (and "band" on the GPU), "rounds" and
    "exchanged_bytes"; gather=True replaces the masks by the whole volume's."""
    comm = comm or _self()
    src = volume if backend == "gpu" else band
    if src is None:
        raise ValueError("run_volume_slabs: backend 'gpu' needs volume=, 'cpu' needs band=")
    depth = int(src.shape[0])
    z0, z1 = slab_bounds(depth, comm.rank, comm.size)
    s = [tuple(int(c) for c in p) for p in (seeds or [])]
    if backend == "gpu":
        from ..models.pipeline import PipelineConfig
        params = (config or PipelineConfig()).pipeline_params()
        runner = runner or native().VolumeRunner(device)
        slab = np.ascontiguousarray(volume[z0:z1], dtype=np.uint16)
        r = dict(runner.run_slab(comm, slab, z0, depth, params, connectivity, dilation, s))
    elif backend == "cpu":
        b = np.ascontiguousarray(band[z0:z1], dtype=np.uint8)
        r = dict(native().golden_volume_slab(comm, b, z0, depth, s, connectivity, dilation))
    else:
        raise ValueError(f"unknown backend {backend!r} (gpu | cpu)")
    r.update(z0=z0, z1=z1)
    if gather:
        for k in ("band", "region", "dilated"):
            if k in r:
                r[k] = _gather(comm, r[k], depth)
    return r
