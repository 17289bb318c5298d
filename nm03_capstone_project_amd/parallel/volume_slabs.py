"""Z-slab domain decomposition of ONE 3D volume across ranks — the spatial analogue of context
parallelism for this workload. The reference has no 3D path at all (it forces 2D with
`setLoadSeries(false)`, test_pipeline.cpp:38-41) and no multi-process anything; the 3D mode of this
framework (BASELINE config 5, `VolumePipeline`) fits a 256³ volume on one MI355X with room to spare,
so this decomposition is for volumes — or volume stacks — that should be split over GPUs.

Rank r owns planes [z0, z1) = shard_bounds(D, r, W) (contiguous, ±1 plane):

1. per-plane preprocessing (median → sharpen → band) is in-plane only: no halo;
2. seeded region growing is a global fixpoint: every rank grows its slab to a local fixpoint (K5
   plane sweeps, `ops.region_grow3d`), then the ranks exchange their two boundary region planes
   (one all-gather of [2, H, W] per round) and add the voxels of their own boundary planes that are
   in band and touch the neighbour's region (6-connectivity: the voxel across the boundary;
   26-connectivity: its 3×3 in-plane neighbourhood). Rounds repeat until no rank adds a voxel
   (all-reduce max). The union of the slab regions is then the region a single-GPU run grows: it
   contains the seeds, is closed under in-band adjacency inside slabs (local fixpoints) and across
   slab boundaries (the final round added nothing), and every voxel was reached along an in-band
   path;
3. cube dilation of size s needs r = s // 2 halo planes from each neighbour: one all-gather of
   [2r, H, W], then the slab plus halo is dilated and the halo rows are dropped (out-of-volume
   samples are ignored, like the single-volume kernel).

Collectives go through torch.distributed — RCCL over xGMI on MI355X (backend "nccl"), gloo on CPU.
Boundary traffic is O(H·W) per round, independent of the slab depth.

Backends: "gpu" runs the HIP kernels on the rank's device; "cpu" runs the golden C++ model (tests
and hosts without a GPU; same results bit for bit)."""
import numpy as np
import torch
import torch.distributed as dist

from .._native import native
from .dist import _active, _dev, allreduce_max, shard_bounds


def _dilate_plane3(m):
    """3×3 in-plane dilation of a bool [H, W] tensor (26-connected boundary seeding)."""
    f = m.to(torch.float32)[None, None]
    return torch.nn.functional.max_pool2d(f, 3, stride=1, padding=1)[0, 0] > 0


def _allgather(t, ctx):
    """All-gather an equally shaped uint8 tensor from every rank → [world, *t.shape] on t.device."""
    if not _active():
        return t.unsqueeze(0)
    dev = _dev(ctx)
    src = t.to(torch.uint8).to(dev).contiguous()
    out = [torch.empty_like(src) for _ in range(dist.get_world_size())]
    dist.all_gather(out, src)
    return torch.stack(out).to(t.device)


class _GpuBackend:
    def __init__(self, device):
        self.device = device

    def band(self, planes, config, pixel_type, stored_bits, slope, intercept):
        from ..ops import median2d, sharpen_band
        raw = torch.from_numpy(np.ascontiguousarray(planes).view(np.int16)).to(self.device)
        med = median2d(raw, config.median_window, pixel_type, stored_bits)
        _, b = sharpen_band(med, config, pixel_type, stored_bits, slope, intercept, want_sharpened=False)
        return b

    def grow(self, band, region, seeds, conn):
        from ..ops import region_grow3d
        return region_grow3d(band, seeds, conn, region)

    def dilate(self, mask, size):
        from ..ops import dilate3d
        return dilate3d(mask, size)


class _CpuBackend:
    device = torch.device("cpu")

    def band(self, planes, config, pixel_type, stored_bits, slope, intercept):
        n = native()
        pp, rp = config.pipeline_params(), config.render_params()
        out = [n.golden_run(np.ascontiguousarray(p), pixel_type, stored_bits, slope, intercept, pp, rp, 1.0, 1.0)["band"]
               for p in planes]
        return torch.from_numpy(np.stack(out).astype(bool))

    def grow(self, band, region, seeds, conn):
        # Growing from region ∪ seeds equals continuing the growth of `region` (region ⊆ band).
        s = list(seeds)
        if region is not None:
            z, y, x = np.nonzero(region.numpy())
            s += list(zip(x.tolist(), y.tolist(), z.tolist()))
        r = native().golden_region_grow3d(band.numpy().astype(np.uint8), s, conn)
        return torch.from_numpy(r.astype(bool)), 0

    def dilate(self, mask, size):
        return torch.from_numpy(native().golden_dilate3d(mask.numpy().astype(np.uint8), size).astype(bool))


def _backend(kind, device):
    if kind == "auto":
        kind = "gpu" if (device is not None and torch.device(device).type == "cuda") else "cpu"
    return _GpuBackend(torch.device(device)) if kind == "gpu" else _CpuBackend()


def grow_slabs(band, z0, seeds, ctx=None, connectivity=6, backend="cpu", device=None, max_rounds=100000):
    """Global 3D region growing over z-slabs. `band`: this rank's bool [dl, H, W] planes starting
    at global plane z0; `seeds`: global (x, y, z) voxels (each rank keeps its own). Returns
    (region bool [dl, H, W], rounds, local sweeps)."""
    be = backend if not isinstance(backend, str) else _backend(backend, device)
    dl = band.shape[0]
    rank = dist.get_rank() if _active() else 0
    world = dist.get_world_size() if _active() else 1
    # Every slab needs a plane (edge planes are exchanged): agreed collectively, so all ranks raise
    # together instead of one rank failing while its peers wait in the all-gather.
    if world > 1 and -allreduce_max(-float(dl), ctx) < 1:
        raise ValueError("grow_slabs: every rank needs at least one plane (depth < world size)")
    mine = [(int(x), int(y), int(z) - z0) for (x, y, z) in seeds if z0 <= int(z) < z0 + dl]
    region, sweeps = be.grow(band, None, mine, connectivity)
    rounds = 1
    while rounds < max_rounds:
        edges = _allgather(torch.stack([region[0], region[-1]]), ctx).bool()
        add_lo = add_hi = None
        if rank > 0:
            nb = edges[rank - 1, 1]
            nb = _dilate_plane3(nb) if connectivity == 26 else nb
            add_lo = band[0] & nb & ~region[0]
        if rank < world - 1:
            nb = edges[rank + 1, 0]
            nb = _dilate_plane3(nb) if connectivity == 26 else nb
            add_hi = band[-1] & nb & ~region[-1]
        grew = bool((add_lo is not None and add_lo.any()) or (add_hi is not None and add_hi.any()))
        if not allreduce_max(1.0 if grew else 0.0, ctx):
            break
        rounds += 1
        if grew:
            region = region.clone()
            if add_lo is not None:
                region[0] |= add_lo
            if add_hi is not None:
                region[-1] |= add_hi
            region, s = be.grow(band, region, [], connectivity)
            sweeps += s
    return region, rounds, sweeps


def dilate_slabs(region, size, ctx=None, backend="cpu", device=None):
    """Cube dilation (size³) of a z-slab decomposed mask with an r = size // 2 plane halo exchange.
    Every slab must have at least r planes."""
    be = backend if not isinstance(backend, str) else _backend(backend, device)
    r = size // 2
    if r == 0:
        return region.clone()
    dl = region.shape[0]
    rank = dist.get_rank() if _active() else 0
    world = dist.get_world_size() if _active() else 1
    if world > 1:
        if -allreduce_max(-float(dl), ctx) < r:
            raise ValueError(f"dilate_slabs: every slab needs >= {r} planes for a {size}^3 dilation")
        halo = _allgather(torch.cat([region[:r], region[-r:]]), ctx).bool()
    parts, lo = [], 0
    if rank > 0:
        parts.append(halo[rank - 1, r:])
        lo = r
    parts.append(region)
    if rank < world - 1:
        parts.append(halo[rank + 1, :r])
    dil = be.dilate(torch.cat(parts).contiguous(), size)
    return dil[lo:lo + dl]


def gather_slabs(local, depth, ctx=None):
    """Reassemble [D, H, W] from every rank's slab (on all ranks): slabs are padded to the
    largest depth for one all-gather, then trimmed by shard_bounds."""
    if not _active():
        return local
    world = dist.get_world_size()
    dmax = max(shard_bounds(depth, r, world)[1] - shard_bounds(depth, r, world)[0] for r in range(world))
    pad = torch.zeros((dmax,) + tuple(local.shape[1:]), dtype=torch.uint8, device=local.device)
    pad[:local.shape[0]] = local.to(torch.uint8)
    allp = _allgather(pad, ctx)
    out = [allp[r, :shard_bounds(depth, r, world)[1] - shard_bounds(depth, r, world)[0]] for r in range(world)]
    return torch.cat(out).to(local.dtype)


def run_volume_slabs(volume=None, ctx=None, config=None, connectivity=6, dilation=7, seeds=None, band=None,
                     pixel_type="u16", stored_bits=16, slope=1.0, intercept=0.0, backend="auto", gather=False):
    """The 3D pipeline (per-plane median/sharpen/band → 3D SRG → cube dilation) on this rank's
    z-slab. Pass the raw `volume` ([D, H, W] u16; an np.memmap is read only for this rank's planes)
    or a precomputed bool `band` of the same shape. Default seeds: the reference seed pattern on the
    middle plane (like VolumePipeline). Returns dict(z0, band, region, dilated, rounds, sweeps) with
    this rank's [z1 - z0, H, W] masks, or the full [D, H, W] masks on every rank with gather=True."""
    from ..models.pipeline import PipelineConfig
    if (volume is None) == (band is None):
        raise ValueError("pass exactly one of volume / band")
    cfg = config or PipelineConfig()
    rank = dist.get_rank() if _active() else 0
    world = dist.get_world_size() if _active() else 1
    depth, h, w = (volume if volume is not None else band).shape
    if depth < world:  # same shape on every rank: all raise together, before any collective
        raise ValueError(f"run_volume_slabs: depth {depth} < {world} ranks leaves empty slabs")
    z0, z1 = shard_bounds(depth, rank, world)
    device = ctx.device if (ctx is not None and ctx.device is not None) else None
    be = _backend(backend, device)
    if volume is not None:
        band_l = be.band(np.asarray(volume[z0:z1]), cfg, pixel_type, stored_bits, slope, intercept)
    else:
        band_l = torch.as_tensor(np.asarray(band[z0:z1])).bool().to(be.device)
    if seeds is None:
        seeds = [(x, y, depth // 2) for (x, y) in native().reference_seeds(w, h)]
    region, rounds, sweeps = grow_slabs(band_l, z0, seeds, ctx, connectivity, be)
    dil = dilate_slabs(region, dilation, ctx, be)
    res = {"z0": z0, "band": band_l, "region": region, "dilated": dil, "rounds": rounds, "sweeps": sweeps}
    if gather:
        for k in ("band", "region", "dilated"):
            res[k] = gather_slabs(res[k], depth, ctx)
    return res
