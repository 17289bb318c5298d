"""torch wrappers of the HIP kernels. Shapes: [N, H, W] (a leading batch dim is added if missing).
Raw pixels are passed as torch.int16 / torch.uint16 tensors (16-bit storage, reinterpreted)."""
import torch

from .._native import native
from ..models.pipeline import PipelineConfig


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _as3d(t):
    return t.unsqueeze(0) if t.dim() == 2 else t


def _check(t, dtypes, name):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype not in dtypes:
        raise ValueError(f"{name} has dtype {t.dtype}, expected one of {dtypes}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_U16 = (torch.int16, torch.uint16)


def median2d(raw, k=7, pixel_type="u16", stored_bits=16):
    """k×k median (clamp-to-edge) of raw 16-bit keys → same-shape tensor of median keys."""
    x = _as3d(raw)
    _check(x, _U16, "raw")
    n, h, w = x.shape
    out = torch.empty_like(x)
    native().k_median(x.data_ptr(), out.data_ptr(), n, h, w, int(k), pixel_type, int(stored_bits), _stream())
    return out if raw.dim() == 3 else out[0]


def threshold(x, lo, hi):
    """BinaryThresholding: lo ≤ x ≤ hi → 1 (uint8), on an f32 CUDA tensor of any shape (K6)."""
    _check(x, (torch.float32,), "x")
    xc = x.contiguous()
    out = torch.empty(xc.shape, dtype=torch.uint8, device=xc.device)
    native().k_threshold(xc.data_ptr(), out.data_ptr(), xc.numel(), float(lo), float(hi), _stream())
    return out


def unpack_bits(words, width):
    """[N, H, wpr] int64 bit-planes → [N, H, width] bool (LSB = left-most pixel)."""
    sh = torch.arange(64, device=words.device, dtype=torch.int64)
    bits = (words.unsqueeze(-1) >> sh) & 1
    return bits.reshape(*words.shape[:-1], -1)[..., :width].bool()


def pack_bits(mask):
    """[N, H, W] bool → [N, H, ceil(W/64)] int64 words."""
    n, h, w = mask.shape
    wpr = (w + 63) // 64
    m = torch.zeros((n, h, wpr * 64), dtype=torch.int64, device=mask.device)
    m[..., :w] = mask.to(torch.int64)
    m = m.reshape(n, h, wpr, 64)
    sh = torch.arange(64, device=mask.device, dtype=torch.int64)
    return (m << sh).sum(-1)


def sharpen_band(median_keys, config: PipelineConfig = None, pixel_type="u16", stored_bits=16, slope=1.0,
                 intercept=0.0, want_sharpened=True):
    """normalise+clip(median keys) → 9×9 Gaussian unsharp mask → SRG band test.
    Returns (sharpened f32 [N,H,W] or None, band bool [N,H,W])."""
    cfg = config or PipelineConfig()
    x = _as3d(median_keys)
    _check(x, _U16, "median_keys")
    n, h, w = x.shape
    wpr = (w + 63) // 64
    band = torch.empty((n, h, wpr), dtype=torch.int64, device=x.device)
    sharp = torch.empty((n, h, w), dtype=torch.float32, device=x.device) if want_sharpened else None
    native().k_sharpen_band(x.data_ptr(), band.data_ptr(), sharp.data_ptr() if sharp is not None else 0, n, h, w,
                            pixel_type, int(stored_bits), float(slope), float(intercept), cfg.pipeline_params(),
                            _stream())
    b = unpack_bits(band, w)
    if median_keys.dim() == 2:
        return (sharp[0] if sharp is not None else None), b[0]
    return sharp, b


def region_grow(band, seeds=None, config: PipelineConfig = None):
    """Seeded region growing on bool band [N,H,W] (LDS-resident ≤ 512², global-memory planes above) + dilation, erosion and the
    renderer border. Returns dict of bool tensors: region, dilated, eroded, border_region."""
    cfg = config or PipelineConfig()
    b = _as3d(band)
    if not b.is_cuda:
        raise ValueError("band must be a CUDA tensor")
    n, h, w = b.shape
    if seeds is None:
        seeds = [(x, y, 0) for (x, y) in native().reference_seeds(w, h)]
    words = pack_bits(b.bool()).contiguous()
    outs = {k: torch.zeros_like(words) for k in ("region", "dilated", "eroded", "border_region")}
    native().k_srg_morph(words.data_ptr(), outs["region"].data_ptr(), outs["dilated"].data_ptr(),
                         outs["eroded"].data_ptr(), outs["border_region"].data_ptr(), n, h, w, list(seeds),
                         cfg.pipeline_params(), int(cfg.border_radius), _stream())
    res = {k: unpack_bits(v, w) for k, v in outs.items()}
    if band.dim() == 2:
        res = {k: v[0] for k, v in res.items()}
    return res


def region_grow3d(band, seeds=(), connectivity=6, region=None):
    """3D seeded region growing (K5 plane sweeps) on a bool band [D, H, W] (CUDA, H, W ≤ 512).
    `seeds` are (x, y, z) voxels; `region` (bool [D, H, W], ⊆ band) is grown further instead of
    starting from nothing — the z-slab decomposition re-grows a slab after its neighbours added
    boundary voxels. Returns (region bool [D, H, W], sweeps)."""
    if band.dim() != 3 or not band.is_cuda:
        raise ValueError("band must be a CUDA tensor [D, H, W]")
    d, h, w = band.shape
    bw = pack_bits(band.bool()).contiguous()
    rw = pack_bits(region.bool() & band.bool()).contiguous() if region is not None else torch.zeros_like(bw)
    sweeps = native().k_srg3d(bw.data_ptr(), rw.data_ptr(), w, h, d, [tuple(map(int, s)) for s in seeds],
                              int(connectivity), region is None, _stream())
    return unpack_bits(rw, w), sweeps


def dilate3d(mask, size=7, ball=False):
    """Cube dilation (size×size×size; `ball`: the digital ball of radius size//2) of a bool
    [D, H, W] CUDA mask, out-of-volume samples ignored."""
    if mask.dim() != 3 or not mask.is_cuda:
        raise ValueError("mask must be a CUDA tensor [D, H, W]")
    d, h, w = mask.shape
    src = pack_bits(mask.bool()).contiguous()
    dst, tmp = torch.empty_like(src), torch.empty_like(src)
    native().k_dilate3d(src.data_ptr(), dst.data_ptr(), tmp.data_ptr(), w, h, d, int(size), _stream(), bool(ball))
    return unpack_bits(dst, w)


JPEG_SAMPLING = {"420": 0, "444": 1, "gray": 2}


def jpeg_encode(canvas, quality=75, header=True, sampling="420"):
    """GPU JPEG of uint8 gray canvases [N,H,W] (H, W multiples of 16) → list of bytes (complete
    JFIF files when header=True, else the entropy-coded segments). `sampling`: "420" (YCbCr
    4:2:0, the default), "444" (YCbCr 4:4:4) or "gray" (one component)."""
    c = _as3d(canvas)
    _check(c, (torch.uint8,), "canvas")
    n, h, w = c.shape
    samp = JPEG_SAMPLING[sampling] if isinstance(sampling, str) else int(sampling)
    segs = native().k_jpeg(c.data_ptr(), n, h, w, int(quality), _stream(), samp)
    if not header:
        return segs
    hdr = native().jpeg_header(w, h, int(quality), samp)
    return [None if s is None else hdr + s + b"\xff\xd9" for s in segs]
