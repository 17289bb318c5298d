"""CPU golden model vs plain-PyTorch references and hand-checked definitions."""
import numpy as np
import pytest
import torch

from nm03_capstone_project_amd.ops import reference as R


def _img(native, h=96, w=80, seed=3):
    raw = native.phantom_slice(h, w, seed, 10, 25, 11)
    return raw


def test_norm_clip_matches_torch(native):
    raw = _img(native)
    p = native.PipelineParams()
    c = native.golden_norm_clip(raw, "u16", 16, 1.0, 0.0, p)
    ref = R.norm_clip(torch.from_numpy(raw.astype(np.float32))).numpy()
    assert np.abs(c - ref).max() <= 1.2e-7
    assert c.min() >= 0.68 - 1e-7


def test_rescale_and_signed(native):
    raw = (np.arange(100 * 100, dtype=np.int32).reshape(100, 100) % 4000 - 1000).astype(np.int16).view(np.uint16)
    p = native.PipelineParams()
    c = native.golden_norm_clip(raw, "i16", 16, 2.0, 10.0, p)
    x = raw.view(np.int16).astype(np.float32) * np.float32(2.0) + np.float32(10.0)
    ref = R.norm_clip(torch.from_numpy(x)).numpy()
    assert np.abs(c - ref).max() <= 2.5e-7


@pytest.mark.parametrize("k", [3, 5, 7])
def test_median_matches_torch(native, k):
    raw = _img(native)
    p = native.PipelineParams()
    c = native.golden_norm_clip(raw, "u16", 16, 1.0, 0.0, p)
    m = native.golden_median(c, k)
    ref = R.median(torch.from_numpy(c), k).numpy()
    assert np.array_equal(m, ref)


def test_median_commutes_with_normalisation(native):
    """median(c(x)) == c(median(x)): the GPU computes on raw keys (pixel_math.h)."""
    raw = _img(native)
    p = native.PipelineParams()
    mk = native.golden_median_u16(raw, 7)
    via_keys = native.golden_norm_clip(mk, "u16", 16, 1.0, 0.0, p)
    direct = native.golden_median(native.golden_norm_clip(raw, "u16", 16, 1.0, 0.0, p), 7)
    assert np.array_equal(via_keys, direct)


def test_vector_median_equals_median(native):
    """App. A.4: FAST's VMF on 1-channel data quantised at 2e-4 is the median."""
    raw = _img(native, 40, 36)
    p = native.PipelineParams()
    c = native.golden_norm_clip(raw, "u16", 16, 1.0, 0.0, p)
    assert np.array_equal(native.golden_vector_median(c, 7), native.golden_median(c, 7))


def test_sharpen_separable_vs_direct_and_torch(native):
    raw = _img(native)
    p = native.PipelineParams()
    m = native.golden_median(native.golden_norm_clip(raw, "u16", 16, 1.0, 0.0, p), 7)
    sep = native.golden_sharpen(m, 2.0, 0.5, 9, False)
    direct = native.golden_sharpen(m, 2.0, 0.5, 9, True)
    ref = R.sharpen(torch.from_numpy(m)).numpy()
    assert np.abs(sep - ref).max() < 2e-6
    assert np.abs(direct - ref).max() < 2e-6
    taps = native.gaussian_taps(0.5, 9)
    assert abs(sum(taps) - 1.0) < 1e-6 and taps[4] > 0.78


@pytest.mark.parametrize("conn", [4, 8])
def test_region_grow_vs_torch(native, conn):
    rng = np.random.default_rng(conn)
    band = (rng.random((70, 90)) < 0.55).astype(np.uint8)
    seeds = [(x, y, 0) for (x, y) in native.reference_seeds(90, 70)]
    g = native.golden_region_grow(band, seeds, conn)
    ref = R.region_grow(torch.from_numpy(band.astype(bool)), seeds, conn).numpy()
    assert np.array_equal(g.astype(bool), ref)


@pytest.mark.parametrize("size", [3, 5])
def test_morphology_vs_torch(native, size):
    rng = np.random.default_rng(size)
    m = (rng.random((50, 70)) < 0.6).astype(np.uint8)
    assert np.array_equal(native.golden_morph(m, size, True).astype(bool), R.dilate(torch.from_numpy(m), size).numpy())
    assert np.array_equal(native.golden_morph(m, size, False).astype(bool), R.erode(torch.from_numpy(m), size).numpy())
    assert np.array_equal(native.golden_border(m, 2).astype(bool), R.border(torch.from_numpy(m.astype(bool)), 2).numpy())


def test_region_grow3d_and_dilate3d(native):
    rng = np.random.default_rng(5)
    band = (rng.random((12, 20, 24)) < 0.5).astype(np.uint8)
    seeds = [(10, 10, 6), (3, 4, 2)]
    r6 = native.golden_region_grow3d(band, seeds, 6).astype(bool)
    # torch reference: iterative 6-neighbour dilation constrained to the band
    reg = torch.zeros(band.shape, dtype=torch.bool)
    for x, y, z in seeds:
        if band[z, y, x]:
            reg[z, y, x] = True
    b = torch.from_numpy(band.astype(bool))
    k = torch.zeros((3, 3, 3))
    k[1, 1, :] = k[1, :, 1] = k[:, 1, 1] = 1
    while True:
        nxt = (torch.nn.functional.conv3d(reg.float()[None, None], k[None, None], padding=1)[0, 0] > 0) & b
        if torch.equal(nxt, reg):
            break
        reg = nxt
    assert np.array_equal(r6, reg.numpy())
    d = native.golden_dilate3d(r6.astype(np.uint8), 5).astype(bool)
    ref = torch.nn.functional.max_pool3d(torch.from_numpy(r6).float()[None, None], 5, 1, 2)[0, 0] > 0
    assert np.array_equal(d, ref.numpy())


def test_render_vs_torch(native):
    raw = _img(native, 256, 256).astype(np.float32)
    lo, hi = float(raw.min()), float(raw.max())
    g = native.golden_render_gray(raw, lo, hi, 1.0, 1.0, 512, 512)
    ref = R.render_gray(torch.from_numpy(raw), lo, hi).numpy()
    assert np.abs(g.astype(int) - ref.astype(int)).max() <= 1
    lab = (raw > 1500).astype(np.uint8)
    brd = native.golden_border(lab, 2)
    gl = native.golden_render_labels(lab, brd, 1.0, 1.0, 512, 512, 153, 255)
    rl = R.render_labels(torch.from_numpy(lab.astype(bool)), torch.from_numpy(brd.astype(bool))).numpy()
    assert np.array_equal(gl, rl)
    assert set(np.unique(gl)) <= {0, 153, 255}
    assert native.opacity_u8(0.6) == 153 and native.opacity_u8(1.0) == 255


def test_render_aspect_fit(native):
    v = np.ones((100, 200), np.float32)
    g = native.golden_render_gray(v, 0.0, 2.0, 1.0, 1.0, 512, 512)
    # 200×100 fitted into 512²: 512×256 band centred vertically, black above/below
    assert g[0].max() == 0 and g[-1].max() == 0 and g[256].min() == 128


def test_full_golden_pipeline_shapes(native):
    raw = native.phantom_slice(256, 256, 2, 12, 25, 3)
    out = native.golden_run(raw)
    assert out["band"].shape == (256, 256)
    assert out["region"].sum() <= out["band"].sum()
    assert out["dilated"].sum() >= out["region"].sum()
    assert (out["eroded"] <= out["region"]).all()
    assert out["jpeg_original"][:2] == b"\xff\xd8" and out["jpeg_processed"][-2:] == b"\xff\xd9"


@pytest.mark.parametrize("size", [3, 5, 7, 9])
def test_disc_morphology_vs_torch(native, size):
    """--se-shape disc (SURVEY App. A.7 / §7.6 risk 1): golden disc dilation/erosion = conv2d counts
    with the digital disc of radius size//2; size 3 is the 4-neighbour cross."""
    rng = np.random.default_rng(size)
    m = (rng.random((61, 77)) < 0.55).astype(np.uint8)
    m[20:40, 30:60] = 1
    t = torch.from_numpy(m)
    assert np.array_equal(native.golden_morph(m, size, True, True).astype(bool), R.dilate_disc(t, size).numpy())
    assert np.array_equal(native.golden_morph(m, size, False, True).astype(bool), R.erode_disc(t, size).numpy())
    if size == 3:
        assert R.disc_se(3).sum() == 5
    # the disc lies inside the square: square dilation ⊇ disc dilation, square erosion ⊆ disc erosion
    assert (native.golden_morph(m, size, True, False) >= native.golden_morph(m, size, True, True)).all()
    assert (native.golden_morph(m, size, False, False) <= native.golden_morph(m, size, False, True)).all()


@pytest.mark.parametrize("size", [3, 5, 7])
def test_ball_dilation3d_vs_torch(native, size):
    rng = np.random.default_rng(size)
    m = (rng.random((9, 23, 70)) < 0.04).astype(np.uint8)
    got = native.golden_dilate3d(m, size, True).astype(bool)
    assert np.array_equal(got, R.dilate_ball(torch.from_numpy(m), size).numpy())
    assert (native.golden_dilate3d(m, size, False) >= got).all()


def test_golden_pipeline_se_shape(native):
    """The whole golden slice pipeline with --se-shape disc differs from square only in the morphology."""
    import nm03_capstone_project_amd as nm
    raw = native.phantom_slice(256, 256, 3, 12, 25, 11)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": 1.0, "spacing_y": 1.0}
    sq = nm.SlicePipeline(nm.PipelineConfig()).golden(raw, meta)
    dc = nm.SlicePipeline(nm.PipelineConfig(se_shape=1)).golden(raw, meta)
    assert np.array_equal(sq["region"], dc["region"])
    assert np.array_equal(dc["dilated"].astype(bool), native.golden_morph(dc["region"].astype(np.uint8), 3, True, True).astype(bool))
    assert np.array_equal(dc["eroded"].astype(bool), native.golden_morph(dc["region"].astype(np.uint8), 3, False, True).astype(bool))
    assert not np.array_equal(sq["dilated"], dc["dilated"])


@pytest.mark.parametrize("shape,spacing", [((256, 256), (1.0, 1.0)), ((200, 160), (0.9, 1.2))])
def test_render_nearest_vs_torch(native, shape, spacing):
    """--render-filter nearest: the golden gray render equals the torch reference's nearest sampling
    (exact-2× fits and general fits); bilinear stays the default."""
    h, w = shape
    v = native.phantom_slice(h, w, 2, 3, 9, 5).astype(np.float32)
    lo, hi = float(v.min()), float(v.max())
    sx, sy = spacing
    got = native.golden_render_gray(v, lo, hi, sx, sy, 512, 512, True)
    if sx == sy:
        ref = R.render_gray(torch.from_numpy(v), lo, hi, nearest=True).numpy()
        assert np.array_equal(got, ref)
    bil = native.golden_render_gray(v, lo, hi, sx, sy, 512, 512)
    assert not np.array_equal(got, bil)
    assert np.array_equal(bil, native.golden_render_gray(v, lo, hi, sx, sy, 512, 512, False))
