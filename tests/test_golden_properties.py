"""Property tests of the golden model against independent definitions: numpy's
median over edge-padded windows, scipy.ndimage morphology and connected-component labelling. The
GPU kernels are held bit-exact to this model by tests/test_gpu.py, so these properties carry over."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

scipy_ndimage = pytest.importorskip("scipy.ndimage")

SETTINGS = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])


@st.composite
def images(draw, max_side=40, lo=0, hi=4095):
    h = draw(st.integers(3, max_side))
    w = draw(st.integers(3, max_side))
    seed = draw(st.integers(0, 2**31 - 1))
    return np.random.default_rng(seed).integers(lo, hi + 1, size=(h, w)).astype(np.uint16)


@st.composite
def masks(draw, max_side=48):
    h = draw(st.integers(2, max_side))
    w = draw(st.integers(2, max_side))
    density = draw(st.floats(0.2, 0.8))
    seed = draw(st.integers(0, 2**31 - 1))
    return (np.random.default_rng(seed).random((h, w)) < density).astype(np.uint8)


@SETTINGS
@given(img=images(), k=st.sampled_from([3, 5, 7, 9]))
def test_median_equals_padded_window_median(native, img, k):
    """Clamp-to-edge k×k median (FAST's VectorMedianFilter on 1-channel data)."""
    r = k // 2
    pad = np.pad(img.astype(np.int64), r, mode="edge")
    win = np.lib.stride_tricks.sliding_window_view(pad, (k, k))
    ref = np.median(win.reshape(img.shape[0], img.shape[1], k * k), axis=-1).astype(np.uint16)
    assert np.array_equal(native.golden_median_u16(img, k), ref)


@SETTINGS
@given(img=images(max_side=24, lo=0, hi=4095), k=st.sampled_from([3, 5, 7]))
def test_vector_median_equals_median_on_quantised_data(native, img, k):
    """The O(n²) vector-median definition picks the scalar median on the 2·10⁻⁴-quantised data of
    this pipeline (App. A.4's argument), so FAST's VMF ≡ the median kernel."""
    p = native.PipelineParams()
    c = native.golden_norm_clip(img, "u16", 16, 1.0, 0.0, p)
    assert np.array_equal(native.golden_vector_median(c, k), native.golden_median(c, k))


def _disc(size, dims=2):
    r = size // 2
    g = np.indices((2 * r + 1,) * dims) - r
    return (g * g).sum(axis=0) <= r * r


@SETTINGS
@given(m=masks(), size=st.sampled_from([1, 3, 5, 7, 9]))
def test_disc_morphology_equals_scipy(native, m, size):
    """--se-shape disc: digital disc of radius size/2 (|d|² ≤ r²), out-of-image samples ignored;
    dilation and erosion are duals through the complement with that border convention."""
    se = _disc(size)
    dil = scipy_ndimage.binary_dilation(m.astype(bool), structure=se)
    ero = scipy_ndimage.binary_erosion(m.astype(bool), structure=se, border_value=1)
    gd = native.golden_morph(m, size, True, True).astype(bool)
    ge = native.golden_morph(m, size, False, True).astype(bool)
    assert np.array_equal(gd, dil) and np.array_equal(ge, ero)
    assert np.array_equal(ge, ~native.golden_morph((1 - m).astype(np.uint8), size, True, True).astype(bool))
    assert (gd >= m.astype(bool)).all() and (ge <= m.astype(bool)).all()  # extensive / anti-extensive


@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(seed=st.integers(0, 2**31 - 1), size=st.sampled_from([3, 5, 7]), density=st.floats(0.01, 0.2))
def test_ball_dilation_equals_scipy(native, seed, size, density):
    """--mode 3d --se-shape disc: the digital ball of radius size/2."""
    m = (np.random.default_rng(seed).random((9, 14, 11)) < density).astype(np.uint8)
    ref = scipy_ndimage.binary_dilation(m.astype(bool), structure=_disc(size, 3))
    assert np.array_equal(native.golden_dilate3d(m, size, True).astype(bool), ref)
    cube = scipy_ndimage.binary_dilation(m.astype(bool), structure=np.ones((size,) * 3, bool))
    assert np.array_equal(native.golden_dilate3d(m, size, False).astype(bool), cube)


@SETTINGS
@given(m=masks(), size=st.sampled_from([1, 3, 5, 7]))
def test_morphology_equals_scipy(native, m, size):
    """Square-SE binary dilation / erosion, out-of-image samples ignored (App. A.7)."""
    se = np.ones((size, size), bool)
    dil = scipy_ndimage.binary_dilation(m.astype(bool), structure=se)
    ero = scipy_ndimage.binary_erosion(m.astype(bool), structure=se, border_value=1)
    assert np.array_equal(native.golden_morph(m, size, True).astype(bool), dil)
    assert np.array_equal(native.golden_morph(m, size, False).astype(bool), ero)


@SETTINGS
@given(m=masks(), conn=st.sampled_from([4, 8]), nseeds=st.integers(1, 6), seed=st.integers(0, 10**6))
def test_region_grow_equals_connected_components(native, m, conn, nseeds, seed):
    """SRG region = union of the band's connected components that contain an in-band seed."""
    h, w = m.shape
    rng = np.random.default_rng(seed)
    seeds = [(int(rng.integers(0, w)), int(rng.integers(0, h)), 0) for _ in range(nseeds)]
    structure = np.ones((3, 3), bool) if conn == 8 else None
    lab, _ = scipy_ndimage.label(m.astype(bool), structure=structure)
    keep = {lab[y, x] for (x, y, _) in seeds if lab[y, x] > 0}
    ref = np.isin(lab, list(keep)) & (lab > 0)
    assert np.array_equal(native.golden_region_grow(m, seeds, conn).astype(bool), ref)


@SETTINGS
@given(m=masks(), radius=st.integers(1, 3))
def test_border_is_mask_minus_erosion(native, m, radius):
    """Renderer border (App. A.9): label pixels with a 0 within Chebyshev radius r (in-image)."""
    se = np.ones((2 * radius + 1,) * 2, bool)
    ero = scipy_ndimage.binary_erosion(m.astype(bool), structure=se, border_value=1)
    assert np.array_equal(native.golden_border(m, radius).astype(bool), m.astype(bool) & ~ero)


@settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(d=st.integers(2, 10), h=st.integers(4, 24), w=st.integers(4, 24), conn=st.sampled_from([6, 26]),
       size=st.sampled_from([1, 3, 5, 7]), seed=st.integers(0, 10**6))
def test_3d_grow_and_cube_dilation_equal_scipy(native, d, h, w, conn, size, seed):
    rng = np.random.default_rng(seed)
    band = (rng.random((d, h, w)) < 0.45).astype(np.uint8)
    seeds = [(int(rng.integers(0, w)), int(rng.integers(0, h)), int(rng.integers(0, d))) for _ in range(4)]
    structure = np.ones((3, 3, 3), bool) if conn == 26 else None
    lab, _ = scipy_ndimage.label(band.astype(bool), structure=structure)
    keep = {lab[z, y, x] for (x, y, z) in seeds if lab[z, y, x] > 0}
    ref = np.isin(lab, list(keep)) & (lab > 0)
    region = native.golden_region_grow3d(band, seeds, conn)
    assert np.array_equal(region.astype(bool), ref)
    dil = scipy_ndimage.binary_dilation(ref, structure=np.ones((size,) * 3, bool))
    assert np.array_equal(native.golden_dilate3d(region, size).astype(bool), dil)
