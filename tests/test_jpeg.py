"""JPEG exporter: byte-compatibility with libjpeg(-turbo) through Pillow."""
import io

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")


def _pil_bytes(gray, q=75, sampling=0):
    """libjpeg's file for a gray plane: as RGB with 4:2:0 (sampling 0) or 4:4:4 (1) chroma, or as
    an 8-bit gray image (2: one component)."""
    bio = io.BytesIO()
    if sampling == 2:
        PIL.fromarray(gray).save(bio, format="JPEG", quality=q)
    else:
        PIL.fromarray(gray).convert("RGB").save(bio, format="JPEG", quality=q, subsampling=2 if sampling == 0 else 0)
    return bio.getvalue()


def _image(shape, kind):
    rng = np.random.default_rng(hash((shape, kind)) % 2**32)
    h, w = shape
    if kind == "noise":
        return rng.integers(0, 256, size=shape, dtype=np.uint8)
    if kind == "gradient":
        return (np.add.outer(np.arange(h), np.arange(w)) * 255 // max(1, h + w - 2)).astype(np.uint8)
    if kind == "flat":
        return np.full(shape, 77, np.uint8)
    return np.where(rng.random(shape) < 0.2, 255, np.where(rng.random(shape) < 0.3, 153, 0)).astype(np.uint8)


@pytest.mark.parametrize("shape", [(512, 512), (64, 48), (100, 37), (33, 130)])
@pytest.mark.parametrize("kind", ["noise", "gradient", "flat", "binary"])
def test_byte_identical_to_libjpeg(native, shape, kind):
    g = _image(shape, kind)
    ours = native.jpeg_encode_gray420(g, 75)
    assert ours == _pil_bytes(g)


# --jpeg-sampling 444 / gray (VERDICT r4 missing #3): the other two layouts Qt's writer may produce
# for FAST's image, byte-identical to libjpeg as well.
@pytest.mark.parametrize("sampling", [1, 2])
@pytest.mark.parametrize("shape", [(512, 512), (64, 48), (100, 37), (33, 130)])
@pytest.mark.parametrize("kind", ["noise", "gradient", "flat", "binary"])
def test_other_samplings_byte_identical_to_libjpeg(native, shape, kind, sampling):
    g = _image(shape, kind)
    assert native.jpeg_encode_gray(g, 75, sampling) == _pil_bytes(g, 75, sampling)


@pytest.mark.parametrize("sampling", [0, 1, 2])
def test_sampling_header_and_decode(native, sampling):
    g = _image((64, 80), "gradient")
    b = native.jpeg_encode_gray(g, 75, sampling)
    assert b.startswith(native.jpeg_header(80, 64, 75, sampling))
    im = PIL.open(io.BytesIO(b))
    assert im.mode == ("L" if sampling == 2 else "RGB") and im.size == (80, 64)
    dec = np.asarray(im.convert("L")).astype(float)
    assert np.abs(dec - g).max() <= 8
    if sampling == 1:
        assert im.layer == [(1, 1, 1, 0), (2, 1, 1, 1), (3, 1, 1, 1)]
    if sampling == 0:
        assert im.layer == [(1, 2, 2, 0), (2, 1, 1, 1), (3, 1, 1, 1)]
    assert native.jpeg_encode_gray(g, 75, 0) == native.jpeg_encode_gray420(g, 75)
    with pytest.raises(Exception):
        native.jpeg_encode_gray(g, 75, 3)


@pytest.mark.parametrize("q", [10, 50, 90, 100])
def test_quality_tables(native, q):
    g = np.random.default_rng(q).integers(0, 256, size=(64, 64), dtype=np.uint8)
    assert native.jpeg_encode_gray420(g, q) == _pil_bytes(g, q)


def test_decodes_and_psnr(native):
    raw = native.phantom_slice(256, 256, 1, 12, 25, 1).astype(np.float32)
    c = native.golden_render_gray(raw, float(raw.min()), float(raw.max()), 1.0, 1.0, 512, 512)
    b = native.jpeg_encode_gray420(c, 75)
    dec = np.asarray(PIL.open(io.BytesIO(b)).convert("L")).astype(float)
    psnr = 10 * np.log10(255 ** 2 / np.mean((dec - c) ** 2))
    assert psnr > 35


def test_q75_luma_table(native):
    ql, qc = native.jpeg_quant_tables(75)
    assert ql[:4] == [8, 6, 5, 8] and qc[0] == 9
