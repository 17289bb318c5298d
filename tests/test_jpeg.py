"""JPEG exporter: byte-compatibility with libjpeg(-turbo) through Pillow."""
import io

import numpy as np
import pytest

PIL = pytest.importorskip("PIL.Image")


def _pil_bytes(gray, q=75):
    bio = io.BytesIO()
    PIL.fromarray(gray).convert("RGB").save(bio, format="JPEG", quality=q)
    return bio.getvalue()


@pytest.mark.parametrize("shape", [(512, 512), (64, 48), (100, 37), (33, 130)])
@pytest.mark.parametrize("kind", ["noise", "gradient", "flat", "binary"])
def test_byte_identical_to_libjpeg(native, shape, kind):
    rng = np.random.default_rng(hash((shape, kind)) % 2**32)
    h, w = shape
    if kind == "noise":
        g = rng.integers(0, 256, size=shape, dtype=np.uint8)
    elif kind == "gradient":
        g = (np.add.outer(np.arange(h), np.arange(w)) * 255 // max(1, h + w - 2)).astype(np.uint8)
    elif kind == "flat":
        g = np.full(shape, 77, np.uint8)
    else:
        g = np.where(rng.random(shape) < 0.2, 255, np.where(rng.random(shape) < 0.3, 153, 0)).astype(np.uint8)
    ours = native.jpeg_encode_gray420(g, 75)
    assert ours == _pil_bytes(g)


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
