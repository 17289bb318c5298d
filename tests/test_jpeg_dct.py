"""Lossy JPEG import: JPEG Baseline (1.2.840.10008.1.2.4.50, 8-bit) and JPEG Extended
(1.2.840.10008.1.2.4.51, 8/12-bit), one component, sequential Huffman DCT (src/io/jpeg_dct.cpp).

FAST imports through DCMTK (main_sequential.cpp:175-177) whose IJG-based codecs decode these syntaxes with
the islow inverse DCT. DCMTK itself is not in the image, so parity with it is UNPINNED; the decoder is held
against libjpeg-turbo through Pillow instead (the same islow arithmetic: 8-bit output must be
byte-identical), and 12-bit images (no 12-bit decoder in Pillow) against properties of the transform."""
import io

import numpy as np
import pytest


def _smooth(rng, shape, hi):
    r, c = shape
    y, x = np.mgrid[0:r, 0:c]
    img = hi * (0.35 + 0.25 * np.sin(x / 9.0) * np.cos(y / 13.0)) + rng.normal(0, hi / 200, size=shape)
    img[r // 3:2 * r // 3, c // 4:c // 2] += hi * 0.2
    return np.clip(img, 0, hi - 1).astype(np.uint16)


@pytest.mark.parametrize("shape", [(64, 64), (37, 53), (256, 256), (9, 300)])
@pytest.mark.parametrize("quality", [50, 75, 95])
def test_decoder_equals_libjpeg_on_pillow_streams(native, shape, quality):
    PIL = pytest.importorskip("PIL.Image")
    img = _smooth(np.random.default_rng(sum(shape) + quality), shape, 256).astype(np.uint8)
    b = io.BytesIO()
    PIL.fromarray(img, "L").save(b, "JPEG", quality=quality)
    got = native.jpeg_dct_decode(b.getvalue())
    assert got["precision"] == 8 and got["sof"] == 0
    assert np.array_equal(got["pixels"], np.asarray(PIL.open(io.BytesIO(b.getvalue()))))


@pytest.mark.parametrize("restart_blocks", [0, 1, 7])
def test_encoder_streams_decode_identically_in_libjpeg(native, restart_blocks):
    PIL = pytest.importorskip("PIL.Image")
    img = _smooth(np.random.default_rng(3), (70, 90), 256)
    j = native.jpeg_dct_encode(img, 8, 85, restart_blocks)
    ours = native.jpeg_dct_decode(j)
    assert ours["restart_interval"] == restart_blocks
    assert np.array_equal(ours["pixels"], np.asarray(PIL.open(io.BytesIO(j))))
    assert np.abs(ours["pixels"].astype(int) - img.astype(int)).max() < 24  # lossy, but close at q85


def test_12bit_extended_properties(native):
    """12-bit (SOF1): DC-only blocks reconstruct exactly, a smooth image to high PSNR; restart markers."""
    flat = np.full((40, 48), 2000, np.uint16)
    d = native.jpeg_dct_decode(native.jpeg_dct_encode(flat, 12, 95, 0))
    assert d["precision"] == 12 and d["sof"] == 1 and np.array_equal(d["pixels"], flat)
    img = _smooth(np.random.default_rng(4), (96, 80), 4096)
    for rb in (0, 5):
        p = native.jpeg_dct_decode(native.jpeg_dct_encode(img, 12, 95, rb))["pixels"].astype(np.float64)
        mse = ((p - img) ** 2).mean()
        assert 10 * np.log10(4095.0 ** 2 / max(mse, 1e-9)) > 50.0
        assert p.max() <= 4095 and p.min() >= 0


def test_other_processes_and_corruption_rejected(native):
    PIL = pytest.importorskip("PIL.Image")
    img = _smooth(np.random.default_rng(5), (64, 64), 256).astype(np.uint8)
    b = io.BytesIO()
    PIL.fromarray(img, "L").save(b, "JPEG", quality=80, progressive=True)
    with pytest.raises(Exception, match="Unsupported JPEG process"):
        native.jpeg_dct_decode(b.getvalue())
    rgb = io.BytesIO()
    PIL.fromarray(np.stack([img] * 3, -1), "RGB").save(rgb, "JPEG", quality=80)
    with pytest.raises(Exception, match="components"):
        native.jpeg_dct_decode(rgb.getvalue())
    j = native.jpeg_dct_encode(img.astype(np.uint16), 8, 80, 0)
    with pytest.raises(Exception, match="Truncated|Corrupt"):
        native.jpeg_dct_decode(j[:len(j) // 4])


@pytest.mark.parametrize("syntax,ptype,bits", [("jpeg-baseline", "u8", 8), ("jpeg-extended", "u16", 12),
                                               ("jpeg-extended", "i16", 12)])
def test_dicom_lossy_jpeg_import(native, syntax, ptype, bits):
    rng = np.random.default_rng(6)
    px = _smooth(rng, (67, 131), 1 << bits)
    b = native.dicom_bytes(px if ptype != "i16" else px, type=ptype, bits_stored=bits, syntax=syntax,
                           jpeg_quality=92, write_rescale=True, slope=1.0, intercept=-1024.0)
    ts = "1.2.840.10008.1.2.4.50" if syntax == "jpeg-baseline" else "1.2.840.10008.1.2.4.51"
    assert ts.encode() in b
    h = native.dicom_parse(b)
    assert h["syntax"] == syntax and (h["rows"], h["cols"]) == (67, 131) and h["intercept"] == -1024.0
    got = native.dicom_pixels(b)
    # the stored samples are the codec's decode of the frame (the writer encodes the stored bits)
    want = native.jpeg_dct_decode(native.jpeg_dct_encode(px & ((1 << bits) - 1), 8 if bits == 8 else 12, 92, 0))["pixels"]
    if ptype == "i16":  # sign-extended from BitsStored, like the native encodings
        want = np.where(want >= 1 << (bits - 1), want.astype(np.int32) - (1 << bits), want).astype(np.int16).view(np.uint16)
    assert np.array_equal(got, want)


def test_dicom_lossy_jpeg_multiframe(native):
    rng = np.random.default_rng(7)
    st = np.stack([_smooth(rng, (40, 48), 4096) for _ in range(3)])
    b = native.dicom_bytes(st, bits_stored=12, syntax="jpeg-extended", jpeg_restart_rows=2)
    for k in range(3):
        want = native.jpeg_dct_decode(native.jpeg_dct_encode(st[k], 12, 90, 2 * 6))["pixels"]
        assert np.array_equal(native.dicom_pixels(b, k), want)


@pytest.mark.parametrize("syntax,sof", [("jpeg-extended", b"\xff\xc1"), ("jpeg-lossless", b"\xff\xc3")])
def test_dicom_jpeg_frame_size_checked_before_decoding(native, syntax, sof):
    """A SOF that disagrees with the dataset's Rows/Columns is rejected at the SOF, before the decoder
    sizes its output from it (a corrupt 65535x65535 SOF must not allocate 8 GiB)."""
    px = _smooth(np.random.default_rng(8), (40, 48), 4096)
    b = bytearray(native.dicom_bytes(px, bits_stored=12, syntax=syntax))
    i = b.find(sof)
    assert i > 0
    b[i + 5:i + 7] = b"\xff\xff"  # SOF rows
    with pytest.raises(Exception, match="expected 48x40"):
        native.dicom_pixels(bytes(b))
