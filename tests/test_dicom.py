"""DICOM Part-10 reader/writer (replaces DCMTK behind DICOMFileImporter, test_pipeline.cpp:33-42)."""
import numpy as np
import pytest


@pytest.mark.parametrize("syntax", ["explicit", "implicit", "big"])
@pytest.mark.parametrize("ptype", ["u16", "i16"])
def test_roundtrip(native, syntax, ptype):
    rng = np.random.default_rng(0)
    px = rng.integers(0, 4000, size=(37, 53)).astype(np.uint16)
    if ptype == "i16":
        px = (px.astype(np.int32) - 2000).astype(np.int16).view(np.uint16)
    b = native.dicom_bytes(px, type=ptype, bits_stored=16, write_rescale=True, slope=2.0, intercept=-5.0,
                           spacing_x=0.5, spacing_y=0.75, instance=9, syntax=syntax)
    h = native.dicom_parse(b)
    assert (h["rows"], h["cols"]) == (37, 53)
    assert h["type"] == ptype
    assert h["slope"] == 2.0 and h["intercept"] == -5.0 and h["has_rescale"]
    assert h["spacing_x"] == 0.5 and h["spacing_y"] == 0.75
    assert h["instance_number"] == 9
    assert np.array_equal(native.dicom_pixels(b), px)


def test_no_preamble_implicit(native):
    px = np.arange(100 * 120, dtype=np.uint16).reshape(100, 120)
    b = native.dicom_bytes(px, syntax="implicit", preamble=False)
    assert np.array_equal(native.dicom_pixels(b), px)


def test_8bit(native):
    px = (np.arange(110 * 100) % 251).astype(np.uint16).reshape(110, 100)
    b = native.dicom_bytes(px, type="u8", bits_stored=8)
    h = native.dicom_parse(b)
    assert h["type"] == "u8" and h["bits_allocated"] == 8
    assert np.array_equal(native.dicom_pixels(b), px)


def test_sequence_skipping(native):
    """An undefined-length SQ with nested items before the image elements must be skipped."""
    px = np.full((4, 4), 7, dtype=np.uint16)
    b = bytearray(native.dicom_bytes(px, syntax="explicit"))
    # insert (0008,1140) SQ undefined length with one undefined-length item containing (0008,1150)
    def tag(g, e):
        return g.to_bytes(2, "little") + e.to_bytes(2, "little")
    inner = tag(0x0008, 0x1150) + b"UI" + (4).to_bytes(2, "little") + b"1.2\x00"
    sq = (tag(0x0008, 0x1140) + b"SQ" + b"\x00\x00" + b"\xff\xff\xff\xff" + tag(0xFFFE, 0xE000) + b"\xff\xff\xff\xff"
          + inner + tag(0xFFFE, 0xE00D) + b"\x00\x00\x00\x00" + tag(0xFFFE, 0xE0DD) + b"\x00\x00\x00\x00")
    pos = b.index(tag(0x0008, 0x0060))  # Modality
    b[pos:pos] = sq
    assert np.array_equal(native.dicom_pixels(bytes(b)), px)


@pytest.mark.parametrize("mode,prefix", [("direct", 16384), ("direct", 1024), ("staged", 0)])
@pytest.mark.parametrize("kind", ["explicit", "implicit", "big", "u8", "long_header", "tiny"])
def test_slice_file_direct_read(native, tmp_path, kind, mode, prefix):
    """SliceFile (engine loader): prefix-parsed header + pread of the pixels (direct; pixel bytes
    inside the prefix come from it) or one whole-file read + streaming stores (staged) must equal
    the whole-file parse for every layout, and fall back to the whole-file path where needed."""
    rng = np.random.default_rng(1)
    shape = (8, 8) if kind == "tiny" else (300, 257)
    px = rng.integers(0, 250 if kind == "u8" else 65535, size=shape).astype(np.uint16)
    syntax = kind if kind in ("implicit", "big") else "explicit"
    b = bytearray(native.dicom_bytes(px, type="u8" if kind == "u8" else "u16",
                                     bits_stored=8 if kind == "u8" else 16, syntax=syntax))
    if kind == "long_header":  # a 40 KiB private OB element pushes the pixels past the prefix
        tag = (0x0009).to_bytes(2, "little") + (0x0010).to_bytes(2, "little")
        blob = tag + b"OB\x00\x00" + (40000).to_bytes(4, "little") + bytes(40000)
        pos = b.index((0x0010).to_bytes(2, "little") + (0x0020).to_bytes(2, "little"))  # PatientID
        b[pos:pos] = blob
    p = tmp_path / "x.dcm"
    p.write_bytes(bytes(b))
    got, direct = native.read_pixels_direct(str(p), mode, prefix)
    assert np.array_equal(got, native.dicom_pixels(bytes(b)))
    assert np.array_equal(got, px)
    assert direct == (mode == "direct" and kind in ("explicit", "implicit"))


def test_rejects_compressed_and_garbage(native):
    with pytest.raises(Exception):
        native.dicom_parse(b"\x00" * 50)
    px = np.zeros((8, 8), dtype=np.uint16)
    b = bytearray(native.dicom_bytes(px))
    i = b.index(b"1.2.840.10008.1.2.1")
    b[i:i + 19] = b"1.2.840.10008.1.2.5"  # RLE lossless → unsupported
    with pytest.raises(Exception, match="transfer syntax"):
        native.dicom_parse(bytes(b))
    with pytest.raises(Exception):
        native.dicom_parse(bytes(native.dicom_bytes(px))[:-20])  # truncated pixel data


def test_synthetic_phantom_ranges(native):
    img = native.phantom_slice(256, 256, 1, 12, 25, 1).astype(np.int32)
    assert img.max() < 3000 and img.min() >= 0
    # the lesion rim must fall inside the SRG band after normalisation (raw 1200–2050, App. A.3)
    assert ((img >= 1200) & (img <= 2050)).sum() > 500
