"""DICOM helpers over the native Part-10 codec (src/io/dicom.cpp).

The reference reads one slice at a time through FAST's DICOMFileImporter
(main_sequential.cpp:177-186) and never looks at a series as a whole; `read_series` is the
volume-mode (BASELINE config 5) counterpart: the series' slices in the reference's file-number
order (main_sequential.cpp:18-30), checked for one shape, stacked into a [D, H, W] volume."""
import os
from dataclasses import dataclass, field

import numpy as np

from .._native import native


def parse_dicom(data: bytes):
    """Header fields of a Part-10 byte string (rows, cols, bits, rescale, spacing, UIDs, pixel offset...)."""
    return native().dicom_parse(data)


def read_slice(path, min_dim=0, frame=-1):
    """→ (uint16 [H, W] raw samples, meta dict: type, stored_bits, slope, intercept, spacing).
    `frame`: -1 rejects multi-frame files, k >= 0 imports frame k. MONOCHROME1 samples come back
    inverted within the stored bits (MONOCHROME2 semantics)."""
    return native().read_slice(path, min_dim, frame)


def dicom_bytes(pixels, **kw):
    return native().dicom_bytes(pixels, **kw)


@dataclass
class Slice:
    """One decoded slice: the stored samples as read (uint16 bit patterns; signed types are
    reinterpreted by `values`) and the header fields the pipeline uses."""
    path: str
    raw: np.ndarray
    meta: dict = field(default_factory=dict)

    @property
    def shape(self):
        return self.raw.shape

    @property
    def spacing(self):
        """(row spacing, column spacing) in mm, PixelSpacing order."""
        return float(self.meta.get("spacing_y", 1.0)), float(self.meta.get("spacing_x", 1.0))

    @property
    def values(self):
        """Stored values with their DICOM sign (int16 for signed 16-bit data, else the samples)."""
        return self.raw.view(np.int16) if self.meta.get("type") == "i16" else self.raw

    def rescaled(self):
        """Modality values: slope · stored + intercept (RescaleSlope/Intercept), float32."""
        slope = float(self.meta.get("slope", 1.0))
        icpt = float(self.meta.get("intercept", 0.0))
        return (self.values.astype(np.float32) * np.float32(slope) + np.float32(icpt)).astype(np.float32)


def load_slice(path, min_dim=0):
    """read_slice as a `Slice` (raises on unreadable or too-small files, as the CLI's import stage)."""
    raw, meta = read_slice(os.fspath(path), min_dim)
    return Slice(os.fspath(path), raw, dict(meta))


def series_files(series_dir):
    """The series' *.dcm files in the reference's order: ascending file number (the integer after
    the last '-' of the stem, main_sequential.cpp:18-30), then name."""
    n = native()
    names = [f for f in os.listdir(series_dir) if f.lower().endswith(".dcm")]
    names.sort(key=lambda f: (n.extract_file_number(f), f))
    return [os.path.join(series_dir, f) for f in names]


def read_series(series_dir, min_dim=0):
    """→ (uint16 [D, H, W] volume of stored samples, [Slice] without pixel copies kept twice).

    Every slice must share one shape (a mixed series cannot be stacked): ValueError naming the
    first slice that differs."""
    files = series_files(series_dir)
    if not files:
        raise ValueError(f"no .dcm files in {series_dir}")
    slices = [load_slice(f, min_dim) for f in files]
    shape = slices[0].shape
    for s in slices[1:]:
        if s.shape != shape:
            raise ValueError(f"{s.path}: shape {s.shape} differs from {slices[0].path}: {shape}")
    vol = np.stack([s.raw for s in slices])
    for i, s in enumerate(slices):
        s.raw = vol[i]  # views into the volume: one copy of the pixels
    return vol, slices
