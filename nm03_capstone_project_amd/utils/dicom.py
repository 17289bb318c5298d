"""DICOM helpers over the native Part-10 codec (src/io/dicom.cpp)."""
from .._native import native


def parse_dicom(data: bytes):
    return native().dicom_parse(data)


def read_slice(path, min_dim=0):
    """→ (uint16 [H, W] raw samples, meta dict: type, stored_bits, slope, intercept, spacing)."""
    return native().read_slice(path, min_dim)


def dicom_bytes(pixels, **kw):
    return native().dicom_bytes(pixels, **kw)
