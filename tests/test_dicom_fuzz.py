"""Mutation fuzzing of the DICOM reader (src/io/dicom.cpp): the files come from outside, so any byte
sequence must either parse or raise the reader's error — never crash the process, hang, or
allocate without bound. Seeds: every transfer syntax, photometric and frame layout the writer
produces; mutants: byte flips, 0xFF runs over length fields, truncations and splices. Deterministic
(fixed RNG seeds); the parsed paths are the in-memory parser, the pixel copy, and the file reader's
prefix/retry path (parse_prefix + SliceFile) that the engine's loaders use."""
import numpy as np
import pytest

_MAX_PIXELS = 1 << 22  # pixel copies are only attempted for headers of plausible size


def _seeds(native):
    rng = np.random.default_rng(11)
    px = rng.integers(0, 4096, size=(24, 20)).astype(np.uint16)
    mf = rng.integers(0, 4096, size=(3, 12, 16)).astype(np.uint16)
    out = []
    for syntax in ("explicit", "implicit", "big", "deflated", "rle"):
        out.append(native.dicom_bytes(px, syntax=syntax, bits_stored=12))
        out.append(native.dicom_bytes(mf, syntax=syntax, bits_stored=12))
    out.append(native.dicom_bytes(px, syntax="explicit", preamble=False))
    out.append(native.dicom_bytes(px, type="i16", bits_stored=12, write_rescale=True, slope=2.0, intercept=-5.0))
    out.append(native.dicom_bytes(px, photometric="MONOCHROME1", bits_stored=12))
    out.append(native.dicom_bytes((px & 0xFF).astype(np.uint16), type="u8", bits_stored=8))
    return out


def _mutants(seed_bytes, rng, n):
    b0 = np.frombuffer(seed_bytes, np.uint8)
    for _ in range(n):
        b = b0.copy()
        kind = rng.integers(0, 5)
        if kind == 0:  # random byte flips
            idx = rng.integers(0, len(b), size=rng.integers(1, 8))
            b[idx] = rng.integers(0, 256, size=len(idx))
        elif kind == 1:  # 0xFF runs (undefined / huge lengths, stuffing)
            i = rng.integers(0, len(b) - 4)
            b[i:i + rng.integers(2, 5)] = 0xFF
        elif kind == 2:  # truncation
            b = b[:rng.integers(0, len(b))]
        elif kind == 3:  # splice a chunk of the file elsewhere
            i, j = rng.integers(0, len(b), size=2)
            k = rng.integers(1, 64)
            b = np.concatenate([b[:i], b0[j:j + k], b[i:]])
        else:  # small integers over a 4-byte field (counts, lengths, offsets)
            i = rng.integers(0, len(b) - 4)
            b[i:i + 4] = np.frombuffer(np.uint32(rng.integers(0, 1 << 20)).tobytes(), np.uint8)
        yield b.tobytes()


def _try_pixels(native, b, h):
    frames = max(1, int(h.get("frames", 1)))
    if h["rows"] * h["cols"] * frames > _MAX_PIXELS:
        return
    for f in range(frames):
        try:
            native.dicom_pixels(b, f)
        except Exception:
            pass


def test_parser_survives_mutations(native):
    rng = np.random.default_rng(2026)
    parsed = failed = 0
    for s in _seeds(native):
        for b in _mutants(s, rng, 300):
            try:
                h = native.dicom_parse(b)
            except Exception:
                failed += 1
                continue
            parsed += 1
            _try_pixels(native, b, h)
    # both outcomes occur (the mutants are not all trivially rejected or all harmless)
    assert parsed > 100 and failed > 100


@pytest.mark.parametrize("mode,prefix", [("direct", 1024), ("direct", 16384), ("staged", 0)])
def test_file_reader_survives_mutations(native, tmp_path, mode, prefix):
    rng = np.random.default_rng(7 + prefix)
    p = tmp_path / "m.dcm"
    for s in _seeds(native)[::2]:
        for b in _mutants(s, rng, 40):
            p.write_bytes(b)
            try:
                h = native.dicom_parse(b)
                if h["rows"] * h["cols"] * max(1, int(h.get("frames", 1))) > _MAX_PIXELS:
                    continue
            except Exception:
                pass
            try:
                native.read_pixels_direct(str(p), mode, prefix, 0)
            except Exception:
                pass
            try:
                native.read_slice(str(p), 0, 0)
            except Exception:
                pass
