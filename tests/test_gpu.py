"""GPU tests (MI355X): every HIP kernel vs the plain-PyTorch fp32 reference and the C++ golden
model, engine end-to-end byte identity, CLIs, fault handling, 3D mode."""
import io
import os

import numpy as np
import pytest
import torch

import nm03_capstone_project_amd as nm
from nm03_capstone_project_amd import ops
from nm03_capstone_project_amd.ops import reference as R

from conftest import run_bin

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _require_gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    # The native extension must be the one actually running (no silent fallback).
    assert nm.native().device_count() >= 1


def _phantom(native, h=256, w=256, p=3, s=12, seed=7):
    return native.phantom_slice(h, w, p, s, 25, seed)


# ---------------------------------------------------------------------------------------------
# K1a median
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("k", [3, 5, 7, 9])
@pytest.mark.parametrize("shape", [(256, 256), (130, 100), (512, 512), (64, 200)])
def test_median_kernel_vs_torch_and_golden(native, k, shape):
    h, w = shape
    raw = _phantom(native, h, w)
    t = torch.from_numpy(raw.view(np.int16)).cuda()
    med = ops.median2d(t, k).cpu().numpy().view(np.uint16)
    assert np.array_equal(med, native.golden_median_u16(raw, k))
    ref = R.median(torch.from_numpy(raw.astype(np.float32)).cuda(), k).cpu().numpy()
    assert np.array_equal(med.astype(np.float32), ref)


def test_median_kernel_batched_random_full_range(native):
    rng = np.random.default_rng(1)
    raw = rng.integers(0, 65536, size=(5, 128, 192), dtype=np.uint16)
    t = torch.from_numpy(raw.view(np.int16)).cuda()
    med = ops.median2d(t, 7).cpu().numpy().view(np.uint16)
    for i in range(5):
        assert np.array_equal(med[i], native.golden_median_u16(raw[i], 7))


def test_median_signed_and_stored_bits(native):
    rng = np.random.default_rng(2)
    vals = rng.integers(-2048, 2048, size=(100, 120)).astype(np.int16)
    raw = vals.view(np.uint16) & np.uint16(0x0FFF)  # 12-bit two's complement in a 16-bit container
    t = torch.from_numpy(raw.view(np.int16)).cuda()
    med = ops.median2d(t, 5, pixel_type="i16", stored_bits=12).cpu().numpy().view(np.uint16)
    keys = ((vals.astype(np.int32) & 0xFFFF) ^ 0x8000).astype(np.uint16)  # order-preserving keys
    assert np.array_equal(med, native.golden_median_u16(keys, 5))


# ---------------------------------------------------------------------------------------------
# K1b sharpen + band
# ---------------------------------------------------------------------------------------------
def test_sharpen_band_vs_golden_and_torch(native):
    raw = _phantom(native)
    mk = native.golden_median_u16(raw, 7)
    t = torch.from_numpy(mk.view(np.int16)).cuda()
    s, band = ops.sharpen_band(t)
    s = s.cpu().numpy()
    p = native.PipelineParams()
    c = native.golden_norm_clip(mk, "u16", 16, 1.0, 0.0, p)
    gs = native.golden_sharpen(c, 2.0, 0.5, 9, False)
    assert np.array_equal(s, gs)  # bit-exact: same separable order, one fma per tap on both sides
    ref = R.sharpen(torch.from_numpy(c)).numpy()
    assert np.abs(s - ref).max() < 2e-6
    assert np.array_equal(band.cpu().numpy(), (gs >= np.float32(0.74)) & (gs <= np.float32(0.91)))


@pytest.mark.parametrize("shape", [(150, 203), (64, 320), (64, 130)])
def test_sharpen_band_odd_size_rescale(native, shape):
    """Odd widths (per-pixel staging) and odd tile counts (a workgroup takes two 64×64 tiles; the
    last one may have a single tile)."""
    raw = _phantom(native, *shape)
    mk = native.golden_median_u16(raw, 7)
    t = torch.from_numpy(mk.view(np.int16)).cuda()
    s, band = ops.sharpen_band(t, slope=1.25, intercept=-40.0)
    p = native.PipelineParams()
    c = native.golden_norm_clip(mk, "u16", 16, 1.25, -40.0, p)
    gs = native.golden_sharpen(c, 2.0, 0.5, 9, False)
    assert np.array_equal(s.cpu().numpy(), gs)


def test_sharpen_band_batched_odd_tile_count(native):
    """3 slices × 3 tiles: workgroups whose two tiles belong to different slices, and a last
    workgroup with one tile."""
    raws = [_phantom(native, 64, 192) for _ in range(3)]
    raws[1] = raws[1][:, ::-1].copy()
    raws[2] = (raws[2] // 2).astype(np.uint16)
    mks = np.stack([native.golden_median_u16(r, 7) for r in raws])
    s, band = ops.sharpen_band(torch.from_numpy(mks.view(np.int16)).cuda())
    p = native.PipelineParams()
    for i in range(3):
        gs = native.golden_sharpen(native.golden_norm_clip(mks[i], "u16", 16, 1.0, 0.0, p), 2.0, 0.5, 9, False)
        assert np.array_equal(s[i].cpu().numpy(), gs)
        assert np.array_equal(band[i].cpu().numpy(), (gs >= np.float32(0.74)) & (gs <= np.float32(0.91)))


# ---------------------------------------------------------------------------------------------
# K2 SRG + morphology
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("conn", [4, 8])
@pytest.mark.parametrize("shape,density", [((256, 256), 0.55), ((512, 512), 0.6), ((131, 77), 0.5), ((256, 256), 0.7)])
def test_region_grow_kernel_vs_golden(native, conn, shape, density):
    h, w = shape
    rng = np.random.default_rng(h * w + conn)
    band = rng.random(shape) < density
    seeds = [(x, y, 0) for (x, y) in native.reference_seeds(w, h)]
    cfg = nm.PipelineConfig(srg_connectivity=conn)
    out = ops.region_grow(torch.from_numpy(band).cuda(), seeds, cfg)
    g = native.golden_region_grow(band.astype(np.uint8), seeds, conn)
    assert np.array_equal(out["region"].cpu().numpy(), g.astype(bool))
    assert np.array_equal(out["dilated"].cpu().numpy(), native.golden_morph(g, 3, True).astype(bool))
    assert np.array_equal(out["eroded"].cpu().numpy(), native.golden_morph(g, 3, False).astype(bool))
    assert np.array_equal(out["border_region"].cpu().numpy(), native.golden_border(g, 2).astype(bool))
    ref = R.region_grow(torch.from_numpy(band).cuda(), seeds, conn).cpu().numpy()
    assert np.array_equal(out["region"].cpu().numpy(), ref)


@pytest.mark.parametrize("shape", [(600, 520), (1024, 768)])
def test_region_grow_above_lds_limit(native, shape):
    """Slices above 512: K2 runs on global-memory bit planes, same results as the golden model."""
    h, w = shape
    rng = np.random.default_rng(h + w)
    band = rng.random(shape) < 0.58
    seeds = [(x, y, 0) for (x, y) in native.reference_seeds(w, h)]
    out = ops.region_grow(torch.from_numpy(band).cuda(), seeds)
    g = native.golden_region_grow(band.astype(np.uint8), seeds, 4)
    assert np.array_equal(out["region"].cpu().numpy(), g.astype(bool))
    assert np.array_equal(out["dilated"].cpu().numpy(), native.golden_morph(g, 3, True).astype(bool))
    assert np.array_equal(out["border_region"].cpu().numpy(), native.golden_border(g, 2).astype(bool))


def test_engine_large_slice_bit_exact(native):
    """A 768×1024 slice end to end (every stage, renders, JPEGs) on the engine = golden model."""
    raw = native.phantom_slice(768, 1024, 2, 5, 11, 3)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": 1.0, "spacing_y": 1.0}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2, max_dim=1024))
    gpu = pipe.run_array(raw, meta)
    ref = pipe.golden(raw, meta)
    for k in ("band", "region", "dilated", "eroded"):
        assert np.array_equal(gpu[k], ref[k]), k
    assert gpu["jpegs"][0] == ref["jpeg_original"]
    assert gpu["jpegs"][4] == ref["jpeg_processed"]


def test_region_grow_spiral_needs_many_turns(native):
    """A 1-pixel spiral corridor forces many alternations of horizontal/vertical run fills."""
    h = w = 128
    band = np.zeros((h, w), bool)
    lo, hi = 2, w - 3
    y = x = 2
    while lo < hi:
        band[lo, lo:hi + 1] = True
        band[lo:hi + 1, hi] = True
        band[hi, lo:hi + 1] = True
        band[lo + 2:hi + 1, lo] = True
        band[lo + 2, lo:lo + 3] = True
        lo += 4
        hi -= 4
    seeds = [(2, 2, 0)]
    out = ops.region_grow(torch.from_numpy(band).cuda(), seeds)
    g = native.golden_region_grow(band.astype(np.uint8), seeds, 4)
    assert np.array_equal(out["region"].cpu().numpy(), g.astype(bool))


# ---------------------------------------------------------------------------------------------
# K4 JPEG
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("kind", ["noise", "phantom", "labels", "black"])
def test_jpeg_kernel_vs_golden_and_libjpeg(native, kind):
    rng = np.random.default_rng(3)
    if kind == "noise":
        c = rng.integers(0, 256, size=(3, 512, 512), dtype=np.uint8)
    elif kind == "black":
        c = np.zeros((2, 512, 512), np.uint8)
    else:
        raw = _phantom(native).astype(np.float32)
        g = native.golden_render_gray(raw, float(raw.min()), float(raw.max()), 1.0, 1.0, 512, 512)
        if kind == "labels":
            g = np.where(g > 140, 153, 0).astype(np.uint8)
            g[::37] = 255
        c = np.stack([g, g[::-1].copy()])
    outs = ops.jpeg_encode(torch.from_numpy(c).cuda(), 75)
    for i in range(c.shape[0]):
        assert outs[i] is not None
        assert outs[i] == native.jpeg_encode_gray420(c[i], 75)
    PIL = pytest.importorskip("PIL.Image")
    bio = io.BytesIO()
    PIL.fromarray(c[0]).convert("RGB").save(bio, format="JPEG", quality=75)
    assert outs[0] == bio.getvalue()


@pytest.mark.parametrize("sampling", [1, 2])
@pytest.mark.parametrize("shape", [(3, 512, 512), (2, 48, 80), (2, 272, 400)])
def test_jpeg_kernel_other_samplings(native, sampling, shape):
    """--jpeg-sampling 444 / gray on K4: raster-order MCUs (workgroups start mid-row: the
    predecessor DC of a part), byte-identical to the golden encoder and to libjpeg via Pillow."""
    rng = np.random.default_rng(sampling * 7 + shape[1])
    c = rng.integers(0, 256, size=shape, dtype=np.uint8)
    c[1, : shape[1] // 2] = np.where(c[1, : shape[1] // 2] > 128, 153, 0)  # flat label-like half
    outs = ops.jpeg_encode(torch.from_numpy(c).cuda(), 75, sampling=sampling)
    PIL = pytest.importorskip("PIL.Image")
    for i in range(shape[0]):
        assert outs[i] is not None
        assert outs[i] == native.jpeg_encode_gray(c[i], 75, sampling)
        bio = io.BytesIO()
        if sampling == 2:
            PIL.fromarray(c[i]).save(bio, format="JPEG", quality=75)
        else:
            PIL.fromarray(c[i]).convert("RGB").save(bio, format="JPEG", quality=75, subsampling=0)
        assert outs[i] == bio.getvalue()


def test_jpeg_capacity_overflow_reports(native):
    # 1024×1024 noise exceeds the per-image staging cap → None (callers fall back to the CPU)
    c = np.random.default_rng(0).integers(0, 256, size=(1, 1024, 1024), dtype=np.uint8)
    outs = ops.jpeg_encode(torch.from_numpy(c).cuda(), 100)
    assert outs[0] is None or outs[0] == native.jpeg_encode_gray420(c[0], 100)


# ---------------------------------------------------------------------------------------------
# Engine: every stage of one slice vs the golden model
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("shape,spacing", [((256, 256), (1.0, 1.0)), ((200, 160), (0.9, 1.2)), ((512, 512), (0.5, 0.5))])
def test_engine_single_all_stages_bit_exact(native, shape, spacing):
    h, w = shape
    raw = _phantom(native, h, w)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": spacing[0],
            "spacing_y": spacing[1]}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2))
    gpu = pipe.run_array(raw, meta)
    ref = pipe.golden(raw, meta)
    assert np.array_equal(gpu["sharpened"], ref["sharpened"])
    for k in ("band", "region", "dilated", "eroded"):
        assert np.array_equal(gpu[k], ref[k].astype(bool)), k
    assert gpu["jpegs"][0] == ref["jpeg_original"]
    assert gpu["jpegs"][4] == ref["jpeg_processed"]
    for j in gpu["jpegs"]:
        assert j[:2] == b"\xff\xd8" and j[-2:] == b"\xff\xd9"


def test_engine_signed_rescaled(native):
    raw = (_phantom(native).astype(np.int32) - 300).astype(np.int16).view(np.uint16)
    meta = {"type": "i16", "stored_bits": 16, "slope": 1.5, "intercept": 100.0}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2))
    gpu, ref = pipe.run_array(raw, meta), pipe.golden(raw, meta)
    for k in ("band", "region", "dilated"):
        assert np.array_equal(gpu[k], ref[k].astype(bool)), k
    assert gpu["jpegs"][0] == ref["jpeg_original"] and gpu["jpegs"][4] == ref["jpeg_processed"]


# ---------------------------------------------------------------------------------------------
# Engine: cohort runs, configurations agree byte-for-byte with each other and the golden model
# ---------------------------------------------------------------------------------------------
def _items(native, root, out):
    base = native.cohort_dir(root)
    items = []
    for pid in native.find_patient_dirs(base):
        _, files = native.list_patient_series(base, pid)
        od = os.path.join(out, pid)
        os.makedirs(od, exist_ok=True)
        items += [(f, od) for f in files]
    return items


def _tree(d):
    res = {}
    for dp, _, fs in os.walk(d):
        for f in fs:
            p = os.path.join(dp, f)
            res[os.path.relpath(p, d)] = open(p, "rb").read()
    return res


def test_engine_cohort_configs_identical(native, cohort_root, tmp_path):
    trees = []
    # (batch, streams, threads, passes through one engine): a second pass rewrites existing files.
    for i, (b, s, t, g) in enumerate([(1, 1, 1, 1), (25, 3, 8, 2), (7, 2, 4, 1), (64, 4, 16, 2), (64, 4, 16, 1)]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)
        ec = nm.PipelineConfig(batch_size=b, streams=s, threads=t).engine_config()
        eng = native.Engine(ec)
        for _ in range(g):
            st, times = eng.run(items)
            assert all(code == 0 for code, _ in st), st
            assert times["slices_ok"] == len(items) and times["jpeg_fallbacks"] == 0
        trees.append(_tree(out))
    assert len(trees[0]) == 2 * len(items)
    for t in trees[1:]:
        assert t == trees[0]
    # spot-check against the golden model
    f, _ = items[len(items) // 2]
    raw, meta = native.read_slice(f)
    g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                          native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
    stem = os.path.splitext(os.path.basename(f))[0]
    pid = os.path.basename(os.path.dirname(os.path.dirname(f)))
    assert trees[0][f"{pid}/{stem}_original.jpg"] == g["jpeg_original"]
    assert trees[0][f"{pid}/{stem}_processed.jpg"] == g["jpeg_processed"]


def test_engine_submit_pipelines_runs_identically(native, cohort_root, tmp_path):
    """Queued runs (Engine.submit/wait, several in flight, the slots moving on to run k+1 while run
    k drains) write exactly what blocking runs write, and report per-run statuses and times."""
    ref_out = str(tmp_path / "ref")
    ref_items = _items(native, cohort_root, ref_out)
    eng = native.Engine(nm.PipelineConfig(batch_size=5, streams=3, threads=8).engine_config())
    st, _ = eng.run(ref_items)
    assert all(code == 0 for code, _ in st)
    ref = _tree(ref_out)
    outs = [str(tmp_path / f"q{k}") for k in range(4)]
    works = [native.WorkList(_items(native, cohort_root, o)) for o in outs]
    tickets = [eng.submit(w) for w in works]  # four runs queued at once
    for t, w in zip(tickets, works):
        codes, msgs, times = eng.wait(t)
        assert len(codes) == len(w) and not msgs and times["slices_ok"] == len(w)
        assert times["batches"] == -(-len(w) // 5)
    for o in outs:
        assert _tree(o) == ref
    # an empty run completes at once; a run after the queue drained still works
    codes, msgs, times = eng.wait(eng.submit(native.WorkList([])))
    assert len(codes) == 0 and times["batches"] == 0
    codes, msgs, _ = eng.run_list(works[0])
    assert not msgs


def test_engine_jpeg_cpu_fallback_identical(native, cohort_root, tmp_path):
    """Every image overflowing the GPU encoder's output capacity (EngineConfig.jpeg_out_cap tiny)
    goes through the host re-encode fallback — under 4 concurrent slots — and the files are
    byte-identical to the GPU-encoded ones; the fallbacks are counted."""
    ref_out = str(tmp_path / "ref")
    items = _items(native, cohort_root, ref_out)
    cfg = nm.PipelineConfig(batch_size=6, streams=4, threads=8).engine_config()
    st, t = native.Engine(cfg).run(items)
    assert all(c == 0 for c, _ in st) and t["jpeg_fallbacks"] == 0
    cfg.jpeg_out_cap = 2048
    fb_out = str(tmp_path / "fb")
    st, t = native.Engine(cfg).run(_items(native, cohort_root, fb_out))
    assert all(c == 0 for c, _ in st)
    assert t["jpeg_fallbacks"] == 2 * len(items)
    assert _tree(fb_out) == _tree(ref_out)


def test_engine_fault_isolation(native, tmp_path):
    d = tmp_path / "series"
    d.mkdir()
    good = native.phantom_slice(256, 256, 1, 5, 25, 1)
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(good))
    (d / "1-2.dcm").write_bytes(b"DICM-but-not-really" * 10)
    (d / "1-3.dcm").write_bytes(native.dicom_bytes(np.zeros((64, 64), np.uint16)))  # < 100 guard
    (d / "1-4.dcm").write_bytes(native.dicom_bytes(good[::-1].copy()))
    out = tmp_path / "out"
    out.mkdir()
    items = [(str(d / f"1-{i}.dcm"), str(out)) for i in range(1, 5)]
    st, times = native.Engine(nm.PipelineConfig(batch_size=4, streams=1, threads=2).engine_config()).run(items)
    codes = [c for c, _ in st]
    assert codes == [0, 1, 2, 0]
    assert "too small" in st[2][1]
    assert sorted(p.name for p in out.iterdir()) == ["1-1_original.jpg", "1-1_processed.jpg", "1-4_original.jpg",
                                                     "1-4_processed.jpg"]
    # compact hot-loop form: same codes, messages only for the failures
    eng = native.Engine(nm.PipelineConfig(batch_size=2, streams=2, threads=2).engine_config())
    codes, msgs, t2 = eng.run_list(native.WorkList(items))
    assert codes.tolist() == [0, 1, 2, 0] and sorted(msgs) == [1, 2] and "too small" in msgs[2]
    assert t2["slices_ok"] == 2 and t2["slices_failed"] == 2


def test_engine_flat_label_waves_vs_golden(native, tmp_path):
    """Label images whose waves are one flat colour skip the FDCT, quantisation and zig-zag walk
    (k4_jpeg.hip): every exported JPEG — all-background label images (uniform and
    noise-only slices: no region grows), phantom slices with a partial region, and a slice whose
    region fills most of the canvas — is byte-identical to the golden encoder's."""
    d = tmp_path / "series"
    d.mkdir()
    rng = np.random.default_rng(5)
    slices = [np.zeros((256, 256), np.uint16), np.full((256, 256), 1000, np.uint16),
              rng.integers(0, 40, (256, 256), dtype=np.uint16)]
    slices += [native.phantom_slice(256, 256, p, s, 23, 7) for p, s in ((0, 3), (1, 11), (2, 20))]
    bright = native.phantom_slice(256, 256, 3, 11, 23, 7).astype(np.float64)
    slices.append(np.clip(bright * 1.6, 0, 4095).astype(np.uint16))  # most of the head in the SRG band
    out = tmp_path / "out"
    out.mkdir()
    items = []
    for i, a in enumerate(slices, start=1):
        (d / f"1-{i}.dcm").write_bytes(native.dicom_bytes(a))
        items.append((str(d / f"1-{i}.dcm"), str(out)))
    st, times = native.Engine(nm.PipelineConfig(batch_size=8, streams=1, threads=2).engine_config()).run(items)
    assert all(c == 0 for c, _ in st), st
    assert times["jpeg_fallbacks"] == 0
    for f, _ in items:
        raw, meta = native.read_slice(f)
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = os.path.splitext(os.path.basename(f))[0]
        assert (out / f"{stem}_original.jpg").read_bytes() == g["jpeg_original"], stem
        assert (out / f"{stem}_processed.jpg").read_bytes() == g["jpeg_processed"], stem


def test_engine_flat_label_workgroups_vs_golden(native, tmp_path):
    """Whole label workgroups of one level (k4_jpeg.hip wgflat: the bit range filled with the
    0x28A28A00 MCU pattern, no render, coding or scan) next to workgroups that code normally: a slice
    entirely in the SRG band (every workgroup flat at the fill level, the image's first DC difference
    ≠ 0), half-band slices (fill above, background below: the boundary workgroup codes the border and
    the next flat workgroup starts with a large negative DC difference), stripes, and a 264×256 slice
    (the label canvas is not an exact 2× fit: generic path). Byte-identical to the golden encoder."""
    d = tmp_path / "series"
    d.mkdir()
    full = np.full((256, 256), 1500, np.uint16)
    half = np.zeros((256, 256), np.uint16)
    half[:128] = 1500
    halfb = np.zeros((256, 256), np.uint16)
    halfb[128:] = 1500
    stripes = np.zeros((256, 256), np.uint16)
    stripes[::40] = 1500
    stripes[:, 100:140] = 1500
    odd = np.full((264, 256), 1500, np.uint16)
    odd[200:] = 0
    out = tmp_path / "out"
    out.mkdir()
    items = []
    for i, a in enumerate([full, half, halfb, stripes, odd], start=1):
        (d / f"1-{i}.dcm").write_bytes(native.dicom_bytes(a))
        items.append((str(d / f"1-{i}.dcm"), str(out)))
    st, times = native.Engine(nm.PipelineConfig(batch_size=8, streams=1, threads=2).engine_config()).run(items)
    assert all(c == 0 for c, _ in st), st
    assert times["jpeg_fallbacks"] == 0
    for f, _ in items:
        raw, meta = native.read_slice(f)
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = os.path.splitext(os.path.basename(f))[0]
        assert (out / f"{stem}_processed.jpg").read_bytes() == g["jpeg_processed"], stem
        assert (out / f"{stem}_original.jpg").read_bytes() == g["jpeg_original"], stem


def test_engine_pack12_identical(native, cohort_root, tmp_path, monkeypatch):
    """12-bit transfer packing (nm03/pack12.h + K0 unpack) on vs off: byte-identical JPEGs and the
    same statuses, on batches mixing packable 12-bit slices, a slice with 13-bit samples (shipped as
    16-bit), an odd-sized slice (n % 16 != 0, shipped as 16-bit) and a corrupt file."""
    d = tmp_path / "mixed"
    d.mkdir()
    hi = native.phantom_slice(256, 256, 4, 11, 25, 9).astype(np.uint32) + 3000
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(np.minimum(hi, 65535).astype(np.uint16)))
    (d / "1-2.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(150, 203, 2, 7, 25, 3)))
    (d / "1-3.dcm").write_bytes(b"DICM-but-not-really" * 10)
    runs = []
    for i, flag in enumerate(["0", "1"]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:30]
        os.makedirs(os.path.join(out, "mixed"), exist_ok=True)
        extra = [(str(d / f"1-{k}.dcm"), os.path.join(out, "mixed")) for k in range(1, 4)]
        items = items[:5] + extra + items[5:]
        monkeypatch.setenv("NM03_PACK12", flag)
        eng = native.Engine(nm.PipelineConfig(batch_size=8, streams=2, threads=4).engine_config())
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    assert runs[0][0] == runs[1][0] and runs[0][0].count(0) == len(runs[0][0]) - 1
    assert runs[0][1] == runs[1][1]


def test_engine_pack12_holes_and_stored_bits(native, cohort_root, tmp_path, monkeypatch):
    """Loader packing paths (engine.cpp load_one) vs no packing: wide 16-bit slices interleaved with
    fitting ones in the same batches (the checked single-pass pack then grows its reservation in
    place or abandons it as a hole), BitsStored = 12 slices whose high 4 bits hold garbage (packed
    unconditionally: every consumer masks to the stored bits), a signed 12-bit slice, and a batch
    with more wide slices than loader threads. Same statuses, byte-identical JPEGs."""
    d = tmp_path / "mixed"
    d.mkdir()
    rng = np.random.default_rng(7)
    files = []
    for k in range(12):
        base = native.phantom_slice(256, 256, 4, 11, 25, 9 + k).astype(np.uint32)
        if k % 3 == 0:  # wide: one sample (anywhere) above 12 bits
            px = base.copy()
            px.flat[int(rng.integers(0, px.size))] = 4096 + k
            blob = native.dicom_bytes(np.minimum(px, 65535).astype(np.uint16))
        elif k % 3 == 1:  # BitsStored 12, garbage in the high nibble
            px = (base & 0xFFF) | (rng.integers(0, 16, size=base.shape, dtype=np.uint32) << 12)
            blob = native.dicom_bytes(px.astype(np.uint16), "u16", 12)
        else:  # signed 12-bit, sign-extended words
            v = (base.astype(np.int32) % 4096) - 2048
            blob = native.dicom_bytes((v & 0xFFFF).astype(np.uint16), "i16", 12)
        f = d / f"1-{k + 1}.dcm"
        f.write_bytes(blob)
        files.append(f)
    runs = []
    for i, flag in enumerate(["0", "1"]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:12]
        os.makedirs(os.path.join(out, "mixed"), exist_ok=True)
        extra = [(str(f), os.path.join(out, "mixed")) for f in files]
        items = [x for pair in zip(items, extra) for x in pair]
        monkeypatch.setenv("NM03_PACK12", flag)
        eng = native.Engine(nm.PipelineConfig(batch_size=16, streams=2, threads=8).engine_config())
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    assert runs[0][0] == runs[1][0] and runs[0][0].count(0) == len(runs[0][0])
    assert runs[0][1] == runs[1][1]


def test_engine_mixed_blob_layouts_identical(native, cohort_root, tmp_path, monkeypatch):
    """The median decodes the upload in its tile load (12-bit pairs, plain 16-bit) and writes the
    expanded samples for the render: batches mixing packed slices, a 13-bit slice (plain 16-bit
    blob, vector loads), an odd-sized slice (plain blob, W % 4 != 0: per-pixel loads) and a packed
    200×112 slice (partial edge tiles in x and y) give the same JPEGs with 12-bit packing on and off,
    and the mixed slices match the golden model."""
    d = tmp_path / "mixed"
    d.mkdir()
    hi = native.phantom_slice(256, 256, 4, 11, 25, 9).astype(np.uint32) + 3000
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(np.minimum(hi, 65535).astype(np.uint16)))
    (d / "1-2.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(150, 203, 2, 7, 25, 3)))
    (d / "1-3.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(112, 200, 2, 9, 25, 5)))
    runs = []
    for i, flag in enumerate(["1", "0"]):
        monkeypatch.setenv("NM03_PACK12", flag)
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:20]
        os.makedirs(os.path.join(out, "mixed"), exist_ok=True)
        extra = [(str(d / f"1-{k}.dcm"), os.path.join(out, "mixed")) for k in range(1, 4)]
        items = items[:5] + extra + items[5:]
        eng = native.Engine(nm.PipelineConfig(batch_size=8, streams=2, threads=4).engine_config())
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    assert runs[0][0] == runs[1][0] and runs[0][0].count(0) == len(runs[0][0])
    assert runs[0][1] == runs[1][1]
    for k in range(1, 4):
        f = str(d / f"1-{k}.dcm")
        raw, meta = native.read_slice(f)
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        assert runs[0][1][f"mixed/1-{k}_processed.jpg"] == g["jpeg_processed"]
        assert runs[0][1][f"mixed/1-{k}_original.jpg"] == g["jpeg_original"]


def test_engine_norm_tables_vs_golden(native, tmp_path):
    """K1b's normalise+clip lookup tables (engine.cpp norm_lut: one per (type, stored bits, slope,
    intercept), built on the host with norm_clip_key): one batch mixing unsigned 16/12/8-bit,
    signed 12/16-bit and rescaled slices (six distinct tables, two slices each) gives the golden
    model's masks and JPEGs for every slice."""
    d = tmp_path / "mix"
    d.mkdir()
    specs = [("u16", 16, False, 1.0, 0.0), ("u16", 12, False, 1.0, 0.0), ("i16", 12, False, 1.0, 0.0),
             ("i16", 16, True, 1.5, 100.0), ("u16", 16, True, 0.75, -20.0), ("u8", 8, False, 1.0, 0.0)]
    files = []
    for k, (ty, bits, resc, slope, icpt) in enumerate(specs * 2):
        base = native.phantom_slice(256, 256, 2, 5 + k, 25, 11 + k).astype(np.int32)
        if ty == "i16":
            v = (base % (1 << bits)) - (1 << (bits - 1))
            px = (v & 0xFFFF).astype(np.uint16)
        elif ty == "u8":
            px = (base >> 4).astype(np.uint16) & 0xFF
        else:
            px = (base & ((1 << bits) - 1)).astype(np.uint16)
        f = d / f"1-{k + 1}.dcm"
        f.write_bytes(native.dicom_bytes(px, ty, bits, resc, slope, icpt))
        files.append(f)
    out = tmp_path / "o"
    out.mkdir()
    eng = native.Engine(nm.PipelineConfig(batch_size=16, streams=1, threads=4).engine_config())
    st, _ = eng.run([(str(f), str(out)) for f in files])
    assert [c for c, _ in st] == [0] * len(files)
    for f in files:
        raw, meta = native.read_slice(str(f))
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = f.name[:-4]
        assert (out / f"{stem}_processed.jpg").read_bytes() == g["jpeg_processed"], stem
        assert (out / f"{stem}_original.jpg").read_bytes() == g["jpeg_original"], stem


def test_engine_norm_table_arena_full_vs_golden(native, tmp_path):
    """More distinct 16-bit rescale sets than the table arena holds (16 tables of 2^16 keys): the
    later slices run with lut_off = kNoLut, i.e. K1b evaluates normalise+clip itself — same masks
    and JPEGs as the golden model either way."""
    d = tmp_path / "many"
    d.mkdir()
    files = []
    for k in range(20):
        px = native.phantom_slice(256, 256, 3, 7 + k, 25, 31 + k).astype(np.uint16)
        f = d / f"1-{k + 1}.dcm"
        f.write_bytes(native.dicom_bytes(px, "u16", 16, True, 1.0 + 0.05 * k, -10.0 * k))
        files.append(f)
    out = tmp_path / "o"
    out.mkdir()
    eng = native.Engine(nm.PipelineConfig(batch_size=8, streams=2, threads=4).engine_config())
    st, _ = eng.run([(str(f), str(out)) for f in files])
    assert [c for c, _ in st] == [0] * len(files)
    for f in files:
        raw, meta = native.read_slice(str(f))
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = f.name[:-4]
        assert (out / f"{stem}_processed.jpg").read_bytes() == g["jpeg_processed"], stem
        assert (out / f"{stem}_original.jpg").read_bytes() == g["jpeg_original"], stem


def test_engine_jpeg_batch_sizes_identical(native, tmp_path):
    """JPEG encoder launches of bench size (96 slices = 192 images, 16 workgroups per gray image)
    vs batches of 16, and a capacity edge: byte-identical trees on a 100-slice cohort plus flat /
    half-band / odd-sized label images. (A 512-block workgroup variant, measured no faster and
    removed, once hung such a batch on the box through an LDS overrun: gpurun_out/r4g.)"""
    d = tmp_path / "extra"
    d.mkdir()
    full = np.full((256, 256), 1500, np.uint16)
    half = np.zeros((256, 256), np.uint16)
    half[:128] = 1500
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(full))
    (d / "1-2.dcm").write_bytes(native.dicom_bytes(half))
    (d / "1-3.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(150, 203, 2, 7, 25, 3)))
    cohort = str(tmp_path / "data") + "/"
    native.synth_cohort(cohort, patients=6, min_slices=16, max_slices=20, threads=4)
    runs = []
    for i, (bs, cap) in enumerate([(96, 0), (16, 0), (96, 20000)]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort, out)
        os.makedirs(os.path.join(out, "extra"), exist_ok=True)
        items = items[:5] + [(str(d / f"1-{k}.dcm"), os.path.join(out, "extra")) for k in (1, 2, 3)] + items[5:]
        ec = nm.PipelineConfig(batch_size=bs, streams=1, threads=4).engine_config()
        ec.jpeg_out_cap = cap
        eng = native.Engine(ec)
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    for r in runs[1:]:
        assert r[0] == runs[0][0] and r[0].count(0) == len(r[0])
        diffs = sorted(k for k in runs[0][1] if r[1].get(k) != runs[0][1][k])[:4]
        assert not diffs, diffs


def test_engine_jpeg_capacity_edge_identical(native, cohort_root, tmp_path):
    """Output capacity at the edge of real segment sizes (20000 bytes: some images fit, some
    overflow mid-image and take the CPU re-encode): statuses and trees identical to the default
    capacity. Guards the encoder's exact end-of-range capacity check (a conservative bound once
    let a workgroup drop its bytes while the image still reported a size)."""
    runs = []
    for i, cap in enumerate([0, 20000]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:40]
        ec = nm.PipelineConfig(batch_size=8, streams=2, threads=4).engine_config()
        ec.jpeg_out_cap = cap
        eng = native.Engine(ec)
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    assert runs[1][0] == runs[0][0] and runs[0][0].count(0) == len(runs[0][0])
    diffs = sorted(k for k in runs[0][1] if runs[1][1].get(k) != runs[0][1][k])[:4]
    assert not diffs, diffs


def test_engine_progressive_upload_identical(native, cohort_root, tmp_path):
    """Progressive H2D (finished prefixes of a batch's raw region queued while loads run) with
    1 KiB / 64 KiB chunks vs one upload per batch: same statuses, byte-identical JPEGs, on a work
    list mixing slice sizes with unreadable and too-small files (failed loads leave holes in the
    allocation order)."""
    d = tmp_path / "extra"
    d.mkdir()
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(160, 200, 2, 7, 25, 3)))
    (d / "1-2.dcm").write_bytes(b"DICM-but-not-really" * 10)
    (d / "1-3.dcm").write_bytes(native.dicom_bytes(np.zeros((64, 64), np.uint16)))
    (d / "1-4.dcm").write_bytes(native.dicom_bytes(native.phantom_slice(512, 384, 3, 9, 25, 4)))
    runs = []
    for i, kb in enumerate([0, 1, 64]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:40]
        os.makedirs(os.path.join(out, "extra"), exist_ok=True)
        extra = [(str(d / f"1-{k}.dcm"), os.path.join(out, "extra")) for k in range(1, 5)]
        items = items[:9] + extra[:2] + items[9:30] + extra[2:] + items[30:]
        ec = nm.PipelineConfig(batch_size=16, streams=3, threads=4).engine_config()
        ec.upload_chunk_kb = kb
        eng = native.Engine(ec)
        st, _ = eng.run(items)
        del eng
        runs.append(([c for c, _ in st], _tree(out)))
    assert runs[0][0].count(0) == len(runs[0][0]) - 2
    for codes, tree in runs[1:]:
        assert codes == runs[0][0]
        assert tree == runs[0][1]


def test_engine_batch_cap_identical(native, cohort_root, tmp_path):
    """The batch cap of the single-pass measurement (run_list(items, cap): small batches, inline
    uploads on the slot's own stream, spin-polled completion) vs full batches: same statuses,
    byte-identical trees."""
    runs = []
    for i, cap in enumerate([0, 5, 16]):
        out = str(tmp_path / f"o{i}")
        items = _items(native, cohort_root, out)[:37]
        eng = native.Engine(nm.PipelineConfig(batch_size=16, streams=3, threads=4).engine_config())
        codes, msgs, _ = eng.run_list(native.WorkList(items), cap)
        del eng
        runs.append((list(codes), _tree(out)))
    assert runs[0][0].count(0) == len(runs[0][0])
    for codes, tree in runs[1:]:
        assert codes == runs[0][0]
        assert tree == runs[0][1]


def test_cli_sequential_equals_parallel(native, cohort_root, tmp_path):
    seq, par = tmp_path / "out-sequential", tmp_path / "out-parallel"
    r1 = run_bin("img_processing_sequential", "--data-root", cohort_root, "--out", str(seq))
    assert r1.returncode == 0, r1.stderr
    r2 = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(par))
    assert r2.returncode == 0, r2.stderr
    t1, t2 = _tree(str(seq)), _tree(str(par))
    assert t1 == t2 and len(t1) > 0
    for line in ("=== Starting Sequential Processing for All Patients ===", "Found 4 patient directories.",
                 "=== Processing Patient: PGBM-001 ===", "Created clean output directory: ", "Using series directory: ",
                 'Processing: "1-01.dcm"', "completed. Successfully processed", "=== All Processing Completed ===",
                 "Successfully processed 4/4 patients."):
        assert line in r1.stdout, line
    for line in ("=== Starting Parallel Processing for All Patients ===",
                 "=== Processing Patient: PGBM-001 using Parallel Processing ===", "Created output directory: ",
                 "images to process for patient PGBM-001", "Using ", " threads", "Successfully processed 4/4 patients."):
        assert line in r2.stdout, line


# ---------------------------------------------------------------------------------------------
# Multi-rank on one GPU: N rank processes share device 0 over the host comm (RCCL refuses two
# ranks per device). Same launcher, plan broadcast, sharding, status gather and printing as an
# N-GPU run.
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("ranks", [2, 4])
def test_cli_parallel_multirank_identical(native, cohort_root, tmp_path, ranks):
    import json
    g1, gn = tmp_path / "g1", tmp_path / f"g{ranks}"
    one = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(g1), "--gpus", "1")
    assert one.returncode == 0, one.stderr
    many = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(gn), "--gpus", str(ranks),
                   "--threads", "4", "--json", str(tmp_path / "m.json"),
                   env={"NM03_DEVICE_OVERRIDE": "0", "NM03_COMM_TIMEOUT_S": "60"}, timeout=240)
    assert many.returncode == 0, many.stderr
    t1, tn = _tree(str(g1)), _tree(str(gn))
    assert t1 == tn and len(t1) > 0
    # rank 0 prints the whole cohort in patient order: identical apart from the paths and threads
    import re
    norm = lambda s, d: re.sub(r"Using \d+ threads", "Using T threads", s.replace(str(d), "OUT"))  # noqa: E731
    assert norm(one.stdout, g1) == norm(many.stdout, gn)
    j = json.load(open(tmp_path / "m.json"))
    assert j["gpus"] == ranks and j["backend"] == "host"
    pr = j["per_rank"]
    assert len(pr["slices"]) == ranks and sum(pr["slices"]) == len(t1) // 2
    assert sum(pr["slices_ok"]) == len(t1) // 2


def test_cli_copy_engine_auto_blit_and_sdma_identical(native, cohort_root, tmp_path):
    """--copy-engine: the small test cohort takes shader (blit) copies by default (auto: ≤ 4096
    slices per rank), --copy-engine sdma the DMA engines; both JSON records say which, and the
    exported trees are identical (and equal the golden model on a sample)."""
    import json
    outs = {}
    for flag in ("auto", "sdma", "blit"):
        d = tmp_path / flag
        r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(d), "--gpus", "1",
                    "--copy-engine", flag, "--json", str(tmp_path / f"{flag}.json"), env={"HSA_ENABLE_SDMA": None})
        assert r.returncode == 0, r.stderr
        j = json.load(open(tmp_path / f"{flag}.json"))
        assert j["copy_engine"] == ("sdma" if flag == "sdma" else "blit"), flag
        outs[flag] = _tree(str(d))
    assert len(outs["auto"]) > 0 and outs["auto"] == outs["sdma"] == outs["blit"]
    r = run_bin("img_processing_parallel", "--copy-engine", "dma", "--data-root", cohort_root, "--out", str(tmp_path / "x"))
    assert r.returncode == 2


def test_cli_parallel_dead_rank_fails_job(native, cohort_root, tmp_path):
    """A rank that dies mid-job (after the plan broadcast) fails the job promptly with its id."""
    import time
    t0 = time.monotonic()
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "o"), "--gpus", "3",
                "--threads", "4", env={"NM03_DEVICE_OVERRIDE": "0", "NM03_FAULT": "rank_exit:2",
                                       "NM03_COMM_TIMEOUT_S": "60"}, timeout=120)
    assert r.returncode != 0
    assert "Rank 2 exited with status 9" in r.stderr
    assert time.monotonic() - t0 < 50


def test_cli_parallel_rejects_more_gpus_than_visible(native, cohort_root, tmp_path):
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "o"), "--gpus", "64")
    assert r.returncode == 1 and "exceeds the" in r.stderr and "visible GPU" in r.stderr


def test_rccl_comm_single_rank(native):
    """The native RCCL communicator end to end on the GPU (non-blocking init, staged collectives,
    bounded waits) with one rank — a second rank needs a second GPU."""
    uid = native.rccl_unique_id()
    c = native.rccl_comm(0, 1, uid, 0, None, 30.0)
    assert c.backend == "rccl" and c.rank == 0 and c.size == 1
    c.barrier()
    assert c.broadcast_bytes(b"work-list" * 1000, 0) == b"work-list" * 1000
    assert c.allgather_bytes(b"abc") == [b"abc"]
    assert c.allreduce_sum([3, 4]) == [3, 4]
    assert c.allreduce_max([1.5]) == [1.5]
    assert c.allgather_f64([2.0, 3.0]) == [2.0, 3.0]


def test_bench_multirank_one_gpu(native, tmp_path):
    """bench.py --gpus 2 launches its own ranks (sharing GPU 0): n_gpus, weak + strong figures."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, NM03_DEVICE_OVERRIDE="0", NM03_COMM_TIMEOUT_S="60")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--threads", "8", "--numa-data", "off",
                        "--cli-runs", "2", "--single-passes", "5",
                        "--data-root", str(tmp_path / "d"), "--out-root", str(tmp_path / "o")],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert rec["n_gpus"] == 2 and rec["value"] > 0 and rec["config"]["comm"]["backend"] == "host"
    # headline: BASELINE config 3 as written (one cohort sharded); weak scaling (2 replicas) secondary
    assert rec["scaling"] == "strong"
    assert rec["config"]["weak"]["value"] > 0 and rec["config"]["weak"]["global_batch"] == 2 * rec["config"]["global_batch"]
    assert sum(rec["config"]["per_rank"]["slices_ok"]) == 2 * rec["config"]["global_batch"]  # 2 steps
    cli = rec["config"]["cli_wall"]  # the whole img_processing_parallel --gpus 2, timed twice
    assert cli["all_ok"] and cli["runs"] == 2 and cli["slices"] == rec["config"]["global_batch"], cli


def test_cli_test_pipeline_gpu_equals_cpu(native, cohort_root, tmp_path):
    a, b = tmp_path / "gpu", tmp_path / "cpu"
    r = run_bin("test_pipeline", "--data-root", cohort_root, "--out", str(a))
    assert r.returncode == 0, r.stderr
    r = run_bin("test_pipeline", "--cpu", "--data-root", cohort_root, "--out", str(b))
    assert r.returncode == 0, r.stderr
    assert _tree(str(a)) == _tree(str(b))


# ---------------------------------------------------------------------------------------------
# 3D mode
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("conn", [6, 26])
def test_volume_vs_golden(native, conn):
    d, h, w = 24, 96, 128
    vol = np.stack([native.phantom_slice(h, w, 2, z, d, 5) for z in range(d)])
    vp = nm.VolumePipeline(connectivity=conn, dilation=5)
    seeds = vp.default_seeds(vol)
    res = vp.run(vol, seeds)
    # band per slice == 2D golden band
    for z in (0, d // 2, d - 1):
        g = native.golden_run(vol[z])
        assert np.array_equal(res["band"][z], g["band"]), z
    region, dil = vp.golden(res["band"], seeds)
    assert np.array_equal(res["region"], region)
    assert np.array_equal(res["dilated"], dil)
    assert res["sweeps"] >= 1


def test_volume_cli_gpu_equals_golden(native, cohort_root, tmp_path):
    """img_processing_parallel --mode 3d: 3D SRG + 7³ dilation on the GPU and the per-plane render
    + JPEG export on the GPU (K3/K4) are byte-identical to the golden CPU 3D path; the same with the
    patients sharded over 2 ranks sharing the GPU."""
    import json
    g, c, m = tmp_path / "gpu", tmp_path / "cpu", tmp_path / "multi"
    r = run_bin("img_processing_parallel", "--mode", "3d", "--data-root", cohort_root, "--out", str(g),
                "--json", str(tmp_path / "g.json"))
    assert r.returncode == 0, r.stderr
    assert "3D region growing converged in" in r.stdout
    r = run_bin("img_processing_parallel", "--mode", "3d", "--cpu", "--data-root", cohort_root, "--out", str(c))
    assert r.returncode == 0, r.stderr
    tg, tc = _tree(str(g)), _tree(str(c))
    assert len(tg) > 0 and tg == tc
    j = json.load(open(tmp_path / "g.json"))
    assert j["backend"] == "gpu" and j["dilation_size"] == 7 and j["jpeg_fallbacks"] == 0
    assert all(p["ok"] and p["sweeps"] >= 1 and p["export_s"] > 0 for p in j["patients"])
    r = run_bin("img_processing_parallel", "--mode", "3d", "--gpus", "2", "--data-root", cohort_root, "--out", str(m),
                "--json", str(tmp_path / "m.json"), env={"NM03_DEVICE_OVERRIDE": "0", "NM03_COMM_TIMEOUT_S": "60"})
    assert r.returncode == 0, r.stderr
    assert _tree(str(m)) == tg
    j = json.load(open(tmp_path / "m.json"))
    assert j["gpus"] == 2 and len(j["per_rank_wall_s"]) == 2


def test_volume_cli_jpeg_sampling_gray_equals_golden(native, cohort_root, tmp_path):
    """--mode 3d --jpeg-sampling gray: the GPU plane export (gray instance of K4, fused renders)
    equals the golden 3D export in the same layout, and the files are one-component JPEGs."""
    g, c = tmp_path / "gpu", tmp_path / "cpu"
    for out, extra in ((g, []), (c, ["--cpu"])):
        r = run_bin("img_processing_parallel", "--mode", "3d", "--jpeg-sampling", "gray", *extra, "--data-root",
                    cohort_root, "--out", str(out))
        assert r.returncode == 0, r.stderr
    tg, tc = _tree(str(g)), _tree(str(c))
    assert len(tg) > 0 and tg == tc
    PIL = pytest.importorskip("PIL.Image")
    f = next(p for p in g.rglob("*.jpg"))
    assert PIL.open(f).mode == "L"


def test_volume_run_series_equals_golden(native, tmp_path):
    """VolumePipeline.run_series on a DICOM series directory (written out of order on disk, 1-10
    after 1-9) equals run() on the stacked planes and the golden 3D model."""
    d, h, w = 12, 64, 80
    planes = [native.phantom_slice(h, w, 2, z, d, 4) for z in range(d)]
    for z in reversed(range(d)):
        (tmp_path / f"1-{z + 1}.dcm").write_bytes(native.dicom_bytes(planes[z], instance=z + 1))
    vp = nm.VolumePipeline(connectivity=6, dilation=7)
    vol = np.stack(planes)
    res = vp.run_series(str(tmp_path))
    ref = vp.run(vol)
    for k in ("band", "region", "dilated"):
        assert np.array_equal(res[k], ref[k]), k
    region, dil = vp.golden(res["band"], vp.default_seeds(vol))
    assert np.array_equal(res["region"], region) and np.array_equal(res["dilated"], dil)


def test_volume_runner_reuse_across_shapes(native):
    """One persistent VolumePipeline runner over volumes of changing shape and content: every
    result equals the golden of that volume (no stale buffers/tables from the previous run)."""
    vp = nm.VolumePipeline(connectivity=6, dilation=3)
    for (d, h, w, seed) in ((8, 64, 64, 1), (12, 80, 96, 2), (8, 64, 64, 3), (8, 64, 64, 3)):
        vol = np.stack([native.phantom_slice(h, w, 2, z, d, seed) for z in range(d)])
        seeds = vp.default_seeds(vol)
        res = vp.run(vol, seeds)
        region, dil = vp.golden(res["band"], seeds)
        assert np.array_equal(res["region"], region), (d, h, w, seed)
        assert np.array_equal(res["dilated"], dil), (d, h, w, seed)
    assert len(vp._runners) == 1


@pytest.mark.parametrize("d,conn", [(64, 6), (16, 26)])
def test_volume_above_512_vs_golden(native, d, conn):
    """Plane sides above 512 (600 × 520): the 3D region growing runs on global-memory planes in one
    cooperative launch that decides convergence on the device, and the cube dilation on global
    scratch — bit-exact to the golden model."""
    h, w = 520, 600
    vol = np.stack([native.phantom_slice(h, w, 2, z, d, 6) for z in range(d)])
    vp = nm.VolumePipeline(connectivity=conn, dilation=7)
    seeds = vp.default_seeds(vol)
    res = vp.run(vol, seeds)
    region, dil = vp.golden(res["band"], seeds)
    assert region.sum() > 1000
    assert np.array_equal(res["region"], region)
    assert np.array_equal(res["dilated"], dil)
    assert res["sweeps"] >= 2


# ---------------------------------------------------------------------------------------------
# Fault injection / resume / log levels
# ---------------------------------------------------------------------------------------------
def test_fault_injection_isolated(native, cohort_root, tmp_path):
    import re
    base = native.cohort_dir(cohort_root)
    n_items = sum(len(native.list_patient_series(base, p)[1]) for p in native.find_patient_dirs(base))
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "o"), "--batch-size", "4",
                env={"NM03_FAULT": "corrupt_dicom:1,fail_batch:2,fail_write:0"})
    assert r.returncode == 0, r.stderr
    assert "injected fault: corrupt DICOM data" in r.stderr
    assert "injected fault: device batch failure" in r.stderr
    assert "Error in export stage: injected fault: export failure" in r.stderr
    ok = sum(int(m) for m in re.findall(r"Successfully processed (\d+)/\d+ images", r.stdout))
    assert ok == n_items - 6  # item 0 (export), item 1 (load), batch 2 = items 8..11
    assert "Successfully processed 4/4 patients." in r.stdout


def test_resume_keeps_existing(native, cohort_root, tmp_path):
    out = tmp_path / "o"
    assert run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(out)).returncode == 0
    files = sorted(out.rglob("*.jpg"))
    victim = files[3]
    victim.unlink()
    key = (victim.parent, victim.name.rsplit("_", 1)[0])  # the slice whose pair gets re-exported
    keep = {f: f.stat().st_mtime_ns for f in files if (f.parent, f.name.rsplit("_", 1)[0]) != key}
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(out), "--resume")
    assert r.returncode == 0, r.stderr
    assert victim.exists()
    assert all(f.stat().st_mtime_ns == t for f, t in keep.items())


def test_log_levels(native, cohort_root, tmp_path):
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "a"), "--quiet",
                env={"NM03_LOG": "info"})
    assert r.returncode == 0 and "[nm03 INFO] engine on device 0" in r.stdout
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "b"), "--quiet")
    assert r.returncode == 0 and "[nm03 INFO]" not in r.stdout


def test_threshold_kernel_vs_torch(native):
    from nm03_capstone_project_amd.ops import reference, threshold
    x = torch.rand(3, 97, 131, device="cuda") * 2.0  # odd total size exercises the tail path
    got = threshold(x, 0.74, 0.91)
    assert got.dtype == torch.uint8 and torch.equal(got, reference.threshold(x, 0.74, 0.91))
    y = torch.tensor([0.74, 0.91, 0.7399999, 0.9100001], device="cuda")
    assert threshold(y, 0.74, 0.91).tolist() == [1, 1, 0, 0]


def test_test_pipeline_dump_mhd_gpu_equals_cpu(native, cohort_root, tmp_path):
    for backend in ("gpu", "cpu"):
        args = ["--data-root", cohort_root, "--out", str(tmp_path / f"o_{backend}"),
                "--dump-mhd", str(tmp_path / f"m_{backend}")]
        r = run_bin("test_pipeline", *(["--cpu"] if backend == "cpu" else []), *args)
        assert r.returncode == 0, r.stderr
    for name in ("input", "sharpened", "band", "segmentation", "erosion", "dilation"):
        a, _ = native.mhd_read(str(tmp_path / "m_gpu" / f"{name}.mhd"))
        b, _ = native.mhd_read(str(tmp_path / "m_cpu" / f"{name}.mhd"))
        assert np.array_equal(a.astype(np.float64), b.astype(np.float64)), name


# ---------------------------------------------------------------------------------------------
# 3D torch ops and the z-slab decomposition (volume_slabs.h, parallel/volume_slabs.py) on the GPU
# ---------------------------------------------------------------------------------------------
def test_region_grow3d_and_dilate3d_ops_vs_golden(native):
    from nm03_capstone_project_amd import ops
    rng = np.random.default_rng(11)
    band = (rng.random((20, 70, 130)) < 0.4).astype(np.uint8)
    seeds = [(int(x), int(y), int(z)) for z, y, x in zip(*np.nonzero(band))][:40:8]
    bt = torch.from_numpy(band.astype(bool)).cuda()
    for conn in (6, 26):
        ref = native.golden_region_grow3d(band, seeds, conn)
        reg, sweeps = ops.region_grow3d(bt, seeds, conn)
        assert sweeps >= 2 and np.array_equal(reg.cpu().numpy().astype(np.uint8), ref)
        # continuing from a partial region (seed voxels only) reaches the same fixpoint
        part = np.zeros_like(band)
        for x, y, z in seeds:
            part[z, y, x] = band[z, y, x]
        reg2, _ = ops.region_grow3d(bt, [], conn, region=torch.from_numpy(part.astype(bool)).cuda())
        assert np.array_equal(reg2.cpu().numpy().astype(np.uint8), ref)
        for size in (3, 7):
            dil = ops.dilate3d(reg, size)
            assert np.array_equal(dil.cpu().numpy().astype(np.uint8), native.golden_dilate3d(ref, size))


def test_region_grow3d_and_dilate3d_large_planes(native):
    """1100 × 600 planes: region growing and the in-plane dilation both on global-memory planes."""
    from nm03_capstone_project_amd import ops
    rng = np.random.default_rng(12)
    band = (rng.random((5, 600, 1100)) < 0.45).astype(np.uint8)
    seeds = [(int(x), int(y), int(z)) for z, y, x in zip(*np.nonzero(band))][:400:40]
    ref = native.golden_region_grow3d(band, seeds, 6)
    reg, sweeps = ops.region_grow3d(torch.from_numpy(band.astype(bool)).cuda(), seeds, 6)
    assert sweeps >= 2 and np.array_equal(reg.cpu().numpy().astype(np.uint8), ref)
    dil = ops.dilate3d(reg, 5)
    assert np.array_equal(dil.cpu().numpy().astype(np.uint8), native.golden_dilate3d(ref, 5))


def test_volume_slabs_single_rank_equals_volume_pipeline(native):
    from nm03_capstone_project_amd.parallel.volume_slabs import run_volume_slabs
    d, h, w = 24, 96, 128
    vol = np.stack([native.phantom_slice(h, w, 2, z, d, 5) for z in range(d)])
    vp = nm.VolumePipeline(connectivity=6, dilation=7)
    ref = vp.run(vol)
    r = run_volume_slabs(volume=vol, connectivity=6, dilation=7, backend="gpu")
    assert ref["region"].sum() > 0 and (r["z0"], r["z1"]) == (0, d) and r["rounds"] == 1
    for k in ("band", "region", "dilated"):
        assert np.array_equal(r[k], ref[k]), k


@pytest.mark.parametrize("ranks,conn,thin", [(2, 6, False), (3, 26, False), (4, 6, True)])
def test_volume_slabs_threads_device_exchange_equals_volume(native, ranks, conn, thin):
    """The device-resident z-slab exchange (Comm::sendrecv_device / allreduce_sum_i64_device, the
    slab seed kernel, halos received straight into the extended dilation buffer) with N rank threads
    on one GPU over loopback comms: region and dilation identical to the single-volume run, with a
    region that crosses every slab boundary (several rounds). `thin`: slabs thinner than the
    dilation halo take the generic all-gather path."""
    d = 8 if thin else 40
    h, w = 96, 128
    vol = np.stack([native.phantom_slice(h, w, 2, z % 7, d, 5) for z in range(d)])
    vol[:, 40:56, :] = 1500  # an in-band slab through every plane: the region spans all slabs
    ref = native.VolumeRunner(0).run(vol, native.PipelineParams(), conn, 7, [])
    r = native.run_volume_slabs_threads(vol, ranks, native.PipelineParams(), conn, 7, 0, 2)
    assert ref["region"].sum() > 0 and len(r["walls_s"]) == 2
    assert max(r["rounds"]) >= 2 or thin
    assert np.array_equal(r["region"], ref["region"])
    assert np.array_equal(r["dilated"], ref["dilated"])


@pytest.mark.parametrize("ranks", [2, 3])
def test_volume_cli_split_volume_identical(native, cohort_root, tmp_path, ranks):
    """img_processing_parallel --mode 3d --split-volume: every volume cut into z-slabs over N ranks
    (host comm, all on GPU 0), boundary planes and dilation halos exchanged natively — the output
    tree is byte-identical to the single-GPU 3D run."""
    import json
    ref, out = tmp_path / "ref", tmp_path / "split"
    r = run_bin("img_processing_parallel", "--mode", "3d", "--data-root", cohort_root, "--out", str(ref), "--quiet")
    assert r.returncode == 0, r.stderr
    r = run_bin("img_processing_parallel", "--mode", "3d", "--split-volume", "--gpus", str(ranks), "--data-root",
                cohort_root, "--out", str(out), "--quiet", "--json", str(tmp_path / "s.json"),
                env={"NM03_DEVICE_OVERRIDE": "0", "NM03_COMM_TIMEOUT_S": "60"})
    assert r.returncode == 0, r.stderr
    assert f"Split over {ranks} ranks" in r.stdout
    t = _tree(str(ref))
    assert len(t) > 0 and _tree(str(out)) == t
    j = json.load(open(tmp_path / "s.json"))
    assert j["split_volume"] and j["gpus"] == ranks and all(p["ok"] and p["rounds"] >= 1 for p in j["patients"])


def test_cli_parallel_sizes_buffers_from_headers(native, cohort_root, tmp_path):
    """The parallel CLI sizes its engine from the cohort's slice headers (cold start): a larger
    slice added to one series still goes through, with the same bytes as the golden model."""
    import shutil
    root = tmp_path / "data"
    shutil.copytree(cohort_root, root)
    base = native.cohort_dir(str(root) + "/")
    pid = native.find_patient_dirs(base)[0]
    series, files = native.list_patient_series(base, pid)
    big = native.phantom_slice(320, 320, 1, 3, 9, 11)
    open(os.path.join(series, "1-99.dcm"), "wb").write(native.dicom_bytes(big))
    out = tmp_path / "o"
    r = run_bin("img_processing_parallel", "--data-root", str(root), "--out", str(out), "--quiet",
                env={"NM03_LOG": "info"})
    assert r.returncode == 0, r.stderr
    assert "max_dim 320" in r.stdout
    assert f"Patient {pid} completed. Successfully processed {len(files) + 1}/{len(files) + 1} images." in r.stdout
    g = native.golden_run(big)
    assert (out / pid / "1-99_processed.jpg").read_bytes() == g["jpeg_processed"]
    assert (out / pid / "1-99_original.jpg").read_bytes() == g["jpeg_original"]


def test_cli_sequential_error_messages(native, cohort_root, tmp_path):
    """img_processing_sequential reports failures with the reference's message pairs: an export
    error prints `Error in export stage: E` then `Error processing file F:` / `Detailed error: E`
    (main_sequential.cpp:74-76, 267-269); a device (non-pipeline) error prints
    `Failed to process image i for patient P. Moving to next image.` (:291-293)."""
    r = run_bin("img_processing_sequential", "--data-root", cohort_root, "--out", str(tmp_path / "o"),
                env={"NM03_FAULT": "fail_write:1,fail_batch:2"})
    assert r.returncode == 0, r.stderr
    err = r.stderr
    assert "Error in export stage: injected fault: export failure" in err
    i = err.index("Error in export stage: injected fault: export failure")
    assert "Detailed error: injected fault: export failure" in err[i:]
    assert "Error processing file " in err[i:]
    assert "Failed to process image 3 for patient PGBM-001. Moving to next image." in err


def test_cli_parallel_patient_level_failures(native, cohort_root, tmp_path):
    """SURVEY §4.2 T5 on the parallel CLI: a patient without a series directory, a patient whose
    series holds no .dcm, and a slice in an unsupported (compressed) transfer syntax are reported
    with the reference's messages (main_parallel.cpp:304, 353, 165-166) and isolated: every other
    slice is exported and every patient is counted, as the reference's catch blocks do."""
    import re
    import shutil
    root = tmp_path / "data"
    shutil.copytree(cohort_root, root)
    base = native.cohort_dir(str(root) + "/")
    pids = native.find_patient_dirs(base)
    # PGBM-9xx: no series directory at all; PGBM-8xx: an empty series directory
    os.makedirs(os.path.join(base, "PGBM-901"))
    os.makedirs(os.path.join(base, "PGBM-801", "1.000000-empty-1"))
    series, files = native.list_patient_series(base, pids[0])
    b = bytearray(native.dicom_bytes(native.phantom_slice(128, 128, 1, 1, 5, 2), syntax="explicit"))
    ts = b"1.2.840.10008.1.2.1\x00"
    i = b.find(ts)
    assert i > 0
    b[i:i + len(ts)] = b"1.2.840.10008.1.2.4.50"[:len(ts)]  # JPEG baseline: not supported
    open(os.path.join(series, "1-77.dcm"), "wb").write(bytes(b))
    out = tmp_path / "o"
    r = run_bin("img_processing_parallel", "--data-root", str(root), "--out", str(out))
    assert r.returncode == 0, r.stderr
    assert "Error loading DICOM files for patient PGBM-901: No series directories found for patient: PGBM-901" in r.stderr
    assert "Error processing patient PGBM-901:" in r.stderr
    assert "Found 0 DICOM files for patient PGBM-801" in r.stdout
    assert "Patient PGBM-801 completed. Successfully processed 0/0 images." in r.stdout
    assert re.search(r"Error processing file .*1-77\.dcm:\nDetailed error: .*transfer syntax", r.stderr)
    n0 = len(files)
    assert f"Patient {pids[0]} completed. Successfully processed {n0}/{n0 + 1} images." in r.stdout
    assert f"Successfully processed {len(pids) + 2}/{len(pids) + 2} patients." in r.stdout
    assert not (out / pids[0] / "1-77_original.jpg").exists()


# ---------------------------------------------------------------------------------------------
# Round 5: --se-shape disc (K2 / K5), the new DICOM import forms through the GPU engine, and the
# render kernel's first launch from slot threads in a fresh CLI process (complete preload)
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("conn", [4, 8])
@pytest.mark.parametrize("shape,sizes", [((256, 256), (3, 3)), ((131, 77), (5, 7)), ((600, 520), (3, 5))])
def test_region_grow_disc_se_vs_golden_and_torch(native, conn, shape, sizes):
    h, w = shape
    rng = np.random.default_rng(h + w + conn)
    band = rng.random(shape) < 0.6
    seeds = [(x, y, 0) for (x, y) in native.reference_seeds(w, h)]
    dsz, esz = sizes
    cfg = nm.PipelineConfig(srg_connectivity=conn, se_shape=1, dilation_size=dsz, erosion_size=esz)
    out = ops.region_grow(torch.from_numpy(band).cuda(), seeds, cfg)
    g = native.golden_region_grow(band.astype(np.uint8), seeds, conn)
    assert np.array_equal(out["region"].cpu().numpy(), g.astype(bool))
    dil, ero = out["dilated"].cpu().numpy(), out["eroded"].cpu().numpy()
    assert np.array_equal(dil, native.golden_morph(g, dsz, True, True).astype(bool))
    assert np.array_equal(ero, native.golden_morph(g, esz, False, True).astype(bool))
    rt = torch.from_numpy(g.astype(bool))
    assert np.array_equal(dil, R.dilate_disc(rt, dsz).numpy())
    assert np.array_equal(ero, R.erode_disc(rt, esz).numpy())
    # the renderer border keeps its square erosion (it is not the Dilation/Erosion SE)
    assert np.array_equal(out["border_region"].cpu().numpy(), native.golden_border(g, 2).astype(bool))


def test_engine_disc_se_bit_exact(native):
    raw = _phantom(native)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": 1.0, "spacing_y": 1.0}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2, se_shape=1))
    gpu, ref = pipe.run_array(raw, meta), pipe.golden(raw, meta)
    for k in ("band", "region", "dilated", "eroded"):
        assert np.array_equal(gpu[k], ref[k].astype(bool)), k
    assert gpu["jpegs"][0] == ref["jpeg_original"] and gpu["jpegs"][4] == ref["jpeg_processed"]


@pytest.mark.parametrize("size", [3, 5, 7])
def test_dilate3d_ball_vs_golden_and_torch(native, size):
    rng = np.random.default_rng(size)
    m = rng.random((12, 70, 130)) < 0.03
    dil = ops.dilate3d(torch.from_numpy(m).cuda(), size, ball=True).cpu().numpy()
    assert np.array_equal(dil.astype(np.uint8), native.golden_dilate3d(m.astype(np.uint8), size, True))
    assert np.array_equal(dil, R.dilate_ball(torch.from_numpy(m), size).numpy())


def test_volume_ball_se_vs_golden(native):
    d, h, w = 16, 96, 128
    vol = np.stack([native.phantom_slice(h, w, 2, z, d, 5) for z in range(d)])
    vp = nm.VolumePipeline(nm.PipelineConfig(se_shape=1), connectivity=6, dilation=7)
    seeds = vp.default_seeds(vol)
    res = vp.run(vol, seeds)
    region, dil = vp.golden(res["band"], seeds)
    assert np.array_equal(res["region"], region)
    assert np.array_equal(res["dilated"], dil)
    cube = nm.VolumePipeline(connectivity=6, dilation=7).run(vol, seeds)["dilated"]
    assert (cube >= res["dilated"]).all() and not np.array_equal(cube, res["dilated"])


def test_engine_new_dicom_forms_bit_exact(native, tmp_path):
    """Deflated, RLE, lossless JPEG, MONOCHROME1 and a selected frame of a multi-frame file through the
    GPU engine: both JPEGs equal the golden export of the same samples as the plain reader imports them
    (lossless JPEG: the decoded samples equal the plain encoding's; parity with DCMTK unpinned)."""
    d = tmp_path / "in"
    d.mkdir()
    a, b, c = (native.phantom_slice(256, 256, 2, k, 9, 3) for k in (2, 4, 6))
    files = {
        "1-1.dcm": native.dicom_bytes(a, bits_stored=12, syntax="deflated"),
        "1-2.dcm": native.dicom_bytes(b, bits_stored=12, syntax="rle"),
        "1-3.dcm": native.dicom_bytes(c, bits_stored=12, photometric="MONOCHROME1"),
        "1-4.dcm": native.dicom_bytes(np.stack([a, b, c]), bits_stored=12, syntax="rle"),
        # round 6: lossless JPEG (SV1 = .4.70; SV5 with restart markers and split fragments = .4.57)
        "1-5.dcm": native.dicom_bytes(a, bits_stored=12, syntax="jpeg-lossless"),
        "1-6.dcm": native.dicom_bytes(c, bits_stored=12, syntax="jpeg-lossless", jpeg_predictor=5,
                                      jpeg_restart_rows=32, jpeg_fragments=3),
        # lossy JPEG Extended (12-bit DCT, .4.51): golden input = the same decoded samples
        "1-7.dcm": native.dicom_bytes(b, bits_stored=12, syntax="jpeg-extended", jpeg_quality=90),
    }
    for name, data in files.items():
        (d / name).write_bytes(data)
    out = tmp_path / "out"
    out.mkdir()
    items = [(str(d / n), str(out)) for n in files]
    st, _ = native.Engine(nm.PipelineConfig(batch_size=4, streams=2, threads=4, frame=1).engine_config()).run(items)
    assert [c for c, _ in st] == [0] * len(files), st
    for name in files:
        raw, meta = native.read_slice(str(d / name), 0, 1)
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = name[:-4]
        assert open(out / f"{stem}_original.jpg", "rb").read() == g["jpeg_original"], name
        assert open(out / f"{stem}_processed.jpg", "rb").read() == g["jpeg_processed"], name
    for name, src in (("1-5.dcm", a), ("1-6.dcm", c)):
        assert np.array_equal(native.read_slice(str(d / name))[0], src)
    # MONOCHROME1 is imported inverted: its golden input is the complement of the stored samples
    raw3, _ = native.read_slice(str(d / "1-3.dcm"))
    assert np.array_equal(raw3, (~c) & np.uint16(0x0FFF))


def test_cli_fresh_process_512_cohort_render_from_slot_threads(native, tmp_path):
    """A fresh img_processing_parallel on a 512² cohort with 4 streams: every slice takes the generic
    render kernel (not the fused exact-2× path), whose first launches come from slot threads — the
    code object must already be loaded (kernels.h preload_kernels). Outputs equal the golden model."""
    root = tmp_path / "data"
    base = root / "Brain-Tumor-Progression" / "T1-Post-Combined-P001-P020"
    files = []
    for p in range(2):
        sd = base / f"PGBM-{p + 1:03d}" / "10.000000-T1post-1"
        sd.mkdir(parents=True)
        for z in range(6):
            raw = native.phantom_slice(512, 512, 2, z, 6, 10 + p)
            f = sd / f"1-{z + 1}.dcm"
            f.write_bytes(native.dicom_bytes(raw, bits_stored=12, instance=z + 1, spacing_x=0.7, spacing_y=0.7))
            files.append((p, f))
    out = tmp_path / "out"
    r = run_bin("img_processing_parallel", "--data-root", str(root), "--out", str(out), "--streams", "4",
                "--batch-size", "2", "--quiet")
    assert r.returncode == 0, r.stderr
    for p, f in files[::5]:
        raw, meta = native.read_slice(str(f))
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = f.name[:-4]
        assert open(out / f"PGBM-{p + 1:03d}" / f"{stem}_original.jpg", "rb").read() == g["jpeg_original"]
        assert open(out / f"PGBM-{p + 1:03d}" / f"{stem}_processed.jpg", "rb").read() == g["jpeg_processed"]


@pytest.mark.parametrize("sampling", [0, 2])
def test_engine_render_nearest_bit_exact(native, cohort_root, tmp_path, sampling):
    """--render-filter nearest through the GPU: every stage image of one slice (K3 canvases) and a
    cohort run's export pairs equal the golden model — 4:2:0 renders nearest gray images inside the
    fused encoder (its own instance), the other layouts through K3 canvases."""
    raw = _phantom(native)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": 1.0, "spacing_y": 1.0}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2, render_filter=1,
                                              jpeg_sampling=sampling))
    gpu, ref = pipe.run_array(raw, meta), pipe.golden(raw, meta)
    assert gpu["jpegs"][0] == ref["jpeg_original"] and gpu["jpegs"][4] == ref["jpeg_processed"]
    out = str(tmp_path / "o")
    items = _items(native, cohort_root, out)[:30]
    cfg = nm.PipelineConfig(batch_size=8, streams=2, threads=4, render_filter=1, jpeg_sampling=sampling)
    st, _ = native.Engine(cfg.engine_config()).run(items)
    assert all(c == 0 for c, _ in st)
    for f, od in items[::7]:
        r, m = native.read_slice(f)
        g = native.golden_run(r, m["type"], m["stored_bits"], m["slope"], m["intercept"], native.PipelineParams(),
                              cfg.render_params(), m["spacing_x"], m["spacing_y"])
        stem = os.path.splitext(os.path.basename(f))[0]
        assert open(os.path.join(od, stem + "_original.jpg"), "rb").read() == g["jpeg_original"]
        assert open(os.path.join(od, stem + "_processed.jpg"), "rb").read() == g["jpeg_processed"]


@pytest.mark.parametrize("sampling", [1, 2])
def test_engine_jpeg_sampling_bit_exact(native, cohort_root, tmp_path, sampling):
    """--jpeg-sampling 444 / gray through the engine: the fused render + encode of a cohort run
    (staged gray and label rows, flat label waves) and one slice's five stage JPEGs equal the golden
    model, whose encoder is byte-identical to libjpeg (tests/test_jpeg.py)."""
    raw = _phantom(native)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": 1.0, "spacing_y": 1.0}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2, jpeg_sampling=sampling))
    gpu, ref = pipe.run_array(raw, meta), pipe.golden(raw, meta)
    assert gpu["jpegs"][0] == ref["jpeg_original"] and gpu["jpegs"][4] == ref["jpeg_processed"]
    out = str(tmp_path / "o")
    items = _items(native, cohort_root, out)[:40]
    cfg = nm.PipelineConfig(batch_size=8, streams=2, threads=4, jpeg_sampling=sampling)
    st, _ = native.Engine(cfg.engine_config()).run(items)
    assert all(c == 0 for c, _ in st)
    for f, od in items[::5]:
        r, m = native.read_slice(f)
        g = native.golden_run(r, m["type"], m["stored_bits"], m["slope"], m["intercept"], native.PipelineParams(),
                              cfg.render_params(), m["spacing_x"], m["spacing_y"])
        stem = os.path.splitext(os.path.basename(f))[0]
        orig = open(os.path.join(od, stem + "_original.jpg"), "rb").read()
        assert orig == g["jpeg_original"]
        assert open(os.path.join(od, stem + "_processed.jpg"), "rb").read() == g["jpeg_processed"]
    PIL = pytest.importorskip("PIL.Image")
    assert PIL.open(io.BytesIO(orig)).mode == ("L" if sampling == 2 else "RGB")


def test_deferred_rccl_comm_single_rank(native):
    """The communicator launch_ranks gives RCCL ranks: shared-memory control plane until promote(),
    RCCL started by start_data_plane() and carrying every collective afterwards (one rank: a second
    needs a second GPU)."""
    seg, name = native.shm_create(1)
    c = native.deferred_rccl_comm(0, 1, 0, seg, 30.0)
    assert c.backend == "rccl" and c.transport_size == -1  # RCCL not up yet
    c.barrier()
    assert c.broadcast_bytes(b"plan" * 100, 0) == b"plan" * 100
    c.start_data_plane()
    c.promote()
    assert c.transport_size == 1 and c.transport_device == 0
    assert c.allreduce_sum([3, 4]) == [3, 4] and c.allgather_bytes(b"xy") == [b"xy"]
    t = c.data_plane_times
    assert t["start_s"] >= 0 and t["init_upper_s"] >= t["wait_s"] >= 0
    seg.wait_attached_and_unlink(5.0)


def test_cli_parallel_rccl_data_plane_one_rank(native, cohort_root, tmp_path):
    """the CLI's RCCL path on hardware. NM03_COMM=rccl at one rank takes launch_ranks'
    deferred communicator: the start-up thread brings HIP up, starts AND settles RCCL, then builds the
    engine (RCCL is never initialising while the engine is constructed or launches); after the run the
    collectives are promoted onto RCCL. Outputs equal the default run and the golden model."""
    import json
    ref, out = tmp_path / "ref", tmp_path / "rccl"
    r0 = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(ref), "--gpus", "1", "--quiet")
    assert r0.returncode == 0, r0.stderr
    js = tmp_path / "rccl.json"
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(out), "--gpus", "1", "--quiet",
                "--repeat", "2", "--json", str(js), env={"NM03_COMM": "rccl", "NM03_COMM_TIMEOUT_S": "60"}, timeout=240)
    assert r.returncode == 0, r.stderr
    j = json.load(open(js))
    assert j["data_plane"] is True and j["backend"] == "rccl", j
    assert j["comm"]["backend"] == "rccl" and j["comm"]["nranks"] == 1 and "rccl_error" not in j["comm"], j["comm"]
    assert j["devices"]["transport_size"] == [1] and j["devices"]["transport_device"] == [0]
    assert j["comm_settle_s"] > 0 and j["data_plane_s"] >= j["comm_settle_s"]
    assert j["slices_ok"] == j["slices"] and j["slices"] > 0
    t_ref, t_out = _tree(str(ref)), _tree(str(out))
    assert t_ref == t_out and len(t_out) == j["slices"]  # two JPEGs per slice; --repeat 2 counts each twice
    for pid in ("PGBM-001", "PGBM-003"):
        _, files = native.list_patient_series(native.cohort_dir(cohort_root), pid)
        f = files[len(files) // 2]
        raw, meta = native.read_slice(f)
        g = native.golden_run(raw, meta["type"], meta["stored_bits"], meta["slope"], meta["intercept"],
                              native.PipelineParams(), native.RenderParams(), meta["spacing_x"], meta["spacing_y"])
        stem = os.path.splitext(os.path.basename(f))[0]
        assert open(out / pid / f"{stem}_original.jpg", "rb").read() == g["jpeg_original"]
        assert open(out / pid / f"{stem}_processed.jpg", "rb").read() == g["jpeg_processed"]


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL refuses two ranks on one device)")
def test_cli_parallel_rccl_two_devices(native, cohort_root, tmp_path):
    """two ranks on distinct devices with NM03_COMM=rccl promote onto RCCL; rank 1's
    collectives run on its main thread, which never selected device 1 itself (RcclComm binds it)."""
    import json
    js = tmp_path / "m.json"
    r = run_bin("img_processing_parallel", "--data-root", cohort_root, "--out", str(tmp_path / "o"), "--gpus", "2",
                "--quiet", "--json", str(js), env={"NM03_COMM": "rccl", "NM03_COMM_TIMEOUT_S": "60"}, timeout=240)
    assert r.returncode == 0, r.stderr
    j = json.load(open(js))
    assert j["backend"] == "rccl" and j["comm"]["nranks"] == 2 and j["devices"]["transport_device"] == [0, 1]
    assert sum(j["per_rank"]["slices_ok"]) == j["slices"]


@pytest.mark.parametrize("shape,spacing", [((256, 256), (1.0, 1.0)), ((200, 160), (1.0, 1.0))])
def test_gpu_canvases_vs_torch_reference(native, cohort_root, tmp_path, shape, spacing):
    """the GPU renders held directly against the plain-PyTorch references
    (ops.reference.render_gray / render_labels), not only transitively through the golden model.
    (1) K3 `render_kernel` canvases of run_single (original, sharpened, region / eroded / dilated
    labels): gray within 1 level (f32 evaluation order), labels exact. (2) The fused K4 render of an
    exact-2× export, which never materialises a canvas: its label JPEG equals the CPU encoding
    (byte-identical to libjpeg) of the torch label canvas, and its gray JPEG decodes to the decoded
    CPU encoding of the torch gray canvas within JPEG rounding."""
    h, w = shape
    raw = native.phantom_slice(h, w, 3, 12, 25, 7)
    meta = {"type": "u16", "stored_bits": 16, "slope": 1.0, "intercept": 0.0, "spacing_x": spacing[0],
            "spacing_y": spacing[1]}
    pipe = nm.SlicePipeline(nm.PipelineConfig(batch_size=1, streams=1, threads=2))
    gpu = pipe.run_array(raw, meta)
    dev = torch.device("cuda")
    v = torch.from_numpy(raw.astype(np.float32)).to(dev)
    ref = R.render_gray(v, float(raw.min()), float(raw.max())).cpu().numpy()
    c0 = np.asarray(gpu["canvases"][0])
    assert c0.shape == (512, 512) and np.abs(c0.astype(int) - ref.astype(int)).max() <= 1
    assert (c0 != ref).mean() < 0.01
    sh = torch.from_numpy(np.asarray(gpu["sharpened"], np.float32).reshape(h, w)).to(dev)
    ref_s = R.render_gray(sh, float(sh.min()), float(sh.max())).cpu().numpy()
    assert np.abs(np.asarray(gpu["canvases"][1]).astype(int) - ref_s.astype(int)).max() <= 1
    for k, plane in ((2, "region"), (3, "eroded"), (4, "dilated")):
        lab = torch.from_numpy(np.asarray(gpu[plane]).reshape(h, w).astype(bool)).to(dev)
        ref_l = R.render_labels(lab, R.border(lab, 2)).cpu().numpy()
        assert np.array_equal(np.asarray(gpu["canvases"][k]), ref_l), plane
    if shape != (256, 256):
        return
    # (2) fused exact-2× export path through the engine
    d = tmp_path / "in"
    d.mkdir()
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(raw))
    out = tmp_path / "out"
    out.mkdir()
    st, times = native.Engine(nm.PipelineConfig(batch_size=4, streams=1, threads=2).engine_config()).run(
        [(str(d / "1-1.dcm"), str(out))])
    assert st[0][0] == 0
    lab = torch.from_numpy(np.asarray(gpu["dilated"]).reshape(h, w).astype(bool)).to(dev)
    ref_l = R.render_labels(lab, R.border(lab, 2)).cpu().numpy()
    assert open(out / "1-1_processed.jpg", "rb").read() == native.jpeg_encode_gray420(ref_l, 75)
    PIL = pytest.importorskip("PIL.Image")
    got = np.asarray(PIL.open(out / "1-1_original.jpg").convert("L"), dtype=np.int32)
    want = np.asarray(PIL.open(io.BytesIO(native.jpeg_encode_gray420(ref, 75))).convert("L"), dtype=np.int32)
    assert R.psnr(torch.from_numpy(got), torch.from_numpy(want)) > 45.0
