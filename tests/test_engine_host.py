"""The engine's host path on the CPU (EngineConfig.host_only: every DICOM load, 12-bit pack and JPEG
file write of a real run, the GPU stages replaced by fixed pre-encoded segments; no HIP call).
Covers the scheduler, directory-fd handling, resume, batch caps and failure isolation without a GPU
(the byte-level JPEG contract is tested against the golden model in test_gpu.py)."""
import io
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(native, **kw):
    import nm03_capstone_project_amd as nm
    cfg = nm.PipelineConfig(**{"batch_size": 4, "streams": 2, "threads": 3, **kw}).engine_config()
    cfg.host_only = True
    return native.Engine(cfg)


def _items(native, root, out):
    base = native.cohort_dir(root)
    items = []
    for pid in native.find_patient_dirs(base):
        _, files = native.list_patient_series(base, pid)
        d = os.path.join(out, pid)
        os.makedirs(d, exist_ok=True)
        items += [(f, d) for f in files]
    return items


def test_host_only_run_writes_every_file(native, cohort_root, tmp_path):
    items = _items(native, cohort_root, str(tmp_path / "out"))
    st, times = _engine(native).run(items)
    assert [c for c, _ in st] == [0] * len(items)
    assert times["kernels_s"] == 0.0 and times["batches"] == (len(items) + 3) // 4
    from PIL import Image
    for f, d in items:
        stem = os.path.basename(f)[:-4]
        for kind in ("original", "processed"):
            b = open(os.path.join(d, f"{stem}_{kind}.jpg"), "rb").read()
            assert b[:2] == b"\xff\xd8" and b[-2:] == b"\xff\xd9"
            im = Image.open(io.BytesIO(b))
            im.load()
            assert im.size == (512, 512)


def test_host_only_batch_cap(native, cohort_root, tmp_path):
    items = _items(native, cohort_root, str(tmp_path / "out"))
    wl = native.WorkList(items)
    eng = _engine(native, batch_size=8)
    codes, msgs, t = eng.run_list(wl, 3)
    assert not msgs and t["batches"] == -(-len(items) // 3)
    codes, msgs, t = eng.run_list(wl)
    assert not msgs and t["batches"] == -(-len(items) // 8)


def test_host_only_resume_skips_existing(native, cohort_root, tmp_path):
    items = _items(native, cohort_root, str(tmp_path / "out"))
    _engine(native).run(items)
    st, _ = _engine(native, resume=True).run(items)
    assert all(c == 0 and "resumed" in m for c, m in st)


def test_host_only_too_small_and_corrupt(native, tmp_path):
    """<100 guard (main_sequential.cpp:189-192) and an unreadable file: per-slice statuses."""
    import numpy as np
    d = tmp_path / "in"
    d.mkdir()
    good = native.phantom_slice(256, 256, 1, 3, 10, 7)
    (d / "1-1.dcm").write_bytes(native.dicom_bytes(good, bits_stored=12))
    (d / "1-2.dcm").write_bytes(native.dicom_bytes(np.zeros((64, 64), np.uint16)))
    (d / "1-3.dcm").write_bytes(b"not a dicom file")
    out = tmp_path / "out"
    out.mkdir()
    st, _ = _engine(native).run([(str(d / f"1-{k}.dcm"), str(out)) for k in (1, 2, 3)])
    assert [c for c, _ in st] == [0, 2, 1]
    assert "too small" in st[1][1]


_FD_SCRIPT = r"""
import os, resource, sys
sys.path.insert(0, {root!r})
resource.setrlimit(resource.RLIMIT_NOFILE, (64, resource.getrlimit(resource.RLIMIT_NOFILE)[1]))
import nm03_capstone_project_amd as nm
n = nm.native()
src = {src!r}
items = []
for k in range(150):  # 150 distinct output directories, far more than 64 descriptors
    d = os.path.join({out!r}, "d%03d" % k)
    os.makedirs(d, exist_ok=True)
    items.append((src[k % len(src)], d))
cfg = nm.PipelineConfig(batch_size=16, streams=3, threads=4).engine_config()
cfg.host_only = True
eng = n.Engine(cfg)
codes, msgs, t = eng.run_list(n.WorkList(items))
ok = sum(1 for k in range(150) if os.path.exists(os.path.join({out!r}, "d%03d" % k)))
print(len(msgs), ok)
"""


def test_host_only_many_directories_low_fd_limit(native, cohort_root, tmp_path):
    """a run touching more directories than RLIMIT_NOFILE allows must not fail with
    EMFILE — directory fds are capped per run, the rest use full paths."""
    src = [f for f, _ in _items(native, cohort_root, str(tmp_path / "o0"))]
    code = _FD_SCRIPT.format(root=ROOT, src=src, out=str(tmp_path / "many"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split() == ["0", "150"], r.stdout
    for k in range(150):
        d = tmp_path / "many" / f"d{k:03d}"
        assert len(os.listdir(d)) == 2


@pytest.mark.parametrize("fault,code", [("corrupt_dicom:2", 1), ("fail_write:1", 4)])
def test_host_only_fault_injection(native, cohort_root, tmp_path, fault, code):
    """NM03_FAULT: the injected slice fails with its code, every other slice succeeds."""
    items = _items(native, cohort_root, str(tmp_path / "out"))
    script = (f"import sys, json; sys.path.insert(0, {ROOT!r}); import nm03_capstone_project_amd as nm; "
              f"n = nm.native(); cfg = nm.PipelineConfig(batch_size=4, streams=2, threads=2).engine_config(); "
              f"cfg.host_only = True; st, _ = n.Engine(cfg).run({items!r}); print(json.dumps([c for c, _ in st]))")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, NM03_FAULT=fault))
    assert r.returncode == 0, r.stderr[-2000:]
    codes = json.loads(r.stdout.strip().splitlines()[-1])
    bad = int(fault.split(":")[1])
    assert codes[bad] == code and all(c == 0 for i, c in enumerate(codes) if i != bad)


def _tree_bytes(items):
    out = {}
    for f, d in items:
        stem = os.path.basename(f)[:-4]
        for kind in ("original", "processed"):
            p = os.path.join(d, f"{stem}_{kind}.jpg")
            out[p] = open(p, "rb").read()
    return out


def test_host_only_queued_runs_fresh_and_existing_trees(native, cohort_root, tmp_path):
    """Pool workers (private fd tables and creds) write the same files across two queued runs into
    two trees, fresh (files created) then existing (rewritten in place)."""
    items = _items(native, cohort_root, str(tmp_path / "a"))
    items_b = _items(native, cohort_root, str(tmp_path / "b"))
    eng = _engine(native, threads=4, batch_size=4, streams=2)
    wa, wb = native.WorkList(items), native.WorkList(items_b)
    for _ in range(2):
        ta, tb = eng.submit(wa), eng.submit(wb)
        assert sum(len(eng.wait(t)[1]) for t in (ta, tb)) == 0
    del eng
    a, b = _tree_bytes(items), _tree_bytes(items_b)
    assert len(a) == 2 * len(items) and sorted(a.values()) == sorted(b.values())


def test_private_fd_tables_do_not_hold_process_fds(native, cohort_root, tmp_path):
    """A worker's private table starts with stdin/out/err only: a pipe the process creates before
    the engine and closes afterwards must reach EOF while the engine (and its pool) is alive."""
    r, w = os.pipe()
    eng = _engine(native, threads=4)
    items = _items(native, cohort_root, str(tmp_path / "o"))
    codes, msgs, _ = eng.run_list(native.WorkList(items))
    assert not msgs
    os.close(w)
    import select
    ready, _, _ = select.select([r], [], [], 5.0)
    assert ready and os.read(r, 1) == b""  # EOF: no worker kept a duplicate of the write end
    os.close(r)
    del eng


def test_host_only_many_queued_runs(native, cohort_root, tmp_path):
    """Eleven runs in flight at once: every run still writes every file."""
    eng = _engine(native, threads=4, batch_size=8, streams=3)
    trees = [_items(native, cohort_root, str(tmp_path / f"t{k}"))[:24] for k in range(11)]
    tickets = [eng.submit(native.WorkList(t)) for t in trees]
    for t in tickets:
        codes, msgs, _ = eng.wait(t)
        assert not msgs
    for t in trees:
        assert len(_tree_bytes(t)) == 2 * len(t)


def test_host_only_compressed_and_photometric_forms(native, tmp_path):
    """Round 5/6 import forms through the engine's loader (host path): Deflated Explicit VR LE, RLE
    Lossless, lossless JPEG (.4.70 / .4.57, split fragments) and MONOCHROME1 load like plain files; a multi-frame file is a per-slice load error by
    default and loads when a frame is selected; a JPEG-family file is skipped and counted."""
    import numpy as np
    d = tmp_path / "in"
    d.mkdir()
    good = native.phantom_slice(256, 256, 1, 3, 10, 7)
    forms = [dict(syntax="deflated"), dict(syntax="rle"), dict(photometric="MONOCHROME1"), dict(syntax="rle", photometric="MONOCHROME1"),
             dict(syntax="jpeg-lossless"), dict(syntax="jpeg-lossless", jpeg_predictor=6, jpeg_fragments=2),
             dict(syntax="jpeg-extended")]
    paths = []
    for k, kw in enumerate(forms, 1):
        p = d / f"1-{k}.dcm"
        p.write_bytes(native.dicom_bytes(good, bits_stored=12, **kw))
        paths.append(p)
    mf = d / "1-9.dcm"
    mf.write_bytes(native.dicom_bytes(np.stack([good, good, good]), bits_stored=12, syntax="rle"))
    paths.append(mf)
    out = tmp_path / "out"
    out.mkdir()
    items = [(str(p), str(out)) for p in paths]
    nf = len(forms)
    st, _ = _engine(native).run(items)
    assert [c for c, _ in st] == [0] * nf + [1]
    assert "Multi-frame DICOM (3 frames)" in st[nf][1]
    st, _ = _engine(native, frame=1).run(items)
    assert [c for c, _ in st] == [0] * (nf + 1)
    st, _ = _engine(native, frame=3).run(items)
    assert [c for c, _ in st] == [0] * nf + [1] and "Frame 3 requested" in st[nf][1]
    # lossless JPEG (round 6) loads the same samples as the plain encoding
    for p in paths[4:6]:
        raw, _ = native.read_slice(str(p))
        assert np.array_equal(raw, good)
