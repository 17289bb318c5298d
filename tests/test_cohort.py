"""Cohort discovery / ordering / output-dir management (main_sequential.cpp:18-168)."""
import os

import pytest


@pytest.mark.parametrize("name,num", [("1-14.dcm", 14), ("1-01.dcm", 1), ("IMG-0001-0007.dcm", 7),
                                      ("abc.dcm", 1000), ("1-x.dcm", 1000), ("1-3a.dcm", 3), ("noext", 1000)])
def test_extract_file_number(native, name, num):
    assert native.extract_file_number(name) == num


def test_reference_seeds(native):
    s = native.reference_seeds(256, 256)
    assert len(s) == 41
    assert s[:5] == [(128, 128), (160, 128), (96, 128), (128, 160), (128, 96)]
    grid = {x for x, _ in s[5:]}
    assert grid == {64, 89, 114, 139, 164, 189}
    assert len(native.reference_seeds(512, 512)) == 41
    assert len(native.reference_seeds(5, 5)) > 0  # step clamped ≥1 (quirk 4), no infinite loop


def test_discovery_and_ordering(native, tmp_path):
    root = str(tmp_path) + "/"
    native.synth_cohort(root, patients=3, min_slices=12, max_slices=12, threads=2, decoy=True)
    base = native.cohort_dir(root)
    os.makedirs(base + "NOT-A-PATIENT")
    pids = native.find_patient_dirs(base)
    assert pids == ["PGBM-001", "PGBM-002", "PGBM-003"]
    series, files = native.list_patient_series(base, "PGBM-002")
    assert series.endswith("/") and "T1post" in series  # lexicographically first, not the decoy
    nums = [native.extract_file_number(os.path.basename(f)) for f in files]
    assert nums == list(range(1, 13))  # numeric, not lexicographic (1-10 after 1-09)
    assert os.path.exists(native.test_slice_path(root))


def test_setup_output_dir_wipes(native, tmp_path):
    d = tmp_path / "out" / "PGBM-001"
    d.mkdir(parents=True)
    (d / "old.jpg").write_bytes(b"x")
    (d / "sub").mkdir()
    native.setup_output_dir(str(d))
    assert d.exists() and list(d.iterdir()) == []
    native.setup_output_dir(str(tmp_path / "new" / "deep"))
    assert (tmp_path / "new" / "deep").is_dir()


def test_missing_series_raises(native, tmp_path):
    base = tmp_path / "Brain-Tumor-Progression" / "T1-Post-Combined-P001-P020" / "PGBM-009"
    base.mkdir(parents=True)
    with pytest.raises(Exception, match="No series directories"):
        native.list_patient_series(str(base.parent), "PGBM-009")


def test_setup_output_dirs_wipes_files_and_subdirs(native, tmp_path):
    """setup_output_dir(s): the reference's `mkdir -p d && rm -rf d/*` (main_sequential.cpp:32-47):
    every entry goes, files and nested directories alike; the directories themselves stay."""
    dirs = []
    for k in range(5):
        d = tmp_path / f"PGBM-{k:03d}"
        (d / "nested" / "deeper").mkdir(parents=True)
        (d / "nested" / "deeper" / "x.jpg").write_bytes(b"x")
        for i in range(30):
            (d / f"1-{i}_original.jpg").write_bytes(b"y" * 10)
        dirs.append(str(d))
    dirs.append(str(tmp_path / "new" / "PGBM-999"))  # created on the way
    native.setup_output_dirs(dirs, 4)
    for d in dirs:
        assert os.path.isdir(d) and os.listdir(d) == []
    native.setup_output_dir(dirs[0])
    assert os.listdir(dirs[0]) == []


def test_cohort_view_and_work_items(native, tmp_path):
    """utils.Cohort: same patients/series/order as the native discovery, a patient without a
    series is skipped with its reason, work items map to out_root/PGBM-XXX."""
    from nm03_capstone_project_amd.utils import Cohort
    root = str(tmp_path) + "/"
    native.synth_cohort(root, patients=3, min_slices=5, max_slices=7, threads=2)
    base = native.cohort_dir(root)
    os.makedirs(os.path.join(base, "PGBM-009"))  # a patient directory with no T1post series
    c = Cohort.discover(root)
    assert [p.pid for p in c] == ["PGBM-001", "PGBM-002", "PGBM-003"]
    assert [pid for pid, _ in c.skipped] == ["PGBM-009"]
    for p in c:
        assert (p.series_dir, p.files) == tuple(native.list_patient_series(base, p.pid))
    out = str(tmp_path / "out")
    items = c.work_items(out)
    assert len(items) == c.n_slices == sum(len(p) for p in c)
    assert items[0] == (c.patients[0].files[0], os.path.join(out, "PGBM-001"))
    assert all(os.path.isdir(od) for _, od in items)


def test_read_series_stacks_in_file_number_order(native, tmp_path):
    """utils.read_series: file-number order (1-10 after 1-9), one volume copy, rescale and the
    signed view; a mixed-shape series is refused."""
    import numpy as np
    from nm03_capstone_project_amd.utils import load_slice, read_series
    d = tmp_path / "series"
    d.mkdir()
    planes = [np.full((6, 5), 100 + k, np.uint16) for k in range(11)]
    for k, p in enumerate(planes, start=1):
        (d / f"1-{k}.dcm").write_bytes(native.dicom_bytes(p, instance=k))
    vol, slices = read_series(str(d))
    assert vol.shape == (11, 6, 5)
    assert [int(v[0, 0]) for v in vol] == list(range(100, 111))
    assert np.shares_memory(slices[3].raw, vol)
    s = native.dicom_bytes(np.array([[0xFFFF, 2]], np.uint16), type="i16", write_rescale=True, slope=2.0,
                           intercept=-10.0)
    (tmp_path / "s.dcm").write_bytes(s)
    sl = load_slice(tmp_path / "s.dcm")
    assert sl.values.dtype == np.int16 and sl.values.tolist() == [[-1, 2]]
    assert sl.rescaled().tolist() == [[-12.0, -6.0]]
    (d / "1-12.dcm").write_bytes(native.dicom_bytes(np.zeros((7, 5), np.uint16)))
    with pytest.raises(ValueError, match="differs"):
        read_series(str(d))


def test_output_reaper_wipes_off_path(tmp_path):
    """OutputReaper: an existing directory is empty right after wipe() (renamed aside and
    re-created), its old files and subdirectories are deleted by the background threads (drain),
    a missing directory is created, and trash left by a killed run in the parent is swept."""
    from nm03_capstone_project_amd import native
    n = native()
    root = tmp_path / "out"
    a, b = root / "PGBM-001", root / "PGBM-002"
    a.mkdir(parents=True)
    for i in range(50):
        (a / f"{i}_original.jpg").write_bytes(b"x" * 100)
    (a / "sub").mkdir()
    (a / "sub" / "f").write_bytes(b"y")
    import subprocess
    dead = subprocess.Popen(["true"])
    dead.wait()  # a pid whose process is gone: its trash is stale
    stale = root / f".nm03-trash-{dead.pid}-7"
    stale.mkdir()
    (stale / "old.jpg").write_bytes(b"z")
    live = root / f".nm03-trash-{os.getppid()}-3"  # a live run's trash is left to its own reaper
    live.mkdir()
    (live / "busy.jpg").write_bytes(b"z")
    r = n.OutputReaper(2)
    r.wipe([str(a), str(b)])
    assert a.is_dir() and list(a.iterdir()) == [] and b.is_dir()
    (a / "new.jpg").write_bytes(b"n")  # the caller writes right away
    r.drain()
    assert sorted(p.name for p in root.iterdir()) == [live.name, "PGBM-001", "PGBM-002"]
    live.joinpath("busy.jpg").unlink()
    live.rmdir()
    assert [p.name for p in a.iterdir()] == ["new.jpg"]
    assert r.files_reaped == 52
    r.wipe([str(a)])  # second pass over the same parent
    r.drain()
    assert list(a.iterdir()) == [] and sorted(p.name for p in root.iterdir()) == ["PGBM-001", "PGBM-002"]
