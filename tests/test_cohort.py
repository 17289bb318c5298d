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
