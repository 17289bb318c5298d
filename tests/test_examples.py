"""The scripts under examples/ run as documented: the cohort example on the host path here, all three
on the MI355X (GPU results checked against the golden model inside the scripts)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, timeout=300):
    return subprocess.run([sys.executable, os.path.join(ROOT, "examples", script), *args], capture_output=True,
                          text=True, timeout=timeout)


def test_process_cohort_example_host_only(tmp_path):
    r = _run("process_cohort.py", "--data-root", str(tmp_path / "d") + "/", "--out", str(tmp_path / "o"), "--synth",
             "--host-only")
    assert r.returncode == 0, r.stderr
    assert "4 patients" in r.stdout and len(glob.glob(str(tmp_path / "o" / "PGBM-*" / "*_processed.jpg"))) > 0


@pytest.mark.gpu
def test_examples_on_gpu(native, tmp_path):
    d, o = str(tmp_path / "d") + "/", str(tmp_path / "o")
    r = _run("process_cohort.py", "--data-root", d, "--out", o, "--synth", "--se-shape", "disc", "--jpeg-sampling", "gray")
    assert r.returncode == 0, r.stderr
    r = _run("single_slice_stages.py", "--dicom", native.test_slice_path(d), "--out", str(tmp_path / "s"))
    assert r.returncode == 0 and "GPU == golden: True" in r.stdout, r.stdout + r.stderr
    series = os.path.dirname(sorted(glob.glob(os.path.join(d, "**", "PGBM-001", "*", "*.dcm"), recursive=True))[0])
    for extra in ([], ["--ball"]):
        r = _run("volume_3d.py", "--series", series, *extra)
        assert r.returncode == 0 and "GPU == golden: True" in r.stdout, r.stdout + r.stderr
