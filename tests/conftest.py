import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BIN = os.path.join(ROOT, "build", "bin")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native():
    import nm03_capstone_project_amd as m
    return m.native()


@pytest.fixture(scope="session")
def cohort_root(tmp_path_factory, native):
    """Small synthetic cohort: 4 patients × 3–5 slices (+ the fixed test_pipeline slice)."""
    root = str(tmp_path_factory.mktemp("data")) + "/"
    native.synth_cohort(root, patients=4, min_slices=3, max_slices=5, threads=4)
    return root


def run_bin(name, *args, cwd=None, env=None, timeout=600):
    exe = os.path.join(BIN, name)
    e = dict(os.environ)
    if env:
        e.update(env)
    e = {k: v for k, v in e.items() if v is not None}  # env={"X": None} removes X
    return subprocess.run([exe, *args], cwd=cwd, env=e, capture_output=True, text=True, timeout=timeout)
