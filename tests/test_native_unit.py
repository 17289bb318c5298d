"""Runs the native host unit tests (tests/native/unit_tests.cpp, also registered with CTest):
cohort naming, DICOM loader paths, streaming copies, JPEG container, golden operators vs brute
force, thread pool, loopback collectives, wire format, CLI defaults. CPU only."""
import os
import subprocess

import pytest

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "bin", "nm03_unit_tests")


def test_native_unit_tests():
    if not os.path.exists(BIN):
        pytest.fail(f"{BIN} missing: run `python build.py` first")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
