"""Cohort layout helpers (reference main_sequential.cpp:18-30, 93-168) and the synthetic cohort."""
from .._native import native


def extract_file_number(name):
    return native().extract_file_number(name)


def cohort_dir(data_root):
    return native().cohort_dir(data_root)


def test_slice_path(data_root):
    return native().test_slice_path(data_root)


def find_patient_dirs(cohort_root):
    return native().find_patient_dirs(cohort_root)


def list_patient_series(cohort_root, pid):
    return native().list_patient_series(cohort_root, pid)


def synth_cohort(data_root, patients=20, min_slices=21, max_slices=25, rows=256, cols=256, seed=20250404,
                 threads=8, test_slice=True, decoy=False, signed=False):
    """Write the synthetic T1+C cohort (20 patients × 21–25 slices of 256² by default)."""
    return native().synth_cohort(data_root, patients, min_slices, max_slices, rows, cols, seed, threads,
                                 test_slice, decoy, signed)
