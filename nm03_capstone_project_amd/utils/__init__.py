"""DICOM / JPEG / cohort helpers and the synthetic T1+C cohort."""
from .cohort import (Cohort, Patient, cohort_dir, extract_file_number, find_patient_dirs,  # noqa: F401
                     list_patient_series, synth_cohort, test_slice_path)
from .dicom import Slice, dicom_bytes, load_slice, parse_dicom, read_series, read_slice, series_files  # noqa: F401
