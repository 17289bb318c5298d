"""DICOM / JPEG / cohort helpers and the synthetic T1+C cohort."""
from .cohort import (cohort_dir, extract_file_number, find_patient_dirs, list_patient_series,  # noqa: F401
                     synth_cohort, test_slice_path)
from .dicom import dicom_bytes, parse_dicom, read_slice  # noqa: F401
from .timing import Timer  # noqa: F401
