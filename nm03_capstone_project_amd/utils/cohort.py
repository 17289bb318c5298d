"""Cohort layout helpers (reference main_sequential.cpp:18-30, 93-168) and the synthetic cohort.

`Cohort` is the Python view of what the CLIs discover natively (src/io/cohort.cpp): the
T1-Post-Combined-P001-P020 directory under the data root, its PGBM-* patients, each patient's
T1post series with slices in file-number order, and the out-*/PGBM-XXX output layout
(`work_items`), which is what `Engine.run` / `SlicePipeline` consume."""
import os
from dataclasses import dataclass, field

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


@dataclass
class Patient:
    pid: str
    series_dir: str
    files: list = field(default_factory=list)

    def __len__(self):
        return len(self.files)


@dataclass
class Cohort:
    """Patients with a T1post series, in the reference's discovery order. Patients without one
    are listed in `skipped` with the reason (the reference prints and continues,
    main_sequential.cpp:111-121)."""
    root: str
    patients: list = field(default_factory=list)
    skipped: list = field(default_factory=list)  # [(pid, reason)]

    @classmethod
    def discover(cls, data_root=None, cohort_root=None):
        """From a data root (…/T1-Post-Combined-P001-P020 below it) or the cohort directory itself."""
        n = native()
        root = cohort_root if cohort_root is not None else n.cohort_dir(data_root)
        c = cls(root)
        for pid in n.find_patient_dirs(root):
            try:
                series, files = n.list_patient_series(root, pid)
            except Exception as e:  # noqa: BLE001 - per-patient isolation, like the CLIs
                c.skipped.append((pid, str(e)))
                continue
            if not files:
                c.skipped.append((pid, "empty series"))
                continue
            c.patients.append(Patient(pid, series, list(files)))
        return c

    def __len__(self):
        return len(self.patients)

    def __iter__(self):
        return iter(self.patients)

    @property
    def n_slices(self):
        return sum(len(p) for p in self.patients)

    def work_items(self, out_root, create=True):
        """[(dicom path, out_root/PGBM-XXX)] in cohort order — the Engine's work list. With
        create=True the patient output directories are made (not wiped: see
        native().setup_output_dir for the reference's wipe)."""
        items = []
        for p in self.patients:
            od = os.path.join(out_root, p.pid)
            if create:
                os.makedirs(od, exist_ok=True)
            items.extend((f, od) for f in p.files)
        return items
