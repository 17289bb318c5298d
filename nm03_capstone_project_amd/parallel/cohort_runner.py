"""Cohort planning for the Python drivers (bench.py): rank 0 discovers the patients, series and
slice order like the reference (main_sequential.cpp:93-168) and prepares the output directories;
the plan travels as bytes over a native Comm (broadcast_bytes) and every rank takes its contiguous
shard (dist.shard_bounds) — the same plan the native `img_processing_parallel` builds
(src/app/processor.cpp)."""
import json
import os
from dataclasses import dataclass, field

from .._native import native


@dataclass
class CohortPlan:
    patients: list = field(default_factory=list)   # [(pid, out_dir, series_dir, files)]

    @property
    def items(self):
        return [(f, od) for (_, od, _, files) in self.patients for f in files]

    def to_bytes(self):
        return json.dumps(self.patients).encode()

    @staticmethod
    def from_bytes(b):
        return CohortPlan([tuple(p) for p in json.loads(b.decode())])


def plan_cohort(data_root, out_root, wipe=True, replicas=1):
    """Discover PGBM-* patients, order slices like the reference, create/wipe output dirs.
    `replicas` > 1 repeats the cohort with distinct output roots (weak-scaling benchmark)."""
    n = native()
    base = n.cohort_dir(data_root)
    pats = []
    for rep in range(replicas):
        root = out_root if replicas == 1 else os.path.join(out_root, f"replica-{rep:02d}")
        for pid in n.find_patient_dirs(base):
            series, files = n.list_patient_series(base, pid)
            od = os.path.join(root, pid)
            if wipe:
                n.setup_output_dir(od)
            else:
                os.makedirs(od, exist_ok=True)
            pats.append((pid, od, series, list(files)))
    return CohortPlan(pats)
