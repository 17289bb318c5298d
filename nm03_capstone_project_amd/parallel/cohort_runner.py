"""Distributed cohort processing with torch.distributed — the Python twin of the native
`img_processing_parallel --gpus N` (src/app/processor.cpp): rank 0 plans (patients, series,
output directories), broadcasts the work list, every rank runs its contiguous shard through its
own native Engine, and rank 0 gathers per-slice statuses in the global order."""
import json
import os
from dataclasses import dataclass, field

from .._native import native
from .dist import allgather_bytes, broadcast_bytes, shard_bounds


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


def run_distributed_cohort(engine, plan, ctx):
    """Run `plan` sharded over ranks. Returns (global statuses on rank 0 or None, local times)."""
    data = broadcast_bytes(plan.to_bytes() if ctx.is_root else b"", ctx)
    plan = CohortPlan.from_bytes(data)
    items = plan.items
    lo, hi = shard_bounds(len(items), ctx.rank, ctx.world)
    statuses, times = engine.run(items[lo:hi])
    gathered = allgather_bytes(json.dumps(statuses).encode(), ctx)
    if not ctx.is_root:
        return None, times
    out = []
    for g in gathered:
        out.extend(tuple(s) for s in json.loads(g.decode()))
    return out, times
