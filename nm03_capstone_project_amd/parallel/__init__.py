"""Data parallelism over MI355X ranks with torch.distributed (backend "nccl" = RCCL over xGMI on
ROCm; "gloo" on CPU for tests): shard planning, byte collectives, and the distributed cohort run."""
from .dist import (DistContext, allgather_bytes, allreduce_max, allreduce_sum, auto_threads,  # noqa: F401
                   barrier, broadcast_bytes, cgroup_cpu_stat, cpu_budget, init_from_env, shard_bounds)
from .cohort_runner import CohortPlan, plan_cohort, run_distributed_cohort  # noqa: F401
from .volume_slabs import dilate_slabs, gather_slabs, grow_slabs, run_volume_slabs  # noqa: F401
