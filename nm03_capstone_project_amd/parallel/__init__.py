"""Data parallelism over MI355X ranks, one process per GPU, on the native communicators
(native_comm.py → src/dist/: RCCL over xGMI, or the host comm when ranks share a GPU): rank
environment, CPU budget and sharding, cohort planning, and the z-slab decomposition of one volume."""
from .dist import auto_threads, cgroup_cpu_stat, cpu_budget, shard_bounds  # noqa: F401
from .cohort_runner import CohortPlan, plan_cohort  # noqa: F401
from .native_comm import make_native_comm, rank_device, rank_env  # noqa: F401
from .volume_slabs import run_volume_slabs, slab_bounds  # noqa: F401
