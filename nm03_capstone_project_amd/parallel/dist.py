"""Rank bookkeeping shared by the Python drivers (bench.py, parallel/*): CPU budget and sharding.
One process per GPU; RANK / WORLD_SIZE / LOCAL_RANK from the launcher's environment
(native_comm.rank_env). All collectives are native (parallel/native_comm.py, src/dist/): only small
control messages travel between ranks — work lists, statuses, timings, z-slab boundary planes — no
pixel data crosses GPUs in the 2D pipeline."""
import os


def cpu_budget():
    """CPUs this process may use: the affinity mask capped by the cgroup v2 CPU quota (cpu.max)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (usage_usec, throttled_usec, nr_throttled, ...); {} when unavailable.
    Deltas over a timed region show whether the host side ran into the CPU quota."""
    out = {}
    try:
        for line in open("/sys/fs/cgroup/cpu.stat"):
            k, v = line.split()[:2]
            out[k] = int(v)
    except (OSError, ValueError):
        pass
    return out


def auto_threads(local_world=None, cap=16):
    """Host I/O threads per rank: the CPU budget shared by the node's ranks (LOCAL_WORLD_SIZE),
    at most `cap` (16 = the reference's omp_set_num_threads(16), main_parallel.cpp:401). The engine
    drivers use the native, topology-aware form (numa.h rank_partition); this is its budget-only
    fallback for callers without a partition."""
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return max(2, min(cap, cpu_budget() // max(1, local_world)))


def shard_bounds(n, rank, world):
    """Contiguous equal blocks (±1 item), deterministic: [n*r/W, n*(r+1)/W)."""
    return n * rank // world, n * (rank + 1) // world
