"""torch.distributed helpers. One process per GPU; RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from
the environment (torchrun). Only small control messages travel (work lists, statuses, timings):
no pixel data crosses GPUs."""
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: "torch.device" = None

    @property
    def is_root(self):
        return self.rank == 0

    @property
    def device_index(self):
        """HIP device of this rank (the local rank unless NM03_DEVICE_OVERRIDE is set)."""
        return self.device.index if (self.device is not None and self.device.type == "cuda") else 0


def init_from_env(backend=None, use_gpu=None):
    """Initialise the default process group when WORLD_SIZE > 1; always returns a DistContext.

    Rehearsal overrides (several ranks on a one-GPU box): NM03_DIST_BACKEND=gloo selects the
    collective backend, NM03_DEVICE_OVERRIDE=<i> pins every rank to device i (RCCL refuses two
    ranks on one device, gloo does not)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    dev_index = int(os.environ.get("NM03_DEVICE_OVERRIDE", local))
    dev = torch.device("cuda", dev_index) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev_index)
    be = backend or os.environ.get("NM03_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": dev} if (be == "nccl" and use_gpu) else {}
        try:
            dist.init_process_group(be, rank=rank, world_size=world, **kw)
        except TypeError:
            dist.init_process_group(be, rank=rank, world_size=world)
    return DistContext(rank, world, local, be if world > 1 else "none", dev)


def _active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _dev(ctx):
    return ctx.device if (ctx is not None and ctx.backend == "nccl") else torch.device("cpu")


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
    at most `cap` (16 = the reference's omp_set_num_threads(16), main_parallel.cpp:401). Running
    more busy threads than the cgroup quota allows gets the whole process throttled."""
    if local_world is None:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return max(2, min(cap, cpu_budget() // max(1, local_world)))


def shard_bounds(n, rank, world):
    """Contiguous equal blocks (±1 item), deterministic: [n*r/W, n*(r+1)/W)."""
    return n * rank // world, n * (rank + 1) // world


def barrier(ctx=None):
    if _active():
        if ctx is not None and ctx.backend == "nccl":
            t = torch.ones(1, device=ctx.device)
            dist.all_reduce(t)
            torch.cuda.synchronize(ctx.device)
        else:
            dist.barrier()
    elif torch.cuda.is_available() and ctx is not None and ctx.device is not None and ctx.device.type == "cuda":
        torch.cuda.synchronize(ctx.device)


def broadcast_bytes(data, ctx=None, src=0):
    """Broadcast a bytes object from `src` (ncclBroadcast of a uint8 tensor under RCCL)."""
    if not _active():
        return data
    dev = _dev(ctx)
    n = torch.tensor([len(data) if data is not None else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    if dist.get_rank() == src and len(data):
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    if buf.numel():
        dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def allgather_bytes(data, ctx=None):
    """All-gather variable-length bytes (sizes first, then padded payloads)."""
    if not _active():
        return [data]
    dev = _dev(ctx)
    world = dist.get_world_size()
    n = torch.tensor([len(data)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = max(int(s.item()) for s in sizes)
    mine = torch.zeros(max(mx, 1), dtype=torch.uint8, device=dev)
    if len(data):
        mine[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    outs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(outs, mine)
    return [bytes(o[:int(s.item())].cpu().numpy().tobytes()) for o, s in zip(outs, sizes)]


def allreduce_max(x, ctx=None):
    if not _active():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=_dev(ctx))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(x, ctx=None):
    if not _active():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_dev(ctx))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.item()
