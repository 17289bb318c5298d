"""Native communicators for independently launched rank processes (torchrun or bench.py's own
launcher): the same C++ `Comm` the CLI uses (src/dist/: RcclComm over xGMI, HostComm over a
process-shared segment), bootstrapped through the torch rendezvous store.

Only the rendezvous uses torch (the env:// TCPStore at MASTER_ADDR:MASTER_PORT, shared with the
torchrun agent when TORCHELASTIC_USE_AGENT_STORE is set); every collective runs in native code
with deadlines (NM03_COMM_TIMEOUT_S) and the job abort flag of the shared segment.

Backend choice (`backend` or NM03_COMM): "rccl" | "host" | "auto". auto = RCCL when every rank has
its own GPU, host when ranks share one (NM03_DEVICE_OVERRIDE; RCCL refuses two ranks per device),
and — auto only — the host comm when RCCL initialisation fails on any rank, with the failure
recorded in the returned info (never silent)."""
import os
from datetime import timedelta

from .._native import native

# Communicators abandoned after a failed RCCL bring-up under auto: kept alive (never used) so their
# teardown does not run while peers may still be inside the failed initialisation.
_ABANDONED = []


def rank_env():
    """(rank, world, local_rank, local_world) from the launcher's environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    return rank, world, local, local_world


def rank_device(local_rank):
    """HIP device of this rank: NM03_DEVICE_OVERRIDE (all ranks on one GPU) or the local rank."""
    ov = os.environ.get("NM03_DEVICE_OVERRIDE", "")
    return int(ov) if ov != "" else local_rank


def resolve_backend(world, backend=None):
    be = backend or os.environ.get("NM03_COMM", "auto") or "auto"
    if be not in ("auto", "rccl", "host"):
        raise ValueError(f"unknown comm backend {be!r} (rccl | host | auto)")
    if be == "auto" and world > 1 and os.environ.get("NM03_DEVICE_OVERRIDE", "") != "":
        return "host", True
    return ("rccl", True) if be == "auto" else (be, False)


def _store(rank, world, timeout_s):
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    store, _, _ = next(dist.rendezvous("env://", rank=rank, world_size=world, timeout=timedelta(seconds=timeout_s)))
    return dist.PrefixStore("nm03_comm", store)


def make_native_comm(rank, world, device, backend=None, timeout_s=None):
    """Returns (comm, info). `comm` is a native `Comm` (rank/size/backend, barrier,
    broadcast_bytes, allgather_bytes, allreduce_sum/max, allgather_f64); `info` records the backend
    used and, if RCCL was abandoned under auto, why."""
    n = native()
    if world <= 1:
        return n.self_comm(), {"backend": "self"}
    timeout_s = float(timeout_s or n.comm_timeout_s())
    be, may_fall_back = resolve_backend(world, backend)
    store = _store(rank, world, timeout_s)
    # Every job has a shared segment: the host collectives, and the abort flag RCCL waits watch.
    if rank == 0:
        seg, name = n.shm_create(world)
        store.set("shm", name)
        seg.wait_attached_and_unlink(timeout_s)
    else:
        store.wait(["shm"], timedelta(seconds=timeout_s))
        seg = n.shm_attach(store.get("shm").decode(), world, timeout_s)
    info = {"backend": be}
    if be == "rccl":
        comm, err = None, ""
        try:
            if rank == 0:
                uid = b""
                try:
                    uid = n.rccl_unique_id()
                finally:
                    store.set("uid", uid)  # empty on failure: peers fail fast instead of waiting
            else:
                store.wait(["uid"], timedelta(seconds=timeout_s))
                uid = store.get("uid")
            comm = n.rccl_comm(rank, world, uid, device, seg, timeout_s)
        except Exception as e:  # noqa: BLE001 - reported below, on every rank
            err = f"{type(e).__name__}: {e}"
        store.set(f"rccl_status_{rank}", err or "ok")
        keys = [f"rccl_status_{r}" for r in range(world)]
        store.wait(keys, timedelta(seconds=timeout_s))
        bad = [(r, store.get(k).decode()) for r, k in enumerate(keys)]
        bad = [(r, s) for r, s in bad if s != "ok"]
        if not bad:
            return comm, info
        if not may_fall_back:
            raise RuntimeError(f"RCCL initialisation failed on rank(s) {bad}")
        info = {"backend": "host", "rccl_error": f"rank {bad[0][0]}: {bad[0][1]}"}
        if comm is not None:
            _ABANDONED.append(comm)
    return n.host_comm(seg, rank, timeout_s), info
