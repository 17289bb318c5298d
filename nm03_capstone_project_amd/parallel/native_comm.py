"""Native communicators for independently launched rank processes (torchrun or bench.py's own
launcher): the same C++ `Comm` the CLI uses (src/dist/: RcclComm over xGMI, HostComm over a
process-shared segment).

Rendezvous: bench.py's launcher hands every rank a job id (NM03_COMM_JOB) that names the segment;
under torchrun, rank 0 publishes the segment name through the env:// TCPStore (shared with the
torchrun agent when TORCHELASTIC_USE_AGENT_STORE is set) — the only use of torch here. Every
collective runs in native code with deadlines (NM03_COMM_TIMEOUT_S).

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
    used and, if RCCL was abandoned under auto, why.

    Rendezvous: with NM03_COMM_JOB set (bench.py's launcher hands every rank the same job id) the
    segment name derives from it; otherwise (torchrun) rank 0 publishes a fresh name through the
    env:// rendezvous store. Everything after that — the RCCL unique id, the agreement on whether
    RCCL came up on every rank — goes over the shared segment."""
    n = native()
    if world <= 1:
        return n.self_comm(), {"backend": "self"}
    timeout_s = float(timeout_s or n.comm_timeout_s())
    be, may_fall_back = resolve_backend(world, backend)
    job = os.environ.get("NM03_COMM_JOB", "")
    if job:
        name = f"/nm03-comm-{job}"
        seg = n.shm_create(world, name)[0] if rank == 0 else n.shm_attach(name, world, timeout_s)
    else:
        store = _store(rank, world, timeout_s)
        if rank == 0:
            seg, name = n.shm_create(world)
            store.set("shm", name)
        else:
            store.wait(["shm"], timedelta(seconds=timeout_s))
            seg = n.shm_attach(store.get("shm").decode(), world, timeout_s)
    if rank == 0:
        seg.wait_attached_and_unlink(timeout_s)
    host = n.host_comm(seg, rank, timeout_s)
    info = {"backend": be}
    if be == "host":
        return host, info
    # RCCL: unique id from rank 0 over the segment, then every rank reports whether its
    # communicator came up (a slow init may use its whole deadline: the agreement waits longer).
    uid, err = b"", ""
    if rank == 0:
        try:
            uid = n.rccl_unique_id()
        except Exception as e:  # noqa: BLE001 - reported below, on every rank
            err = f"{type(e).__name__}: {e}"
    uid = host.broadcast_bytes(uid, 0)
    comm = None
    if uid:
        try:
            # No segment for RCCL's own waits: a timed-out init must not raise the segment's abort
            # flag, which would also fail the agreement below and with it the host fallback.
            comm = n.rccl_comm(rank, world, uid, device, None, min(timeout_s, 60.0))  # init is seconds
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    elif not err:
        err = "no RCCL unique id from rank 0"
    agree = n.host_comm(seg, rank, 2 * timeout_s + 10)
    errs = [e.decode() for e in agree.allgather_bytes(err.encode())]
    bad = [(r, e) for r, e in enumerate(errs) if e]
    if not bad:
        return comm, info
    if not may_fall_back:
        raise RuntimeError(f"RCCL initialisation failed on rank(s) {bad}")
    if comm is not None:
        _ABANDONED.append(comm)
    return host, {"backend": "host", "rccl_error": f"rank {bad[0][0]}: {bad[0][1]}"}
