"""Native communicators for independently launched rank processes (torchrun or bench.py's own
launcher): the same C++ `Comm` the CLI uses (src/dist/: RcclComm over xGMI, HostComm over a
process-shared segment). No torch.distributed anywhere.

Rendezvous (one node): every rank derives the same segment name without talking to the others —
from bench.py's job id (NM03_COMM_JOB), or under torchrun from the agent that spawned the local
ranks (its pid and start time, which no other process shares, plus MASTER_PORT). Rank 0 creates the
segment, the others attach; the RCCL unique id and the agreement on whether RCCL came up on every
rank go over it. Every collective runs in native code with deadlines (NM03_COMM_TIMEOUT_S).

Backend choice (`backend` or NM03_COMM): "rccl" | "host" | "auto". auto = RCCL when every rank has
its own GPU, host when ranks share one (NM03_DEVICE_OVERRIDE; RCCL refuses two ranks per device),
and — auto only — the host comm when RCCL initialisation fails on any rank, with the failure
recorded in the returned info (never silent)."""
import atexit
import os

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


def _proc_start_time(pid):
    """Start time of `pid` in clock ticks since boot (field 22 of /proc/<pid>/stat)."""
    with open(f"/proc/{pid}/stat") as f:
        st = f.read()
    return st[st.rindex(")") + 2:].split()[19]


def segment_name():
    """Segment name every local rank of this job derives on its own: bench.py's job id, or the
    spawning agent's (pid, start time) + MASTER_PORT under torchrun, plus the elastic restart count
    and run id: a torchrun restart (--max-restarts) spawns a new generation of workers under the
    same agent, which must not find the previous generation's segment. (pid, start time) names one
    process since boot, so a segment left behind by an earlier job can never be picked up."""
    job = os.environ.get("NM03_COMM_JOB", "")
    if job:
        return f"/nm03-comm-{job}"
    ppid = os.getppid()
    gen = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    run = os.environ.get("TORCHELASTIC_RUN_ID", "")
    run = "".join(c for c in run if c.isalnum())[:24]
    return (f"/nm03-comm-{ppid}-{_proc_start_time(ppid)}-{os.environ.get('MASTER_PORT', '0')}-g{gen}"
            + (f"-{run}" if run else ""))


def unlink_segment(name):
    """Remove a job's named segment if it is still there (a rank 0 that died before unlinking)."""
    try:
        os.unlink("/dev/shm" + name)
    except FileNotFoundError:
        pass


def make_native_comm(rank, world, device, backend=None, timeout_s=None):
    """Returns (comm, info). `comm` is a native `Comm` (rank/size/backend, barrier,
    broadcast_bytes, allgather_bytes, allreduce_sum/max, allgather_f64, sendrecv); `info` records the
    backend used and, if RCCL was abandoned under auto, why."""
    n = native()
    if world <= 1:
        return n.self_comm(), {"backend": "self"}
    timeout_s = float(timeout_s or n.comm_timeout_s())
    be, may_fall_back = resolve_backend(world, backend)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if local_world != world:
        raise RuntimeError(f"native comm: LOCAL_WORLD_SIZE={local_world} != WORLD_SIZE={world}: the shared-segment "
                           "rendezvous serves one node only (launch every rank on this node)")
    name = segment_name()
    if rank == 0:
        unlink_segment(name)  # a segment of this name can only be a dead generation's leftover
    seg = n.shm_create(world, name)[0] if rank == 0 else n.shm_attach(name, world, timeout_s)
    # Every rank removes the name at exit in case rank 0 died before unlinking it (all ranks have
    # attached before any collective returns, so this never races an attach).
    atexit.register(unlink_segment, name)
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
            # No segment for RCCL's own waits during init: a timed-out init must not raise the
            # segment's abort flag, which would also fail the agreement below and with it the
            # host fallback. The segment is attached once every rank agreed.
            comm = n.rccl_comm(rank, world, uid, device, None, min(timeout_s, 60.0))  # init is seconds
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"
    elif not err:
        err = "no RCCL unique id from rank 0"
    agree = n.host_comm(seg, rank, 2 * timeout_s + 10)
    errs = [e.decode() for e in agree.allgather_bytes(err.encode())]
    bad = [(r, e) for r, e in enumerate(errs) if e]
    if not bad:
        # From here on a peer that dies is noticed through the abort flag within milliseconds,
        # not at the collective deadline.
        comm.set_abort_segment(seg)
        return comm, info
    if not may_fall_back:
        raise RuntimeError(f"RCCL initialisation failed on rank(s) {bad}")
    if comm is not None:
        _ABANDONED.append(comm)
    return host, {"backend": "host", "rccl_error": f"rank {bad[0][0]}: {bad[0][1]}"}
