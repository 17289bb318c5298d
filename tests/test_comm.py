"""Distributed layer on CPU: loopback Comm, fork launcher, torch.distributed (gloo) helpers,
sharding coverage."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from nm03_capstone_project_amd.parallel import dist as D


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_loopback_collectives(native, n):
    assert native.loopback_selftest(n) == [""] * n


def test_launcher_exit_codes(native):
    assert native.launcher_selftest(1) == 0
    assert native.launcher_selftest(2, "ok") == 0
    assert native.launcher_selftest(4, "ok") == 0
    assert native.launcher_selftest(3) == 7  # a failing rank fails the job


def test_launcher_dead_rank_fails_fast(native, capfd):
    """Rank 2 of 3 dies while ranks 0/1 block in a collective: the supervisor raises the abort
    flag, the blocked ranks fail within milliseconds (not at the deadline) and the job exits with
    the dead rank's status, naming it on stderr."""
    import time
    t0 = time.monotonic()
    rc = native.launcher_selftest(3, "die", 60.0, 5.0)
    dt = time.monotonic() - t0
    err = capfd.readouterr().err
    assert rc == 3
    assert "Rank 2 exited with status 3" in err
    assert "rank 2 failed; job aborted" in err
    assert dt < 20, dt  # far below the 60 s collective deadline


def test_launcher_hung_rank_times_out(native, capfd):
    """Rank 2 of 3 hangs outside any collective: the others hit the collective deadline, the job
    is aborted, and the supervisor terminates the straggler after the grace period."""
    import time
    t0 = time.monotonic()
    rc = native.launcher_selftest(3, "hang", 1.5, 1.0)
    dt = time.monotonic() - t0
    err = capfd.readouterr().err
    assert rc != 0
    assert "timed out after 1 s" in err
    assert "sending SIGTERM" in err
    assert dt < 30, dt


def test_host_comm_named_segment(native):
    """Named segment rendezvous (the bench.py / torchrun path): create, attach from a forked
    process, collectives both ways, unlink once everyone attached."""
    seg, name = native.shm_create(2)
    pid = os.fork()
    if pid == 0:  # child: rank 1
        code = 1
        try:
            s1 = native.shm_attach(name, 2, 10.0)
            c1 = native.host_comm(s1, 1, 10.0)
            b = c1.broadcast_bytes(b"", 0)
            g = c1.allgather_bytes(b"r1")
            s = c1.allreduce_sum([5])
            code = 0 if (b == b"plan" and g == [b"rank0", b"r1"] and s == [7]) else 2
        finally:
            os._exit(code)
    seg.wait_attached_and_unlink(10.0)
    assert not os.path.exists("/dev/shm" + name)
    c0 = native.host_comm(seg, 0, 10.0)
    assert c0.backend == "host" and c0.size == 2 and c0.rank == 0
    assert c0.broadcast_bytes(b"plan", 0) == b"plan"
    assert c0.allgather_bytes(b"rank0") == [b"rank0", b"r1"]
    assert c0.allreduce_sum([2]) == [7]
    _, st = os.waitpid(pid, 0)
    assert os.WEXITSTATUS(st) == 0


@pytest.mark.parametrize("n,world", [(0, 3), (1, 4), (466, 8), (25, 2), (7, 7)])
def test_shard_bounds_cover_once(n, world):
    seen = []
    for r in range(world):
        lo, hi = D.shard_bounds(n, r, world)
        seen.extend(range(lo, hi))
        assert hi - lo in (n // world, n // world + 1)
    assert seen == list(range(n))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    try:
        b = D.broadcast_bytes(b"work-list" if rank == 0 else b"", ctx)
        g = D.allgather_bytes(bytes([rank]) * (rank + 1), ctx)
        mx = D.allreduce_max(rank * 2.5, ctx)
        sm = D.allreduce_sum(rank + 1, ctx)
        D.barrier(ctx)
        q.put((rank, b, g, mx, sm))
    finally:
        torch.distributed.destroy_process_group()


def test_torch_gloo_collectives():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, b, g, mx, sm in res:
        assert b == b"work-list"
        assert g == [b"\x00", b"\x01\x01"]
        assert mx == 2.5 and sm == 3


def _cohort_worker(rank, world, port, data_root, out_root, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from nm03_capstone_project_amd.parallel import cohort_runner as C
    ctx = D.init_from_env(backend="gloo", use_gpu=False)
    try:
        plan = C.plan_cohort(data_root, out_root) if rank == 0 else C.CohortPlan()
        data = D.broadcast_bytes(plan.to_bytes() if rank == 0 else b"", ctx)
        plan = C.CohortPlan.from_bytes(data)
        lo, hi = D.shard_bounds(len(plan.items), rank, world)
        q.put((rank, len(plan.items), lo, hi))
    finally:
        torch.distributed.destroy_process_group()


def test_distributed_plan_broadcast(cohort_root, tmp_path):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_cohort_worker, args=(r, world, port, cohort_root, str(tmp_path / "out"), q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
    n = res[0][1]
    assert all(r[1] == n for r in res) and n > 0
    assert res[0][2] == 0 and res[-1][3] == n and res[0][3] == res[1][2]


def test_auto_threads_respects_budget(monkeypatch):
    from nm03_capstone_project_amd.parallel import dist
    monkeypatch.setattr(dist, "cpu_budget", lambda: 16)
    assert dist.auto_threads(1) == 16
    assert dist.auto_threads(8) == 2
    monkeypatch.setattr(dist, "cpu_budget", lambda: 256)
    assert dist.auto_threads(8) == 16
    assert dist.cpu_budget.__name__  # patched
