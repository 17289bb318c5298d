"""Distributed layer on CPU: loopback Comm, fork launcher, native host comm across processes,
sharding coverage."""
import os

import pytest

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


def test_plan_broadcast_over_native_host_comm(cohort_root, tmp_path, native):
    """bench.py's planning path without torch: rank 0 plans the cohort, the plan travels over the
    native host comm (forked rank), every rank takes its contiguous shard."""
    from nm03_capstone_project_amd.parallel import cohort_runner as C
    seg, name = native.shm_create(2)
    r_out, w_out = os.pipe()
    pid = os.fork()
    if pid == 0:  # rank 1
        code = 1
        try:
            c1 = native.host_comm(native.shm_attach(name, 2, 10.0), 1, 10.0)
            plan = C.CohortPlan.from_bytes(c1.broadcast_bytes(b"", 0))
            lo, hi = D.shard_bounds(len(plan.items), 1, 2)
            os.write(w_out, f"{len(plan.items)} {lo} {hi}".encode())
            code = 0
        finally:
            os._exit(code)
    seg.wait_attached_and_unlink(10.0)
    c0 = native.host_comm(seg, 0, 10.0)
    plan = C.plan_cohort(cohort_root, str(tmp_path / "out"))
    assert C.CohortPlan.from_bytes(c0.broadcast_bytes(plan.to_bytes(), 0)).items == plan.items
    _, st = os.waitpid(pid, 0)
    assert os.WEXITSTATUS(st) == 0
    n, lo, hi = map(int, os.read(r_out, 100).decode().split())
    assert n == len(plan.items) > 0 and lo == D.shard_bounds(n, 0, 2)[1] and hi == n


def test_auto_threads_respects_budget(monkeypatch):
    from nm03_capstone_project_amd.parallel import dist
    monkeypatch.setattr(dist, "cpu_budget", lambda: 16)
    assert dist.auto_threads(1) == 16
    assert dist.auto_threads(8) == 2
    monkeypatch.setattr(dist, "cpu_budget", lambda: 256)
    assert dist.auto_threads(8) == 16
    assert dist.cpu_budget.__name__  # patched


def test_segment_name_changes_with_elastic_restart(monkeypatch):
    """Under torchrun a restarted generation of workers (same agent, same MASTER_PORT) derives a new
    segment name (TORCHELASTIC_RESTART_COUNT / RUN_ID), so it never attaches to a segment the
    previous generation left behind."""
    from nm03_capstone_project_amd.parallel import native_comm as nc
    monkeypatch.delenv("NM03_COMM_JOB", raising=False)
    monkeypatch.setenv("MASTER_PORT", "29500")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job/1")
    a = nc.segment_name()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    b = nc.segment_name()
    assert a != b and a.startswith("/nm03-comm-") and "/" not in a[1:] and "/" not in b[1:]
    monkeypatch.setenv("NM03_COMM_JOB", "abc")
    assert nc.segment_name() == "/nm03-comm-abc"


def test_native_comm_refuses_multi_node_world(monkeypatch):
    from nm03_capstone_project_amd.parallel import native_comm as nc
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    import pytest
    with pytest.raises(RuntimeError, match="LOCAL_WORLD_SIZE"):
        nc.make_native_comm(0, 4, 0, "host", timeout_s=1)


def test_deferred_rccl_comm_control_plane_without_gpu(native):
    """Before promote() the deferred RCCL communicator is the shared-memory host comm (no HIP): the
    start-up collectives work on a machine without a GPU; promote() finds RCCL unusable, the ranks
    agree on it over the control plane and stay there (backend "host", the reason recorded) instead
    of failing or hanging."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    seg, name = native.shm_create(1)
    c = native.deferred_rccl_comm(0, 1, 0, seg, 5.0)
    c.barrier()
    assert c.broadcast_bytes(b"work-list", 0) == b"work-list"
    assert c.allreduce_max([2.5]) == [2.5]
    assert c.transport_size == -1 and c.data_plane_times["start_s"] == -1
    c.promote()
    assert c.backend == "host" and c.fallback_error and c.transport_size == -1
    assert c.allreduce_sum([7]) == [7] and c.broadcast_bytes(b"after", 0) == b"after"
    seg.wait_attached_and_unlink(5.0)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_deferred_rccl_falls_back_together(native, n):
    """launch_ranks' RCCL ranks without a GPU: the start-up collectives run on the shared-memory
    control plane, every rank's RCCL bring-up fails, the ranks agree on it in promote() and finish on
    the control plane — the job succeeds instead of hanging or failing one rank."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check")
    assert native.launcher_selftest(n, "ok", 30.0, 5.0, "rccl") == 0
