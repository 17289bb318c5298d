"""bench.py's own rank launcher, rendezvous, native comm and JSON aggregation on the CPU
(--dry-run: everything but the engine). The GPU twin is tests/test_gpu.py::test_bench_multirank."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(tmp_path, *extra, env=None, timeout=240):
    e = dict(os.environ, NM03_COMM_TIMEOUT_S="30")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "2", "--warmup", "1",
           "--data-root", str(tmp_path / "data"), "--out-root", str(tmp_path / "out"), "--numa-data", "off", *extra]
    return subprocess.run(cmd, cwd=str(tmp_path), env=e, capture_output=True, text=True, timeout=timeout)


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launch_n_ranks(tmp_path, n):
    """`python bench.py --gpus N` starts N ranks itself: n_gpus, per-rank arrays; the headline is
    BASELINE config 3 as written (strong: one cohort sharded), weak scaling the secondary."""
    r = _bench(tmp_path, "--gpus", str(n), "--comm", "host")
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == n and rec["config"]["parallelism"] == f"dp{n}"
    assert rec["scaling"] == "strong"
    assert rec["config"]["comm"]["backend"] == "host"
    cohort = rec["config"]["global_batch"]
    assert rec["config"]["weak"]["global_batch"] == n * cohort  # weak: N replicas
    pr = rec["config"]["per_rank"]
    assert all(len(v) == n for v in pr.values())
    # strong: one cohort sharded, every slice exactly once
    assert sum(pr["slices"]) == cohort * 2
    # weak: every rank processes one full cohort per step
    assert rec["config"]["weak"]["per_rank"]["slices"] == [float(cohort * 2)] * n
    # auto batch size: at most 117 slices (233 → 117 + 116, 155 → 78 + 77); passes in flight: 6 when a
    # pass is one or two batches, else 2 (a full cohort per rank: 4 batches)
    assert rec["config"]["batch_size"] == 117
    assert rec["config"]["pipeline_depth"] == 6 and rec["config"]["weak"]["pipeline_depth"] == 2


def test_bench_auto_comm_records_rccl_failure(tmp_path):
    """auto: RCCL cannot come up without a GPU; the run goes on over the host comm and says why."""
    r = _bench(tmp_path, "--gpus", "2", "--no-secondary")
    assert r.returncode == 0, r.stderr
    comm = _json_line(r.stdout)["config"]["comm"]
    assert comm["backend"] == "host" and "rccl_error" in comm


def test_bench_dead_rank_fails_job(tmp_path):
    """A rank that dies makes the job exit non-zero, naming the rank, well before the deadline."""
    t0 = time.monotonic()
    r = _bench(tmp_path, "--gpus", "3", "--comm", "host", env={"NM03_FAULT": "rank_exit:1"})
    dt = time.monotonic() - t0
    assert r.returncode != 0
    assert "rank 1 exited with status 5" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert dt < 120, dt


def test_bench_world_size_mismatch(tmp_path):
    r = _bench(tmp_path, "--gpus", "4", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_bench_single_rank_dry(tmp_path):
    r = _bench(tmp_path)
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and rec["config"]["comm"]["backend"] == "self"
    assert rec["steps"] == 2 and rec["warmup"] == 1
    r = _bench(tmp_path, "--pipeline-depth", "3", "--steps", "4", "--wipe-passes", "3")
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["config"]["pipeline_depth"] == 3 and rec["config"]["per_rank"]["slices"] == [4.0 * 465]


def test_bench_under_torchrun(tmp_path):
    """The driver's multi-GPU form: `python -m torch.distributed.run --nproc-per-node N ... bench.py
    --gpus N` — ranks from torchrun, segment name through the env:// store, one JSON line."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    e = dict(os.environ, NM03_COMM_TIMEOUT_S="30")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "NM03_COMM_JOB"):
        e.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1",
           "--data-root", str(tmp_path / "data"), "--out-root", str(tmp_path / "out"), "--numa-data", "off"]
    r = subprocess.run(cmd, cwd=str(tmp_path), env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 2 and all(len(v) == 2 for v in rec["config"]["per_rank"].values())
    assert rec["config"]["comm"]["backend"] == "host"  # auto: no RCCL without a GPU, recorded
    assert "rccl_error" in rec["config"]["comm"]


def test_bench_emulate_shard_of(tmp_path):
    """--emulate-shard-of N: one rank processes rank 0's share of an N-rank strong-scaling step (465 // N
    slices per pass), with the small-shard pipeline depth, and the record says it is an emulation."""
    r = _bench(tmp_path, "--emulate-shard-of", "8", "--no-secondary", "--wipe-passes", "0")
    assert r.returncode == 0, r.stderr
    rec = _json_line(r.stdout)
    assert rec["metric"].startswith("EMULATION") and rec["vs_baseline"] is None
    assert rec["config"]["emulate_shard_of"] == 8 and rec["config"]["pipeline_depth"] == 6
    assert rec["config"]["batch_size"] == 465 // 8  # the whole 58-slice shard as one batch
    assert rec["config"]["per_rank"]["slices"] == [2.0 * (465 // 8)]
