#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json metric): DICOM slices/sec through the full pipeline on the
T1+C cohort, one MI355X per rank.

One step = the whole synthetic T1+C cohort (20 patients × 21–25 slices of 256² u16)
per rank, end to end: read every DICOM file from disk, parse, upload, median 7×7 → 9×9 unsharp →
SRG band → seeded region growing → dilation 3 → render 512² (original + segmentation) → JPEG q75 on
the GPU → write both JPEG files per slice. Nothing is cached between steps.

Headline = BASELINE config 3 as written (strong scaling, round 5): every step is ONE 465-slice
cohort sharded contiguously over the N ranks, so the total work per step is fixed as N grows
("scaling": "strong", config.global_batch = 465). The weak-scaling figure (N cohort replicas with
distinct output trees, one full cohort per rank per step) is measured right after and reported under
config.weak; `--scaling weak` swaps the two. At N = 1 they coincide.

Ranks: `python bench.py --gpus N` starts N rank processes itself (before anything touches a GPU)
and supervises them; under torchrun (WORLD_SIZE set) each process is one rank. Either way the
ranks talk through the native communicator the CLI uses (src/dist: RCCL over xGMI, or the
shared-memory host comm when ranks share a GPU), bootstrapped via the torch rendezvous store.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
    NM03_DEVICE_OVERRIDE=0 python bench.py --gpus 4      # 4 ranks sharing GPU 0 (rehearsal)
"""
import argparse
import json
import os
import resource
import shutil
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "DICOM slices/sec through full pipeline (T1+C cohort) at 1/2/4/8 MI355X"
# The reference publishes no number; BASELINE.md defines the comparison point as the measured
# reference-equivalent CPU run of the same cohort (golden model, 16 threads, batch 25, serial
# export: profiles/baselines/c3_cpu.json).
BASELINE_SLICES_PER_S = 171.43


class _roctx_range:
    """roctx range for rocprofv3 --marker-trace timelines (tools/timeline.py); no-op unless NM03_ROCTX=1."""
    _lib = None

    def __init__(self, name):
        self.name = name.encode()
        if _roctx_range._lib is None:
            _roctx_range._lib = False
            if os.environ.get("NM03_ROCTX", "0") not in ("", "0"):
                import ctypes
                try:
                    _roctx_range._lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
                except OSError:
                    pass

    def __enter__(self):
        if self._lib:
            self._lib.roctxRangePushA(self.name)

    def __exit__(self, *exc):
        if self._lib:
            self._lib.roctxRangePop()


def _scratch():
    """Where the synthetic cohort and the JPEGs live: tmpfs (/dev/shm) when writable, else /tmp.

    The box's root filesystem is an overlay whose metadata/journal path serialises small-file
    writes across processes (round-1 I/O scaling probe: 4 processes reach ~2.6x one process on /tmp,
    ~4x on /dev/shm; profiles/io_scaling.txt). Every byte is still read and written through the
    same syscalls; tmpfs only removes that container artefact, the analogue of a local NVMe with a
    warm page cache where the reference's cohort lives."""
    shm = "/dev/shm"
    return shm if os.path.isdir(shm) and os.access(shm, os.W_OK) else "/tmp"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="which figure is the headline value (default strong: BASELINE config 3, one cohort "
                         "sharded over the ranks); the other is reported next to it")
    ap.add_argument("--no-secondary", action="store_true", help="skip the other scaling mode's measurement")
    # 200 wipe passes ≈ 0.3-0.7 s timed (20 passes were 43 ms: one 10 ms hiccup or the reaper's final
    # drain moved the figure by 25-40%).
    ap.add_argument("--wipe-passes", type=int, default=200,
                    help="also time this many passes that each first wipe their output directories (the "
                         "reference's per-run rm -rf; reported as config.wipe_each_pass; 0 = skip)")
    ap.add_argument("--wipe-mode", choices=("reaper", "inline"), default="reaper",
                    help="wipe passes: rename each output directory aside and delete it on 2 background "
                         "reaper threads (cohort.h OutputReaper; the final drain is inside the clock), or "
                         "unlink everything before the pass on 8 threads (round 3)")
    # 6 deletion threads: the wipe figure over 200 passes rose in three interleaved experiments on three
    # boxes against 4 (179k -> 190k, 203k -> 239k with 2 creators, 196k -> 202k; 8 threads 220k in the
    # third), profiles/r6/wipe_knobs/.
    ap.add_argument("--reaper-threads", type=int, default=6,
                    help="background deletion threads of the wipe passes (--wipe-mode reaper)")
    ap.add_argument("--wipe-depth", type=int, default=3,
                    help="passes in flight (output trees) for the wipe passes")
    # One upload copy per batch, after its loads (progressive upload off): with batches fitted to the
    # shard the engine's progressive copies (2 MiB, or a quarter of the batch) cost more in slot-thread
    # wake-ups and copy set-up than their overlap with the loads saves. Minimum copy size 2 MiB → 4 →
    # 6 → 64 MiB → off: headline 431k → 441k → 453k → 479k ≈ 460k (off), and at the driver's 20 steps
    # the 8-rank shard 333k → 340k → 370k → 367k ≈ 357k, the 4-rank one 388k → 403k → 405k → 421k ≈
    # 404k (interleaved, several boxes: profiles/r6/upload_chunk/).
    ap.add_argument("--upload-chunk-kb", type=int, default=0,
                    help="EngineConfig.upload_chunk_kb: smallest progressive upload copy (-1 = engine default, 2 MiB; "
                         "a copy is also at least a quarter of the batch); 0 = one copy per batch after its loads")
    ap.add_argument("--create-writers", type=int, default=-1,
                    help="EngineConfig.create_writers: pool workers writing a batch's JPEGs at once while "
                         "its directories are being filled (-1 = engine default, 0 = no limit)")
    # 4 slots (round 2: 96 slices × 4 won over 64 × 6, profiles/r2/batch_streams/; round 6: 4 slots over
    # 5 and 6, profiles/r6/streams/). Batch size: see `batch` below.
    ap.add_argument("--batch-size", type=int, default=0,
                    help="slices per batch (engine capacity); 0 = auto: the rank's shard if at most 117 slices, "
                         "else 117 (equal-size batches)")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--threads", type=int, default=0,
                    help="host I/O threads per rank (0 = the rank's CPU partition and budget share, ≤16)")
    ap.add_argument("--single-pass-cap", type=int, default=0,
                    help="batch cap of the capped single passes (0 = ceil(shard / streams))")
    ap.add_argument("--single-passes", type=int, default=100,
                    help="also time this many single strong-scaling passes (one cohort sharded over the "
                         "ranks, nothing else in flight; config.strong.single_pass_ms; 0 = skip)")
    ap.add_argument("--comm", choices=("auto", "rccl", "host"), default=os.environ.get("NM03_COMM", "auto"))
    ap.add_argument("--data-root", default=os.path.join(_scratch(), "nm03_bench_data"))
    ap.add_argument("--out-root", default=os.path.join(_scratch(), "nm03_bench_out"))
    ap.add_argument("--keep-data", action="store_true", help="keep a generated dataset in tmpfs after the run")
    ap.add_argument("--keep-output", action="store_true")
    ap.add_argument("--pipeline-depth", type=int, default=0,
                    help="passes in flight (each with its own output tree); 0 = auto: 6 when the rank's pass is "
                         "one or two batches (strong-scaling shards: a pass is then mostly latency, and more "
                         "passes in flight overlap it), else 2")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one blocking engine call per pass; by default pass k+1 is submitted before pass k "
                         "finished (Engine.submit/wait) so the slot ring never drains between passes")
    ap.add_argument("--stream-steps", action="store_true",
                    help="submit the K timed cohort passes as one work stream (the engine pipelines across pass "
                         "boundaries as it does across patients) instead of one engine call per pass; every pass "
                         "writes its own output tree")
    ap.add_argument("--emulate-shard-of", type=int, default=1,
                    help="one rank only: measure rank 0's strong-scaling shard of an N-rank job (465 / N slices "
                         "per pass) — the per-GPU rate of config 3 at N GPUs without N GPUs (host DRAM and CPU "
                         "contention between ranks not included); the JSON says so")
    ap.add_argument("--host-only", action="store_true",
                    help="host path only (EngineConfig.host_only): every DICOM load and JPEG write of a real "
                         "run, the GPU stages replaced by fixed JPEG segments; measures slices per host "
                         "CPU-second, no GPU needed. Not the headline metric (the JSON says so)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the launcher, rendezvous, comm, sharding and aggregation: every step "
                         "of a real run except the engine (no GPU); the JSON value is meaningless")
    ap.add_argument("--cli-runs", type=int, default=10,
                    help="also time this many whole invocations of the unmodified img_processing_parallel --gpus N "
                         "on the bench cohort, as the reference measured its binaries (hyperfine, README.md:92-96); "
                         "reported as config.cli_wall (0 = skip)")
    ap.add_argument("--numa-data", choices=("auto", "off"), default="auto",
                    help="auto: one input copy per NUMA node, each rank reads the copy on its GPU's node")
    ap.add_argument("--cpu-profile", default="",
                    help="sample the host CPU over the headline's timed steps (cpu_sampler.h) into PATH.rank<r>; "
                         "symbolise with tools/cpu_profile.py")
    ap.add_argument("--cpu-profile-period-us", type=int, default=250,
                    help="one sample per this much process CPU time (--cpu-profile)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------------
# Launcher: `--gpus N` without WORLD_SIZE. Runs before anything touches a GPU (no torch.cuda, no
# HIP call in this process): it only spawns the N rank processes and watches them.
# ------------------------------------------------------------------------------------------------
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def thread_cpu_by_name():
    """CPU seconds of this process's live threads, summed per thread name. Each thread's CPU clock
    (clockid (~tid << 3) | 6, the kernel's per-thread CPUCLOCK_SCHED) has ns resolution; the
    user + system ticks of /proc/.../stat (10 ms) are the fallback — too coarse for the threads
    that run a few ms in a 20-step window."""
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        try:
            sec = time.clock_gettime_ns(((~int(tid)) << 3) | 6) * 1e-9
        except OSError:  # the thread exited meanwhile, or no per-thread clocks
            fields = st[st.rindex(")") + 2:].split()
            sec = (int(fields[11]) + int(fields[12])) / tick
        out[name] = out.get(name, 0.0) + sec
    return out


def launch(args, argv, grace_s=5.0):
    n = args.gpus
    port = _free_port()  # only for code that wants an env:// store; the native comm uses the job id
    job = os.urandom(8).hex()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NM03_COMM_JOB=job)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc, failed_at = 0, None
    while any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            code = p.poll()
            if code not in (None, 0) and rc == 0:
                rc = code if code > 0 else 128 - code
                failed_at = time.monotonic()
                print(f"bench: rank {r} exited with status {code}", file=sys.stderr, flush=True)
        if failed_at is not None:
            waited = time.monotonic() - failed_at
            for p in procs:
                if p.poll() is None:
                    if waited > 2 * grace_s:
                        p.kill()
                    elif waited > grace_s:
                        p.send_signal(signal.SIGTERM)
        time.sleep(0.01)
    for r, p in enumerate(procs):
        if p.returncode not in (0, None) and rc == 0:
            rc = p.returncode if p.returncode > 0 else 128 - p.returncode
            print(f"bench: rank {r} exited with status {p.returncode}", file=sys.stderr, flush=True)
    # A rank 0 killed before it unlinked the job's segment leaves it in /dev/shm (RAM): remove it.
    try:
        os.unlink(f"/dev/shm/nm03-comm-{job}")
    except FileNotFoundError:
        pass
    return rc


# ------------------------------------------------------------------------------------------------
# One rank
# ------------------------------------------------------------------------------------------------
def _pass_items(items, out_root, k):
    """The work list of stream-steps pass k: same inputs, output tree out_root/pass-k/..."""
    out = []
    made = set()
    for f, od in items:
        d = os.path.join(out_root, f"pass-{k:03d}", os.path.relpath(od, out_root))
        if d not in made:
            os.makedirs(d, exist_ok=True)
            made.add(d)
        out.append((f, d))
    return out


class _DryEngine:
    """--dry-run stand-in for the native Engine: every slice 'succeeds' instantly."""

    def submit(self, work, batch_cap=0):
        return work

    def wait(self, work):
        return self.run_list(work)

    def run_list(self, work, batch_cap=0):
        import numpy as np
        zero = {k: 0.0 for k in ("load_s", "load_cpu_s", "h2d_s", "kernels_s", "write_s", "write_cpu_s",
                                 "slot_cpu_s")}
        return np.zeros(len(work), dtype=np.int32), {}, zero


def run_rank(args):
    import torch  # the native extension shares torch's HIP runtime: import torch first

    import nm03_capstone_project_amd as nm
    from nm03_capstone_project_amd.parallel.cohort_runner import CohortPlan, plan_cohort
    from nm03_capstone_project_amd.parallel.dist import cgroup_cpu_stat, shard_bounds
    from nm03_capstone_project_amd.parallel.native_comm import make_native_comm, rank_device, rank_env
    from nm03_capstone_project_amd.parallel.numa_data import (ensure_node_replicas, localize_items, numa_nodes,
                                                              replica_root)

    rank, world, local_rank, local_world = rank_env()
    device = rank_device(local_rank)
    n = nm.native()
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(device)
    comm, comm_info = make_native_comm(rank, world, device, args.comm)
    is_root = rank == 0

    # Where this rank runs: its GPU's PCI bus id, and a CPU partition of that GPU's NUMA node that no
    # other local rank shares, with a pool sized to it and to the rank's share of the CPU budget
    # (numa.h; the reference has one machine-wide budget, main_parallel.cpp:401). All-gathered: the
    # record shows N distinct devices, or the job fails when two ranks resolved to the same GPU
    # without NM03_DEVICE_OVERRIDE asking for that.
    shared_device = os.environ.get("NM03_DEVICE_OVERRIDE", "") != ""
    rank_nodes = [n.numa_device_node(rank_device(r)) if gpu else -1 for r in range(local_world)]
    part = n.rank_partition(rank_nodes, local_rank, n.cpu_budget())
    if args.threads <= 0:
        args.threads = part["threads"]
    bus = n.device_bus_id(device) if gpu else ""
    devices = comm.gather_rank_devices(device, bus, part["node"], n.format_cpulist(part["cpus"]), args.threads)
    comm_info["nranks"] = comm.transport_size
    dup = [(a, b) for a in range(world) for b in range(a + 1, world)
           if devices[a]["bus_id"] and devices[a]["bus_id"] == devices[b]["bus_id"]]
    if dup and not shared_device:
        a, b = dup[0]
        raise SystemExit(f"bench: ranks {a} and {b} resolved to the same GPU {devices[a]['bus_id']} "
                         "(set NM03_DEVICE_OVERRIDE=<device> to share one GPU deliberately)")

    # Input cohort in tmpfs: one copy per NUMA node on multi-socket hosts (numa_data.py), so every
    # rank reads the copy on its own GPU's node.
    nodes = numa_nodes(n.numa_node_cpus) if args.numa_data == "auto" else []
    roots = [replica_root(args.data_root, k) for k in nodes] or [args.data_root]
    if local_rank == 0:
        ensure_node_replicas(args.data_root, nodes, lambda root: n.synth_cohort(root, threads=16), n.numa_node_cpus)
    comm.barrier()
    dev_node = n.numa_device_node(device) if nodes else -1
    local_root = replica_root(args.data_root, dev_node) if dev_node in nodes else roots[0]

    # Fault injection (tests): NM03_FAULT=rank_exit:<r> makes rank r die here (log.h FaultPlan).
    fail_rank = next((f.split(":", 1)[1] for f in os.environ.get("NM03_FAULT", "").split(",")
                      if f.startswith("rank_exit:")), "")
    if fail_rank != "" and int(fail_rank) == rank:
        print(f"bench: rank {rank}: injected failure", file=sys.stderr, flush=True)
        os._exit(5)
    def pipeline_depth(shard_len):
        if args.pipeline_depth > 0:
            return args.pipeline_depth
        # Passes in flight by batches per pass. One or two (the strong-scaling shards of 4- and 8-rank
        # jobs): 6, so the slots still find queued batches while this thread wakes up to submit the
        # next pass — at the driver's 20 steps the 58-slice shard measured the same median with 4 and
        # 6 but no slow outliers with 6 (worst of 9 runs 304k vs 204k slices/s, profiles/r6/
        # shard_depth/), and a job's time is its slowest rank's. Three or more (the whole cohort, the
        # 2-rank shard): 2 — depths 2, 3 and 4 were within the box noise for the cohort over three
        # interleaved experiments at 20 steps and equal at 3000 (412k vs 409k), while 6 trailed 2 and 3
        # for the 2-rank shard in all three (profiles/r6/depth_full/).
        batches = -(-shard_len // max(1, batch))
        return 6 if batches <= 2 else 2

    def shard(scaling, out_root):
        """This rank's work list: weak = its own cohort replica, strong = its block of one cohort."""
        replicas = world if scaling == "weak" else 1
        plan_bytes = plan_cohort(roots[0], out_root, wipe=True, replicas=replicas).to_bytes() if is_root else b""
        plan = CohortPlan.from_bytes(comm.broadcast_bytes(plan_bytes, 0))
        items = plan.items
        lo, hi = shard_bounds(len(items), rank, world)
        if world == 1 and args.emulate_shard_of > 1 and scaling == "strong":
            hi = len(items) // args.emulate_shard_of  # rank 0's share of an N-rank job
        return localize_items(items[lo:hi], roots[0], local_root), len(items)

    # Slices per batch (the engine's capacity) from the rank's primary shard, unless --batch-size
    # says: the whole shard when it is at most 117 slices (the 58- and 116-slice shards of 8- and
    # 4-rank jobs run as one batch sized to fit), else batches of at most 117 (the 465-slice cohort as
    # 4 × 116-117, the 233-slice shard of a 2-rank job as 117 + 116). Fixed 96-slice batches left a
    # 116-slice shard as 58 + 58 and the cohort as 5 × 93; at the driver's 20 steps the fitted sizes
    # measured 392k vs 346k (4 ranks) and 333k vs 329k (8 ranks) slices/s per GPU, and the cohort
    # 428k vs 406k over 3000 steps (profiles/r6/batch_size/). Much larger batches (233, 465) gained
    # more over long runs but spread widely over 20 steps, where a pass's fill and drain weigh more.
    if args.batch_size > 0:
        batch = args.batch_size
    else:
        batch = max(1, min(len(shard(args.scaling, args.out_root)[0]), 117))
    cfg = nm.PipelineConfig(batch_size=batch, streams=args.streams, threads=args.threads, device=device)
    ecfg = cfg.engine_config()
    ecfg.cpus = part["cpus"]
    ecfg.host_only = args.host_only
    if args.create_writers >= 0:
        ecfg.create_writers = args.create_writers
    if args.upload_chunk_kb >= 0:
        ecfg.upload_chunk_kb = args.upload_chunk_kb
    engine = _DryEngine() if args.dry_run else n.Engine(ecfg)

    def measure(scaling, out_root, steps, warmup, wipe=False, profile=""):
        mine, global_items = shard(scaling, out_root)
        work = n.WorkList(mine)  # the shard's work list in native form (built once, like the plan)
        # Pipelined passes rotate over `depth` output trees: runs in flight never write the same
        # file (pass k+depth is submitted only after pass k finished).
        depth = 1 if args.no_pipeline else pipeline_depth(len(mine))
        if wipe and not args.no_pipeline:
            # A wipe pass's set-up (wipe + rediscovery) runs on this thread while earlier passes are
            # in the engine; with 3 trees it overlaps two passes instead of one.
            depth = max(depth, args.wipe_depth)
        trees = [mine] + [_pass_items(mine, out_root, j) for j in range(1, depth)]
        works = [work] + [n.WorkList(t) for t in trees[1:]]
        # wipe: every pass first empties its patients' output directories, as every reference run
        # does (setupOutputDirectory, main_sequential.cpp:32-47), so files are created, not rewritten.
        tree_dirs = [sorted({od for _, od in t}) for t in trees]
        # Wipe passes over whole cohorts (weak scaling, or one rank) also redo the rest of a
        # reference run's set-up inside the timed region (main_sequential.cpp:93-168): discover the
        # patients, list and order every series, and build the work list from that, every pass.
        rediscover = wipe and (scaling == "weak" or world == 1)
        my_out = out_root if world == 1 else os.path.join(out_root, f"replica-{rank:02d}")

        reaper = n.OutputReaper(args.reaper_threads) if wipe and args.wipe_mode == "reaper" else None
        # Output root of tree j (pass-j trees mirror the layout under out_root/pass-00j).
        tree_roots = [my_out] + [os.path.join(out_root, f"pass-{j:03d}", os.path.relpath(my_out, out_root))
                                 for j in range(1, depth)]

        def discover(j, with_reaper):
            """One native call: patients, per-patient wipe (reaper) or mkdir, series, work list."""
            return n.WorkList.discover(local_root, tree_roots[j], reaper if with_reaper else None)

        if rediscover and [tuple(x) for x in discover(0, False).items()] != [tuple(x) for x in mine]:
            raise SystemExit(f"rank {rank}: rediscovered cohort differs from the planned shard")

        def pass_work(k):
            """Native work list of pass k; wipe passes first empty the pass's output tree (the
            reference's per-run rm -rf + mkdir)."""
            j = k % depth
            if rediscover and reaper is not None:
                return discover(j, True)  # wipes each patient directory as it goes
            if reaper is not None:
                reaper.wipe(tree_dirs[j])
            elif wipe:
                n.setup_output_dirs(tree_dirs[j], 8)
            if not rediscover:
                return works[j]
            return discover(j, False)

        def passes(k_total, sink):
            if args.no_pipeline:
                for k in range(k_total):
                    w = pass_work(k)
                    with _roctx_range("bench.step"):
                        sink(*engine.run_list(w))
                return
            pending = []
            for k in range(k_total):
                pending.append(engine.submit(pass_work(k)))
                if len(pending) == depth:
                    sink(*engine.wait(pending.pop(0)))
            for t in pending:
                sink(*engine.wait(t))

        def check_warm(codes, msgs, _):
            if msgs:
                raise SystemExit(f"rank {rank}: {len(msgs)} slices failed in warmup: {list(msgs.items())[:3]}")
        # Every output tree is written once before the clock starts: with fewer warmup passes than
        # trees (depth 4 for small shards, warmup 1 for the secondary figure) the first pass into a
        # fresh tree — file creation, 100-250 ms for 930 files — landed inside the timed region.
        passes(max(warmup, depth), check_warm)
        stream = None
        if args.stream_steps:
            stream = n.WorkList([it for k in range(steps) for it in _pass_items(mine, out_root, k)])
        stage = {"load_s": 0.0, "load_cpu_s": 0.0, "h2d_s": 0.0, "kernels_s": 0.0, "write_s": 0.0,
                 "write_cpu_s": 0.0, "slot_cpu_s": 0.0}
        ok = 0
        comm.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        cg0 = cgroup_cpu_stat()
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        th0 = thread_cpu_by_name()
        if profile and not n.cpu_profile_start(args.cpu_profile_period_us):
            raise SystemExit(f"rank {rank}: cannot start the CPU sampler")
        t0 = time.perf_counter()
        if stream is not None:
            with _roctx_range("bench.steps"):
                codes, msgs, times = engine.run_list(stream)
            ok += len(codes) - len(msgs)
            for k in stage:
                stage[k] += times[k]
        else:
            def sink(codes, msgs, times):
                nonlocal ok
                ok += len(codes) - len(msgs)
                for k in stage:
                    stage[k] += times[k]
            with _roctx_range("bench.steps"):
                passes(steps, sink)
        if reaper is not None:
            reaper.drain()  # the timed passes' deletions are part of their cost
        t_own = time.perf_counter() - t0  # this rank's own time, before waiting for the others
        if profile:
            nsamp = n.cpu_profile_stop(f"{profile}.rank{rank}")
            print(f"bench: rank {rank}: {nsamp} CPU samples -> {profile}.rank{rank}", file=sys.stderr, flush=True)
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        comm.barrier()
        dt = time.perf_counter() - t0
        cg1 = cgroup_cpu_stat()
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        th1 = thread_cpu_by_name()
        cpu_ms = (ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) * 1e3 / steps
        dt = comm.allreduce_max([dt])[0]
        total_ok = comm.allreduce_sum([ok])[0]
        fields = ["slices", "slices_ok", "own_s", "process_cpu_ms_per_step"] + list(stage)
        row = [float(len(mine) * steps), float(ok), t_own, cpu_ms] + [stage[k] for k in stage]
        allrows = comm.allgather_f64(row)
        per_rank = {f: [round(allrows[r * len(fields) + i], 6) for r in range(world)] for i, f in enumerate(fields)}
        per_rank["slices_per_s"] = [round(s / max(t, 1e-12), 1) for s, t in zip(per_rank["slices_ok"], per_rank["own_s"])]
        own = per_rank["own_s"]
        return {
            "value": total_ok / dt,
            "ms_per_step": dt * 1e3 / steps,
            "global_batch": global_items,
            "slices_ok": int(total_ok),
            "per_rank": per_rank,
            "own_time_imbalance": round(max(own) / max(min(own), 1e-12), 4),
            "pipeline_depth": depth,
            "rank0_stage_s": {k: round(v, 4) for k, v in stage.items()},
            "rank0_process_cpu_ms_per_step": round(cpu_ms, 3),
            # rank 0's CPU per step by thread name (nm03-pool: loads + writes, nm03-slot: batch
            # threads; other names are the interpreter's and the HIP runtime's threads)
            "rank0_thread_cpu_ms_per_step": {k: round((th1.get(k, 0.0) - th0.get(k, 0.0)) * 1e3 / steps, 3)
                                             for k in sorted(set(th0) | set(th1))
                                             if th1.get(k, 0.0) - th0.get(k, 0.0) > 0},
            # host CPU of the whole cgroup over the timed region (all ranks of this container)
            "cgroup_cpu_ms_per_step": {k[:-5]: round((cg1[k] - cg0.get(k, 0)) / 1e3 / steps, 3)
                                       for k in ("usage_usec", "throttled_usec") if k in cg1},
        }

    def single_pass(out_root, passes, capped, ranks_like=0):
        """BASELINE config 3 as written, as a latency: ONE cohort sharded over the ranks, one engine
        pass per rank, nothing else in flight; each pass bracketed by barriers, max over ranks.
        `capped`: the shard cut into ⌈shard / streams⌉-slice batches, so its loads, uploads,
        kernels and writes overlap across the slots (a 58-slice shard at 8 ranks is otherwise one
        batch run stage after stage). `ranks_like` > 0 (one rank only): time the shard rank 0 would
        get with that many ranks (465 / 8 = 58 slices) — the 8-GPU strong-scaling latency of one
        GPU's share. Returns (median ms, min ms)."""
        mine, _ = shard("strong", out_root)
        if ranks_like > 0:
            mine = mine[:len(mine) // ranks_like]
        work = n.WorkList(mine)
        cap = (args.single_pass_cap or -(-len(mine) // args.streams)) if capped else 0
        times = []
        for k in range(passes + 1):  # pass 0 warms the output files
            comm.barrier()
            if gpu:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            with _roctx_range("bench.step"):
                codes, msgs, _ = engine.run_list(work, cap)
            dt = time.perf_counter() - t0
            if msgs:
                raise SystemExit(f"rank {rank}: {len(msgs)} slices failed in the single pass")
            dt = comm.allreduce_max([dt])[0]
            if k:
                times.append(dt)
        times.sort()
        return round(times[len(times) // 2] * 1e3, 4), round(times[0] * 1e3, 4)

    primary = measure(args.scaling, args.out_root, args.steps, args.warmup, profile=args.cpu_profile)
    len_mine_primary = [primary["per_rank"]["slices"][rank] / args.steps]
    secondary = None
    other = "strong" if args.scaling == "weak" else "weak"
    if not args.no_secondary and world > 1:
        secondary = measure(other, os.path.join(args.out_root, other), args.steps, 1)
    elif not args.no_secondary:
        secondary = {"value": primary["value"], "ms_per_step": primary["ms_per_step"],
                     "global_batch": primary["global_batch"], "note": "1 rank: weak and strong coincide"}
    wiped = None
    if args.wipe_passes > 0:
        wiped = measure(args.scaling, os.path.join(args.out_root, "wipe"), args.wipe_passes, 1, wipe=True)
    sp = None
    if args.single_passes > 0:
        sp_root = os.path.join(args.out_root, "single")
        med, best = single_pass(sp_root, args.single_passes, capped=True)
        med_u, best_u = single_pass(sp_root, args.single_passes, capped=False)
        sp = {"single_pass_ms": med, "single_pass_min_ms": best, "single_pass_batch_cap": args.single_pass_cap or "ceil(shard/streams)",
              "single_pass_uncapped_ms": med_u, "single_pass_uncapped_min_ms": best_u,
              "single_pass_passes": args.single_passes}
        if world == 1:
            # One GPU's share of the 8-GPU config-3 run (58 of 465 slices), capped vs one batch.
            m8, b8 = single_pass(sp_root, args.single_passes, capped=True, ranks_like=8)
            m8u, b8u = single_pass(sp_root, args.single_passes, capped=False, ranks_like=8)
            sp.update({"single_pass_shard8_ms": m8, "single_pass_shard8_min_ms": b8,
                       "single_pass_shard8_uncapped_ms": m8u, "single_pass_shard8_uncapped_min_ms": b8u})

    cli = None
    if args.cli_runs > 0 and not args.dry_run:
        # After the engine is gone (its pool threads would compete with the CLI's): rank 0 runs the
        # whole CLI --gpus N, reaped with wait4 (exact wall + rusage); the other ranks wait.
        del engine
        engine = None
        if is_root:
            cli = cli_wall(args, world, local_root)
        comm.barrier()

    if is_root:
        value = primary["value"]
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "slices/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(primary["ms_per_step"], 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": (round(value / BASELINE_SLICES_PER_S, 3) if BASELINE_SLICES_PER_S else None),
            "dtype": "fp32",
            "data": "synthetic (20-patient T1+C-shaped DICOM cohort, 256x256 u16, generated on the box)",
            "config": {
                "model": "NM03 T1+C pipeline: norm/clip -> VMF 7x7 -> sharpen 9x9 -> SRG[0.74,0.91] -> "
                         "dilate 3 -> render 512^2 x2 -> JPEG q75",
                "global_batch": primary["global_batch"],
                "seq_len": 256,
                "parallelism": f"dp{world}",
                "batch_size": batch,
                "streams": args.streams,
                "threads": args.threads,
                "create_writers": ecfg.create_writers,
                "stream_steps": bool(args.stream_steps),
                "pipelined_passes": not args.no_pipeline and not args.stream_steps,
                "pipeline_depth": primary["pipeline_depth"],
                "comm": comm_info,
                "rank0_stage_s": primary["rank0_stage_s"],
                "cgroup_cpu_ms_per_step": primary["cgroup_cpu_ms_per_step"],
                "rank0_process_cpu_ms_per_step": primary["rank0_process_cpu_ms_per_step"],
                "rank0_thread_cpu_ms_per_step": primary["rank0_thread_cpu_ms_per_step"],
                "per_rank": primary["per_rank"],
                "own_time_imbalance": primary["own_time_imbalance"],
                "storage": {"data": local_root, "input_copies": len(roots), "out": args.out_root},
            },
        }
        if wiped is not None:
            rec["config"]["wipe_each_pass"] = {"value": round(wiped["value"], 2),
                                               "per_pass": "wipe + mkdir of the output tree, patient discovery, "
                                                           "series listing and ordering, work-list build"
                                                           if (args.scaling == "weak" or world == 1) else "wipe + mkdir",
                                               "ms_per_step": round(wiped["ms_per_step"], 3),
                                               "steps": args.wipe_passes,
                                               "timed_s": round(wiped["ms_per_step"] * args.wipe_passes / 1e3, 4),
                                               "rank0_process_cpu_ms_per_step": wiped["rank0_process_cpu_ms_per_step"],
                                               "cgroup_cpu_ms_per_step": wiped["cgroup_cpu_ms_per_step"],
                                               "wipe_mode": args.wipe_mode,
                                               "reaper_threads": args.reaper_threads,
                                               "rank0_stage_s": wiped["rank0_stage_s"]}
        if secondary is not None:
            rec["config"][other] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in secondary.items()
                                    if k in ("value", "ms_per_step", "global_batch", "per_rank", "note",
                                             "own_time_imbalance", "pipeline_depth")}
        if sp is not None:
            rec["config"].setdefault("strong", {}).update(sp)
        if cli is not None:
            rec["config"]["cli_wall"] = cli
        if args.emulate_shard_of > 1 and world == 1:
            rec["metric"] = (f"EMULATION, not the headline: one GPU processing rank 0's strong-scaling shard of "
                             f"a {args.emulate_shard_of}-rank job per step")
            rec["vs_baseline"] = None
            rec["config"]["emulate_shard_of"] = args.emulate_shard_of
        if args.host_only:
            rec["metric"] = "host path only: DICOM loads + JPEG writes per s (GPU stages replaced by fixed segments)"
            rec["vs_baseline"] = None
            rec["config"]["host_only"] = True
        # Host efficiency: slices per second of this process's CPU time (rank 0).
        cpu = primary["rank0_process_cpu_ms_per_step"]
        rec["config"]["rank0_slices_per_cpu_s"] = round(len_mine_primary[0] / (cpu * 1e-3), 1) if cpu > 0 else None
        # Device identity of every rank (PCI bus id, HIP index, NUMA node, CPU partition, pool size,
        # and the communicator's own view: RCCL's ncclCommCount / ncclCommCuDevice).
        pr = rec["config"]["per_rank"]
        pr["device"] = [d["bus_id"] for d in devices]
        pr["hip_device"] = [d["device"] for d in devices]
        pr["numa_node"] = [d["numa_node"] for d in devices]
        pr["cpus"] = [d["cpus"] for d in devices]
        pr["threads"] = [d["threads"] for d in devices]
        pr["transport_device"] = [d["transport_device"] for d in devices]
        rec["config"]["comm"]["distinct_devices"] = len({d["bus_id"] for d in devices if d["bus_id"]})
        print(json.dumps(rec), flush=True)
    comm.barrier()
    del engine
    if not args.keep_output and is_root:
        shutil.rmtree(args.out_root, ignore_errors=True)
    # tmpfs holds data in RAM: drop a generated dataset unless asked to keep it (local rank 0,
    # after the final barrier every rank has passed).
    if local_rank == 0 and not args.keep_data and args.data_root.startswith("/dev/shm/"):
        for r in roots:
            shutil.rmtree(r, ignore_errors=True)
    return 0


def cli_wall(args, world, data_root):
    """config.cli_wall: `img_processing_parallel --gpus N --quiet --json` on the bench cohort, run
    args.cli_runs times. Every invocation is a cold reference-style run: process start, HIP
    initialisation, cohort discovery, per-patient output wipe (main_parallel.cpp:49-64), every
    slice, exit. Median/min wall and the CLI's own phase split (hip_init_s, engine_ctor_s,
    processing_wall_s)."""
    from nm03_capstone_project_amd.utils.cli_wall import time_cli
    exe = os.path.join(ROOT, "build", "bin", "img_processing_parallel")
    if not os.path.exists(exe):
        return {"skipped": f"{exe} not built"}
    out = os.path.join(args.out_root, "cli")
    js = os.path.join(args.out_root, "cli.json")
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "NM03_COMM_JOB")}
    argv = [exe, "--gpus", str(world), "--data-root", data_root, "--out", out, "--quiet", "--json", js]
    res = time_cli(argv, runs=args.cli_runs, json_path=js, env=env)
    slices = None
    try:
        with open(js) as f:
            slices = json.load(f).get("slices")
    except (OSError, ValueError):
        pass
    res["cmd"] = f"img_processing_parallel --gpus {world} --quiet --json (cohort of {slices} slices)"
    res["slices"] = slices
    if slices and res["wall_median_s"] > 0:
        res["slices_per_s_median"] = round(slices / res["wall_median_s"], 1)
    return res


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        if args.gpus > 1:
            return launch(args, argv)
    elif int(world_env) != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world_env} but --gpus {args.gpus}: launch with matching values")
    return run_rank(args)


if __name__ == "__main__":
    sys.exit(main())
