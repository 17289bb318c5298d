#!/bin/bash
# (gpurun) Cold CLI anatomy: whole-process walls of img_processing_parallel by GPU_MAX_HW_QUEUES
# (exact wait4 timing + the CLI's own phase split incl. exec → main), per-batch timelines of fresh
# runs (NM03_BATCH_TRACE=1), and one rocprofv3 trace of a cold run (kernels, copies, HIP and HSA API:
# what the runtime calls inside hipInit and the first stream creations).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-cold}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
D=/dev/shm/cold_data
CLI="$R/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/cold_out --quiet"
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
# Interleaved: run r of every GPU_MAX_HW_QUEUES value before run r + 1 (box drift hits all alike).
timeout -k 10 600 python3 - "$D" "$O" <<'PY' || exit 2
import json, os, sys, time
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from nm03_capstone_project_amd.utils.cli_wall import time_cli
d, o = sys.argv[1:3]
# VARIANTS: ";"-separated, each "-" or "NAME=VAL,NAME=VAL" (environment) with an optional
# "ARGS=..." (CLI flags) and "SLEEP=s" (pause before the run: time since the previous GPU process
# exited); QUEUES (legacy): one variant per --hw-queues value.
if os.environ.get("VARIANTS"):
    queues = os.environ["VARIANTS"].split(";")
else:
    queues = [f"ARGS=--hw-queues {q}" for q in os.environ.get("QUEUES", "4 2 1").split()]
rows = {q: [] for q in queues}
for r in range(int(os.environ.get("RUNS", "7"))):
    for k, q in enumerate(queues):
        js = f"/tmp/cold_v{k}.json"
        env, extra = dict(os.environ), []
        for kv in ([] if q == "-" else q.split(",")):
            name, val = kv.split("=", 1)
            if name == "ARGS":
                extra += val.split()
            elif name == "SLEEP":
                time.sleep(float(val))
            else:
                env[name] = val
        argv = [os.path.join(os.environ["GRAFT_REPO_ROOT"], "build/bin/img_processing_parallel"), "--data-root",
                d + "/", "--out", "/dev/shm/cold_out", "--quiet", "--json", js] + extra
        res = time_cli(argv, runs=1, json_path=js, env=env)
        rows[q].append(res)
        with open(os.path.join(o, "cli_runs.jsonl"), "a") as f:
            f.write(json.dumps({"variant": q, "run": r, **res}) + "\n")
for q in queues:
    walls = sorted(x["wall_median_s"] for x in rows[q])
    ph = {}
    for x in rows[q]:
        for k, v in (x.get("phases_median_s") or {}).items():
            ph.setdefault(k, []).append(v)
    med = {k: round(sorted(v)[len(v) // 2], 4) for k, v in ph.items()}
    line = {"variant": q, "wall_median_s": walls[len(walls) // 2], "walls_s": [x["wall_median_s"] for x in rows[q]],
            "phases_median_s": med}
    with open(os.path.join(o, "cli_wall.jsonl"), "a") as f:
        f.write(json.dumps(line) + "\n")
    print(json.dumps(line))
PY
for r in 1 2; do
  (cd /tmp && NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $CLI --json $R/$O/trace_$r.json > $R/$O/trace_$r.log 2>&1) || exit 3
done
cd /tmp || exit 4
NM03_ROCTX=1 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --hip-runtime-trace --hsa-trace \
  --output-format csv -d $R/$O/trace -o cli -- $R/build/bin/img_processing_parallel --data-root $D/ \
  --out /dev/shm/cold_out --quiet --json $R/$O/traced.json > $R/$O/traced.log 2>&1 || exit 5
rm -rf $D /dev/shm/cold_out
echo done
