#!/bin/bash
# (gpurun) Cold CLI anatomy: whole-process walls of img_processing_parallel by GPU_MAX_HW_QUEUES
# (exact wait4 timing + the CLI's own phase split incl. exec → main), per-batch timelines of fresh
# runs (NM03_BATCH_TRACE=1), and one rocprofv3 trace of a cold run (kernels, copies, HIP API).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-cold}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
D=/dev/shm/cold_data
CLI="$R/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/cold_out --quiet"
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for q in ${QUEUES:-4 2 1}; do
  timeout -k 10 300 python3 - "$q" "$D" "$O" <<'PY' || exit 2
import json, os, sys
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
from nm03_capstone_project_amd.utils.cli_wall import time_cli
q, d, o = sys.argv[1:4]
js = f"/tmp/cold_q{q}.json"
argv = [os.path.join(os.environ["GRAFT_REPO_ROOT"], "build/bin/img_processing_parallel"), "--data-root", d + "/",
        "--out", "/dev/shm/cold_out", "--quiet", "--json", js]
env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
res = time_cli(argv, runs=int(os.environ.get("RUNS", "7")), json_path=js, env=env)
res["GPU_MAX_HW_QUEUES"] = q
with open(os.path.join(o, "cli_wall.jsonl"), "a") as f:
    f.write(json.dumps(res) + "\n")
print(q, res["wall_median_s"], res.get("phases_median_s"))
PY
done
for r in 1 2; do
  (cd /tmp && NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $CLI --json $R/$O/trace_$r.json > $R/$O/trace_$r.log 2>&1) || exit 3
done
cd /tmp || exit 4
NM03_ROCTX=1 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --hip-runtime-trace \
  --output-format csv -d $R/$O/trace -o cli -- $R/build/bin/img_processing_parallel --data-root $D/ \
  --out /dev/shm/cold_out --quiet --json $R/$O/traced.json > $R/$O/traced.log 2>&1 || exit 5
rm -rf $D /dev/shm/cold_out
echo done
