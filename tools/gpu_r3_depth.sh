#!/bin/bash
# (gpurun) Deep pipelining after the warmup fix (every output tree written before timing): 96 x 6
# and 96 x 4 at depth 4 vs 2, plus GPU tests. gpurun_out/r3dp/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3dp; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 31
run() {
  local name=$1; shift
  timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --wipe-passes 0 --single-passes 0 "$@" > $O/$name.log 2>&1 || return 1
  python3 - $O/$name.log $name >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = c['global_batch'] * j['steps']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} load={s['load_cpu_s']/n*1e6:5.1f}us write={s['write_cpu_s']/n*1e6:5.1f}us depth={c.get('pipeline_depth')}")
PY
}
for rep in 1 2; do
  run s6_d4 --batch-size 96 --streams 6 || exit 40
  run s4_d4 --batch-size 96 --streams 4 --pipeline-depth 4 || exit 41
  run s4_d2 --batch-size 96 --streams 4 || exit 42
done
