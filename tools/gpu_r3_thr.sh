#!/bin/bash
# (gpurun) Pool threads 16 (default) vs 14 vs 12 with private fd tables + shared upload stream,
# interleaved 3 rounds. gpurun_out/r3th/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3th; mkdir -p $O
for rep in 1 2 3; do
  for t in 16 14 12; do
    timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 --threads $t > $O/t${t}_$rep.log 2>&1 || exit 40
    python3 - $O/t${t}_$rep.log t$t >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = c['global_batch'] * j['steps']
        print(f"{sys.argv[2]} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} load={s['load_cpu_s']/n*1e6:5.1f} write={s['write_cpu_s']/n*1e6:5.1f}")
PY
  done
done
