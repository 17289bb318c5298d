#!/bin/bash
# (gpurun) Batch size x streams re-tune of bench.py with the shared upload stream, 2 interleaved
# rounds. gpurun_out/r3bs/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3bs; mkdir -p $O
for rep in 1 2; do
  for cfg in "96 4" "64 6" "128 3" "96 6" "80 5" "160 3"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 --batch-size $1 --streams $2 > $O/b$1_s$2_$rep.log 2>&1 || exit 40
    python3 - $O/b$1_s$2_$rep.log "b$1 s$2" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']
        print(f"{sys.argv[2]:9s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} kern_s={s['kernels_s']} h2d_s={s['h2d_s']}")
PY
  done
done
