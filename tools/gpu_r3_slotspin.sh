#!/bin/bash
# (gpurun) Idle slot threads spinning for the next run (NM03_SLOT_SPIN_US=500) vs sleeping, 4 pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3ss; mkdir -p $O
for rep in 1 2 3 4; do
  for v in 0 500; do
    NM03_SLOT_SPIN_US=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 10 > $O/s${v}_$rep.log 2>&1 || exit 40
    python3 - $O/s${v}_$rep.log slot$v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:8s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} sp={st.get('single_pass_ms')} sp8={st.get('single_pass_shard8_ms')}/{st.get('single_pass_shard8_min_ms')}")
PY
  done
done
