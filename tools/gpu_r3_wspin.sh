#!/bin/bash
# (gpurun) Slot-thread waits: default (spin 200 us for batches of <= 16 slices) vs no spin
# (NM03_WAIT_SPIN_US=0), interleaved 4 pairs. gpurun_out/r3ws/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3ws; mkdir -p $O
for rep in 1 2 3 4; do
  for v in def 0; do
    E="NM03_X=1"; [ "$v" = "0" ] && E="NM03_WAIT_SPIN_US=0"; env $E timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 10 > $O/w${v}_$rep.log 2>&1 || exit 40
    python3 - $O/w${v}_$rep.log wspin$v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:9s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} sp8={st.get('single_pass_shard8_ms')}/{st.get('single_pass_shard8_min_ms')}")
PY
  done
done
