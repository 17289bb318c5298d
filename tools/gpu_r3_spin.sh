#!/bin/bash
# (gpurun) Pool spin-before-sleep (NM03_POOL_SPIN_US=50) vs none, interleaved 3 pairs: headline,
# host CPU, single-pass latency. gpurun_out/r3sn/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3sn; mkdir -p $O
for rep in 4 5 6 7; do
  for v in 0 50 200; do
    NM03_POOL_SPIN_US=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 10 > $O/s${v}_$rep.log 2>&1 || exit 40
    python3 - $O/s${v}_$rep.log spin$v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:7s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} sp={st.get('single_pass_ms')} sp8={st.get('single_pass_shard8_ms')}/{st.get('single_pass_shard8_min_ms')}")
PY
  done
done
