#!/bin/bash
# (gpurun) Pool-thread CPU outside loads/writes vs the pool's idle spin (NM03_POOL_SPIN_US 200 / 0),
# 3 interleaved pairs at 50 steps. gpurun_out/r3spin/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3spin; mkdir -p $O
for rep in 1 2 3; do
  for us in 200 0; do
    NM03_POOL_SPIN_US=$us timeout -k 10 300 python3 bench.py --steps 50 --wipe-passes 0 --single-passes 0 > $O/s${us}_$rep.log 2>&1 || exit 40
    python3 - $O/s${us}_$rep.log "spin$us rep$rep" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = j['steps']
        th = c['rank0_thread_cpu_ms_per_step']
        io = (s['load_cpu_s'] + s['write_cpu_s']) * 1e3 / n
        print(f"{sys.argv[2]:14s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} pool={th.get('nm03-pool')} io={io:5.2f} pool-io={th.get('nm03-pool', 0) - io:5.2f} slot={th.get('nm03-slot')} py={th.get('python3')}")
PY
  done
done
