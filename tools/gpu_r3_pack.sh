#!/bin/bash
# (gpurun) 12-bit packing on (default) vs off (NM03_PACK12=0) with the shared upload stream and
# private worker fd tables, interleaved 3 pairs. gpurun_out/r3pk/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3pk; mkdir -p $O
for rep in 1 2 3; do
  for v in 1 0; do
    NM03_PACK12=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 > $O/p${v}_$rep.log 2>&1 || exit 40
    python3 - $O/p${v}_$rep.log pack$v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = c['global_batch'] * j['steps']
        print(f"{sys.argv[2]} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} load={s['load_cpu_s']/n*1e6:5.1f}us write={s['write_cpu_s']/n*1e6:5.1f}us h2d_s={s['h2d_s']} kern_s={s['kernels_s']}")
PY
  done
done
