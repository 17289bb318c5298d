#!/bin/bash
# (gpurun) NM03_PIN=l3 (loads/exports of slice i on L3 domain i mod G, workers pinned per L3 domain)
# vs the default, re-measured with private worker fd tables and the shared upload stream; bench.py
# and --host-only, interleaved. gpurun_out/r3l3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3l3; mkdir -p $O
summ() {
python3 - $1 $2 >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = c['global_batch'] * j['steps']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} "
              f"load_cpu={s['load_cpu_s']/n*1e6:5.1f}us write_cpu={s['write_cpu_s']/n*1e6:5.1f}us/pair")
PY
}
for rep in 1 2 3; do
  for v in set l3; do
    NM03_PIN=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 > $O/gpu_${v}_$rep.log 2>&1 || exit 40
    summ $O/gpu_${v}_$rep.log gpu_$v
    NM03_PIN=$v timeout -k 10 300 python3 bench.py --host-only --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 > $O/host_${v}_$rep.log 2>&1 || exit 41
    summ $O/host_${v}_$rep.log host_$v
  done
done
