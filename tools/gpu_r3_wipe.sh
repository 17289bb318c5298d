#!/bin/bash
# (gpurun) Cold (wipe-each-pass) figure with CPU breakdown: bench.py and --host-only. gpurun_out/r3w/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3w; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --wipe-passes 20 --single-passes 0 > $O/gpu_$rep.log 2>&1 || exit 40
  timeout -k 10 300 python3 bench.py --host-only --steps 20 --warmup 3 --wipe-passes 20 --single-passes 0 > $O/host_$rep.log 2>&1 || exit 41
done
for f in $O/*.log; do
python3 - $f >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; w = c['wipe_each_pass']; n = c['global_batch'] * w['steps']; n0 = c['global_batch'] * j['steps']
        s, s0 = w['rank0_stage_s'], c['rank0_stage_s']
        print(f"{sys.argv[1].split('/')[-1]:12s} warm={j['value']:8.0f} cpu={c['rank0_process_cpu_ms_per_step']:5.1f} load={s0['load_cpu_s']/n0*1e6:5.1f} write={s0['write_cpu_s']/n0*1e6:5.1f} | "
              f"wipe={w['value']:8.0f} cpu={w['rank0_process_cpu_ms_per_step']:5.1f} load={s['load_cpu_s']/n*1e6:5.1f} write={s['write_cpu_s']/n*1e6:5.1f} write_wall={s['write_s']/n*1e6:5.1f}")
PY
done
