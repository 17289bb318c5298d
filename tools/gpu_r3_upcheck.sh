#!/bin/bash
# (gpurun) Shared vs own upload streams on the configurations that collapsed in the batch sweep
# (96 x 6 slots, 160 x 3) and on configs 2 and 4 (native nm03_bench). gpurun_out/r3uc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3uc; mkdir -p $O
T=/tmp/r3uc
build/bin/nm03_synth --data-root $T/patient/ --patients 1 --threads 16 > /dev/null || exit 41
build/bin/nm03_synth --data-root $T/stress/ --stress 2000 --stress-dim 512 --threads 16 > /dev/null || exit 42
for v in shared own; do
  for cfg in "96 6" "160 3"; do
    set -- $cfg
    NM03_UPLOAD_STREAM=$v timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --wipe-passes 0 --single-passes 0 --batch-size $1 --streams $2 > $O/${v}_b$1_s$2.log 2>&1 || exit 40
    python3 - $O/${v}_b$1_s$2.log "$v b$1 s$2" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']
        print(f"{sys.argv[2]:16s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} kern_s={s['kernels_s']} h2d_s={s['h2d_s']}")
PY
  done
  NM03_UPLOAD_STREAM=$v timeout -k 10 120 build/bin/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/r3uc_o2 --steps 50 --warmup 5 --batch-size 25 --streams 3 > $O/c2_$v.json 2>&1 || exit 43
  echo "$v c2 $(tail -1 $O/c2_$v.json)" >> $O/summary.txt
  NM03_UPLOAD_STREAM=$v timeout -k 10 300 build/bin/nm03_bench --config cohort --data-root $T/stress/ --out /tmp/r3uc_o4 --steps 3 --warmup 1 --batch-size 64 --streams 3 --median-window 5 --max-dim 512 > $O/c4_$v.json 2>&1 || exit 44
  echo "$v c4 $(tail -1 $O/c4_$v.json)" >> $O/summary.txt
done
rm -rf $T /tmp/r3uc_o2 /tmp/r3uc_o4
