#!/bin/bash
# (gpurun) JPEG encoder at 5 workgroups per CU (NM03_JPEG_OCC=5) vs 4, in the bench (4 streams,
# batch 96): kernel stats of one profiled run each + 3 interleaved headline pairs. gpurun_out/r3oc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3oc; mkdir -p $O
for occ in 4 5; do
  NM03_JPEG_OCC=$occ timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$occ -o b -- python3 bench.py --steps 30 --warmup 2 --wipe-passes 0 --single-passes 0 > $O/prof$occ.log 2>&1 || exit 50
  python3 tools/kstats.py $O/prof$occ/b_kernel_stats.csv > $O/kernels_occ$occ.txt || exit 51
done
for rep in 1 2 3; do
  for occ in 4 5; do
    NM03_JPEG_OCC=$occ timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 > $O/b${occ}_$rep.log 2>&1 || exit 40
    python3 - $O/b${occ}_$rep.log occ$occ >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']
        print(f"{sys.argv[2]} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} kern_s={s['kernels_s']}")
PY
  done
done
