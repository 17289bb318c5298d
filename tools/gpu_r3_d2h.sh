#!/bin/bash
# (gpurun) JPEG output path A/B in the bench (4 streams, batch 96), interleaved: encoder stores into
# host-mapped memory (default, NM03_JPEG_D2H=0) vs encoder into HBM + gather kernel storing into
# host-mapped memory (=2). Kernel stats of one profiled run each. gpurun_out/r3d/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "jpeg_d2h or jpeg_kernel or cohort_configs" > $O/pytest.log 2>&1 || exit 31
for rep in 1 2 3; do
  for m in 0 2; do
    NM03_JPEG_D2H=$m timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 5 > $O/m${m}_$rep.log 2>&1 || exit 40
    python3 - $O/m${m}_$rep.log m$m >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']; s = c['rank0_stage_s']
        print(f"{sys.argv[2]} value={j['value']:9.0f} cpu={c['rank0_process_cpu_ms_per_step']:6.2f} kern_s={s['kernels_s']} h2d_s={s['h2d_s']} sp8={st['single_pass_shard8_ms']}")
PY
  done
done
for m in 0 2; do
  NM03_JPEG_D2H=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$m -o b -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 0 > $O/prof$m.log 2>&1 || exit 50
  python3 tools/kstats.py $O/prof$m/b_kernel_stats.csv > $O/kernels_m$m.txt || exit 51
done
