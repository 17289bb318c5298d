#!/bin/bash
# (gpurun) Shared upload stream A/B (NM03_UPLOAD_STREAM=shared vs per-slot streams): engine GPU tests
# with it on, then bench.py interleaved 4 pairs. gpurun_out/r3us/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3us; mkdir -p $O
NM03_UPLOAD_STREAM=shared timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "engine or cli_sequential_equals or cli_parallel_multirank" > $O/pytest.log 2>&1 || exit 31
for rep in 1 2 3 4; do
  for v in shared own; do
    NM03_UPLOAD_STREAM=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 3 > $O/${v}_$rep.log 2>&1 || exit 40
    python3 - $O/${v}_$rep.log $v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']
        print(f"{sys.argv[2]:7s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} h2d_s={s['h2d_s']} kern_s={s['kernels_s']} sp8={c['strong'].get('single_pass_shard8_ms')}")
PY
  done
done
