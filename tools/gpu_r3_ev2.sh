#!/bin/bash
# (gpurun) Batch-completion event: default (polled, no blocking-sync) vs blocking-sync event
# (NM03_EV2_BLOCKING=1, the previous default), interleaved 3 pairs; thread CPU by name. gpurun_out/r3ev/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3ev; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "engine" > $O/pytest.log 2>&1 || exit 31
for rep in 1 2 3; do
  for v in 0 1; do
    NM03_EV2_BLOCKING=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 3 > $O/e${v}_$rep.log 2>&1 || exit 40
    python3 - $O/e${v}_$rep.log blocking$v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']
        print(f"{sys.argv[2]} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} threads={c['rank0_thread_cpu_ms_per_step']} sp8={c['strong'].get('single_pass_shard8_ms')}")
PY
  done
done
