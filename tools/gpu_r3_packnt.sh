#!/bin/bash
# (gpurun) 12-bit pack output through streaming stores (default) vs regular cached stores
# (NM03_PACK_NT=0): 4 interleaved bench pairs at 50 steps + the host-only figure, CPU per step.
# gpurun_out/r3nt/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3nt; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "engine" > $O/pytest.log 2>&1 || exit 31
for rep in 1 2 3 4; do
  for nt in 1 0; do
    NM03_PACK_NT=$nt timeout -k 10 300 python3 bench.py --steps 50 --wipe-passes 0 --single-passes 0 > $O/nt${nt}_$rep.log 2>&1 || exit 40
    python3 - $O/nt${nt}_$rep.log "nt$nt rep$rep" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = j['steps']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} load_cpu/step={s['load_cpu_s']*1e3/n:6.2f} h2d/step={s['h2d_s']*1e3/n:5.2f}")
PY
  done
done
