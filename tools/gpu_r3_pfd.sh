#!/bin/bash
# (gpurun) Private per-worker fd tables A/B (NM03_PRIVATE_FDS=1 default vs 0): GPU tests first, then
# bench.py and bench.py --host-only interleaved, 3 pairs each. gpurun_out/r3p/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 31
summ() {
python3 - $1 $2 >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; s = c['rank0_stage_s']; n = c['global_batch'] * j['steps']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} "
              f"load_cpu={s['load_cpu_s']/n*1e6:5.1f}us write_cpu={s['write_cpu_s']/n*1e6:5.1f}us/pair "
              f"sp8={c['strong'].get('single_pass_shard8_ms')}")
PY
}
for rep in 1 2 3; do
  for v in 1 0; do
    NM03_PRIVATE_FDS=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 3 --wipe-passes 0 --single-passes 5 > $O/gpu_p${v}_$rep.log 2>&1 || exit 40
    summ $O/gpu_p${v}_$rep.log gpu_p$v
  done
done
for rep in 1 2; do
  for v in 1 0; do
    NM03_PRIVATE_FDS=$v timeout -k 10 300 python3 bench.py --host-only --steps 50 --warmup 3 --wipe-passes 0 --single-passes 0 > $O/host_p${v}_$rep.log 2>&1 || exit 41
    summ $O/host_p${v}_$rep.log host_p$v
  done
done
