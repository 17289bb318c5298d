#!/bin/bash
# (gpurun) Single-pass latency A/B: NM03_POOL_PREWAKE (pool woken at submit; measured, not adopted, code removed) and
# NM03_SMALL_UPLOAD=inline (small batches copy on their own stream, no upload-stream events),
# 3 interleaved rounds of 4 variants. gpurun_out/r3sp2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3sp2; mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "engine" > $O/pytest.log 2>&1 || exit 31
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --wipe-passes 0 --single-passes ${SP_PASSES:-20} > $O/$n.log 2>&1 || exit 40
  python3 - $O/$n.log $n >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} sp={st.get('single_pass_ms')} sp8={st.get('single_pass_shard8_ms')}/{st.get('single_pass_shard8_min_ms')}")
PY
}
for rep in 1 2 3; do
  run base_$rep NM03_POOL_PREWAKE=0
  run wake_$rep NM03_POOL_PREWAKE=1
  run inl_$rep NM03_SMALL_UPLOAD=inline
  run both_$rep NM03_POOL_PREWAKE=1 NM03_SMALL_UPLOAD=inline
done
