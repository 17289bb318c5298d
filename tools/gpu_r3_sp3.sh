#!/bin/bash
# (gpurun) Small-batch completion spin-poll (default) vs the EMA sleep (NM03_SMALL_POLL=0), with the
# inline small uploads; 200 single passes per figure, 3 interleaved rounds. gpurun_out/r3sp3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3sp3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "engine" > $O/pytest.log 2>&1 || exit 31
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --wipe-passes 0 --single-passes 200 > $O/$n.log 2>&1 || exit 40
  python3 - $O/$n.log $n >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:10s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} sp={st.get('single_pass_ms')}/{st.get('single_pass_min_ms')} sp8={st.get('single_pass_shard8_ms')}/{st.get('single_pass_shard8_min_ms')} sp8u={st.get('single_pass_shard8_uncapped_ms')}")
PY
}
for rep in 1 2 3; do
  run poll_$rep NM03_SMALL_POLL=1
  run ema_$rep NM03_SMALL_POLL=0
done
