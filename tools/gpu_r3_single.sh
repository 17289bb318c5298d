#!/bin/bash
# (gpurun) Single-pass latency A/B (bench.py config.strong.single_pass*): per-slice wait estimate
# (default) vs per-batch EMA (NM03_EVENT_EMA=batch) vs plain 20 µs polling (NM03_EVENT_ADAPT=0),
# interleaved. gpurun_out/r3s/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3s; mkdir -p $O
for rep in 1 2 3; do
  for v in slice batch poll; do
    case $v in
      slice) E="";; batch) E="NM03_EVENT_EMA=batch";; poll) E="NM03_EVENT_ADAPT=0";;
    esac
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 20 > $O/${v}_$rep.log 2>&1 || exit 40
    python3 - $O/${v}_$rep.log $v >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']; st = c['strong']
        print(f"{sys.argv[2]:6s} value={j['value']:9.0f} cpu={c['rank0_process_cpu_ms_per_step']:6.2f} "
              f"sp={st['single_pass_ms']:.3f}/{st['single_pass_uncapped_ms']:.3f} "
              f"sp8={st['single_pass_shard8_ms']:.3f}(min {st['single_pass_shard8_min_ms']:.3f})/{st['single_pass_shard8_uncapped_ms']:.3f}")
PY
  done
done
