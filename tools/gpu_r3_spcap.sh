#!/bin/bash
# (gpurun) Single-pass batch-cap sweep (bench.py --single-pass-cap; shard8 = 58 slices), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3sp; mkdir -p $O
for rep in 1 2; do
  for c in 0 8 10 20 30; do
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --wipe-passes 0 --single-passes 20 --single-pass-cap $c > $O/c${c}_$rep.log 2>&1 || exit 40
    python3 - $O/c${c}_$rep.log cap$c >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); st = j['config']['strong']
        print(f"{sys.argv[2]:6s} sp={st['single_pass_ms']}/{st['single_pass_min_ms']} sp8={st['single_pass_shard8_ms']}/{st['single_pass_shard8_min_ms']} uncapped8={st['single_pass_shard8_uncapped_ms']}")
PY
  done
done
