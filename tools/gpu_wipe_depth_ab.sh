#!/bin/bash
# Wipe-each-pass figure with 2 (auto) vs 3 passes in flight (gpurun): with 3, the wipe of pass k's
# tree runs while two passes are queued instead of one. 4 interleaved pairs. gpurun_out/wdepth/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/wdepth; mkdir -p $O
for i in 1 2 3 4; do
  for dp in 0 3; do
    NM03_BENCH_DEPTH=$dp timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary --wipe-passes 50 > $O/d${dp}_$i.log 2>&1 || exit 33
    echo "depth=$dp round $i $(grep -o '"value": [0-9.]*' $O/d${dp}_$i.log | head -1) wipe $(grep -o '"wipe_each_pass": {"value": [0-9.]*' $O/d${dp}_$i.log)" >> $O/summary.txt
  done
done
