#!/bin/bash
# Host pool threads at the 96 × 4 default: 12 / 16 / 20, 4 interleaved rounds (gpurun). gpurun_out/thr96/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/thr96; mkdir -p $O
for i in 1 2 3 4; do
  for t in 12 16 20; do
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 --threads $t > $O/t${t}_$i.log 2>&1 || exit 33
    echo "threads $t round $i $(grep -o '"value": [0-9.]*' $O/t${t}_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/t${t}_$i.log | head -1) $(grep -o '"throttled": [0-9.]*' $O/t${t}_$i.log | head -1)" >> $O/summary.txt
  done
done
