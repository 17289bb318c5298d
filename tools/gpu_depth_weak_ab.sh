#!/bin/bash
# Weak headline (1 rank) with 2 (auto) vs 3 passes in flight, 5 interleaved pairs (gpurun). gpurun_out/depthw/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/depthw; mkdir -p $O
for i in 1 2 3 4 5; do
  for dp in 0 3; do
    NM03_BENCH_DEPTH=$dp timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 > $O/d${dp}_$i.log 2>&1 || exit 33
    echo "depth=$dp round $i $(grep -o '"value": [0-9.]*' $O/d${dp}_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/d${dp}_$i.log | head -1)" >> $O/summary.txt
  done
done
