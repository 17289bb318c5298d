#!/bin/bash
# Interleaved A/B of the headline bench: batch 64 × 6 slots vs 96 × 4, 6 rounds (gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/bs_focus3; mkdir -p $O
for i in 1 2 3 4 5 6; do
  for cfg in "64 6" "96 4"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 --batch-size $1 --streams $2 \
      > $O/b$1_s$2_$i.log 2>&1 || exit 33
    echo "batch $1 streams $2 round $i $(grep -o '"value": [0-9.]*' $O/b$1_s$2_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/b$1_s$2_$i.log | head -1)" >> $O/summary.txt
  done
done
