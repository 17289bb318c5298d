#!/bin/bash
# Interleaved A/B/C of the headline bench: batch 96 × 4 (default) vs 117 × 4 (4 equal batches per
# 465-slice pass) vs 155 × 3 (3 equal batches), 4 rounds (gpurun). gpurun_out/bs_focus4/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/bs_focus4; mkdir -p $O
for i in 1 2 3 4; do
  for cfg in "96 4" "117 4" "155 3"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 --batch-size $1 --streams $2 \
      > $O/b$1_s$2_$i.log 2>&1 || exit 33
    echo "batch $1 streams $2 round $i $(grep -o '"value": [0-9.]*' $O/b$1_s$2_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/b$1_s$2_$i.log | head -1)" >> $O/summary.txt
  done
done
