#!/bin/bash
# Headline bench over batch size × slot count on the current tree, 2 interleaved rounds (gpurun).
# gpurun_out/bs_sweep/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/bs_sweep; mkdir -p $O
for i in 1 2; do
  for b in 48 64 96 128; do
    for s in 4 6; do
      timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 --batch-size $b --streams $s \
        > $O/b${b}_s${s}_$i.log 2>&1 || exit 33
      echo "batch $b streams $s round $i $(grep -o '"value": [0-9.]*' $O/b${b}_s${s}_$i.log | head -1)" >> $O/summary.txt
    done
  done
done
