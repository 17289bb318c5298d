#!/bin/bash
# Progressive-upload chunk at the 96 × 4 default: 2 MiB vs 1 MiB, 6 interleaved rounds (confirmation)
# (gpurun). gpurun_out/chunk2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/chunk2; mkdir -p $O
for i in 1 2 3 4 5 6; do
  for kb in 2048 1024; do
    NM03_UPLOAD_CHUNK_KB=$kb timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 > $O/c${kb}_$i.log 2>&1 || exit 33
    echo "chunk_kb $kb round $i $(grep -o '"value": [0-9.]*' $O/c${kb}_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/c${kb}_$i.log | head -1)" >> $O/summary.txt
  done
done
