#!/bin/bash
# bench.py pipeline depth A/B for the strong-scaling figure (gpurun): passes in flight 2 vs auto (4
# when a rank's shard is below one batch per slot), 2 and 8 ranks sharing GPU 0, 3 rounds.
# gpurun_out/depth/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/depth; mkdir -p $O
export NM03_DEVICE_OVERRIDE=0
for i in 1 2 3; do
  for g in 2 8; do
    for dp in 2 0; do
      NM03_BENCH_DEPTH=$dp timeout -k 10 400 python bench.py --gpus $g --steps 50 --warmup 3 --wipe-passes 0 > $O/g${g}_d${dp}_$i.log 2>&1 || exit 33
      echo "gpus $g depth=$dp round $i weak $(grep -o '"value": [0-9.]*' $O/g${g}_d${dp}_$i.log | head -1) strong $(grep -o '"strong": {"value": [0-9.]*' $O/g${g}_d${dp}_$i.log)" >> $O/summary.txt
    done
  done
done
