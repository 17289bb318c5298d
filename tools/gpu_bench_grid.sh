#!/bin/bash
# bench.py over batch-size × streams configurations, interleaved repeats (gpurun). gpurun_out/grid/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/grid
CONFIGS=${CONFIGS:-"64:6 48:6 96:6 128:6 64:5 64:7 96:5"}
for i in 1 2 3; do
  for c in $CONFIGS; do
    b=${c%%:*}; s=${c##*:}
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --batch-size $b --streams $s --keep-data \
      > gpurun_out/grid/b${b}_s${s}_$i.log 2>&1 || exit 7
  done
done
rm -rf /dev/shm/nm03_bench_data*
