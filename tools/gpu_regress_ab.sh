#!/bin/bash
# Bench A/B on one box, interleaved: current tree (adaptive completion wait on/off) vs abprev/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/reg
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary > gpurun_out/reg/cur_$i.log 2>&1 || exit 41
  NM03_EVENT_ADAPT=0 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary > gpurun_out/reg/noadapt_$i.log 2>&1 || exit 42
  (cd abprev && timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary > ../gpurun_out/reg/prev_$i.log 2>&1) || exit 43
done
