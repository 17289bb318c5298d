#!/bin/bash
# Bench A/B on one box, interleaved: current tree vs abprev/ (a worktree of an earlier commit,
# built in place; take abprev/ out of .gpurunignore for the call). Logs in gpurun_out/ab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
uname -r > gpurun_out/ab/uname.txt
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > gpurun_out/ab/cur_$i.log 2>&1 || exit 41
  (cd abprev && timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > ../gpurun_out/ab/prev_$i.log 2>&1) || exit 43
done
