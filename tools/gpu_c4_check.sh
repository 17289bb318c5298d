#!/bin/bash
# (gpurun) GPU tests + config 4 with the adaptive upload chunk (streams 3 and 6), 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 30
O=gpurun_out/c4_check.txt
: > $O
B=build/bin
T=/tmp/nm03_c4
$B/nm03_synth --data-root $T/stress/ --stress 10000 --stress-dim 512 --threads 16 > /dev/null || exit 101
for r in 1 2; do
  for st in 3 6; do
    echo "streams$st $(timeout -k 10 200 $B/nm03_bench --config cohort --data-root $T/stress/ --out /tmp/c4o --steps 3 --warmup 1 --batch-size 64 --streams $st --median-window 5 --max-dim 512)" >> $O || exit 102
  done
done
