#!/bin/bash
# (gpurun) config 4 (512² × 10k, 5×5 median) upload sweep: progressive chunk size and streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c4_sweep.txt
: > $O
B=build/bin
T=/tmp/nm03_c4
$B/nm03_synth --data-root $T/stress/ --stress 10000 --stress-dim 512 --threads 16 > /dev/null || exit 101
for r in 1 2; do
  for v in "0 6" "2048 6" "8192 6" "2048 3" "8192 3" "2048 4"; do
    set -- $v
    echo "chunk$1 streams$2 $(NM03_UPLOAD_CHUNK_KB=$1 timeout -k 10 200 $B/nm03_bench --config cohort --data-root $T/stress/ --out /tmp/c4o --steps 3 --warmup 1 --batch-size 64 --streams $2 --median-window 5 --max-dim 512)" >> $O || exit 102
  done
done
