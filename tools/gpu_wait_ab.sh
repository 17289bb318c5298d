#!/bin/bash
# A/B (gpurun): slot-thread batch wait — blocking-sync hipEventSynchronize vs event polling with
# 20 / 50 µs sleeps (NM03_EVENT_WAIT, NM03_EVENT_POLL_US), interleaved 3x.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/wait_ab.txt
: > $O
for r in 1 2 3; do
  for v in "block 20" "poll 20" "poll 50"; do
    set -- $v
    echo "$1 $2" >> $O
    NM03_EVENT_WAIT=$1 NM03_EVENT_POLL_US=$2 timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
