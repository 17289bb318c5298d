#!/bin/bash
# (gpurun) host pool size A/B after the polled waits: 16 / 20 / 24 threads, interleaved 3x.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/threads_ab.txt
: > $O
for r in 1 2 3; do
  for t in 16 20 24; do
    echo "threads$t" >> $O
    timeout -k 10 200 python bench.py --keep-data --threads $t 2>/dev/null | grep metric >> $O || exit 31
  done
done
