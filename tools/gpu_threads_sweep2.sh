#!/bin/bash
# Host pool size sweep on the pipelined bench (gpurun): --threads 10/12/14/16, interleaved, twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/thr2; mkdir -p $O
for i in 1 2; do
  for t in 16 12 14 10; do
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --threads $t > $O/t${t}_$i.log 2>&1 || exit 41
  done
done
