#!/bin/bash
# 12-bit transfer packing on (default) vs off (NM03_PACK12=0) on the pipelined bench, 4 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/pk; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/on_$i.log 2>&1 || exit 41
  NM03_PACK12=0 timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/off_$i.log 2>&1 || exit 42
done
