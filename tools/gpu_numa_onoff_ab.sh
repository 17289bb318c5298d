#!/bin/bash
# NUMA placement of host threads on vs off (NM03_NUMA=0) on the pipelined bench, 4 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/nu; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/on_$i.log 2>&1 || exit 41
  NM03_NUMA=0 timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/off_$i.log 2>&1 || exit 42
done
