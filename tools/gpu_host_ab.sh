#!/bin/bash
# Host-path A/B on one GPU (pipelined passes; host CPU is the bound), interleaved: pack straight
# into pinned memory through an L1 bounce buffer (default) vs full-size intermediate + copy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/host_ab
for i in 1 2 3 4; do
  for b in 1 0; do
    NM03_PACK_BOUNCE=$b timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary \
      > gpurun_out/host_ab/bounce${b}_$i.log 2>&1 || exit 40
  done
done
