#!/bin/bash
# Loader read-path A/B under pipelined passes (host CPU is the bound): staged + 12-bit packing
# (default) vs direct pread into the pinned blob (16-bit upload, no pack/copy passes). Interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/load_ab
for i in 1 2 3; do
  for mode in staged direct; do
    NM03_LOAD_MODE=$mode timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary \
      > gpurun_out/load_ab/${mode}_$i.log 2>&1 || exit 40
  done
done
