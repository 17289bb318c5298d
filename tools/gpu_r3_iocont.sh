#!/bin/bash
# (gpurun; host only, no GPU use) Per-op CPU of engine-style loads and JPEG rewrites on tmpfs:
# 16 threads with private fd tables, + private fs_struct, 16 processes. Interleaved, 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3io; mkdir -p $O
for r in 1 2; do
  for P in 2 3 1; do
    R=/dev/shm/r3io_${P}; rm -rf $R; mkdir -p $R
    timeout -k 10 120 build/bin/io_contention $R 16 4000 3 $P >> $O/io_fs.txt 2>&1 || exit 10
    rm -rf $R
  done
done
