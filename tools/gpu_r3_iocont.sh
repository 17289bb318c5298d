#!/bin/bash
# (gpurun; host only, no GPU use) Per-op CPU of engine-style loads (pread, or mmap+touch+munmap) and
# JPEG rewrites on tmpfs: 16 threads of one process (shared / unshared fd tables) vs 16 processes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3io; mkdir -p $O
for mm in 0 1; do
  for P in 2 1 0; do
    R=/dev/shm/r3io_${P}_$mm; rm -rf $R; mkdir -p $R
    timeout -k 10 120 build/bin/io_contention $R 16 4000 3 $P $mm >> $O/io_mmap.txt 2>&1 || exit 10
    rm -rf $R
  done
done
