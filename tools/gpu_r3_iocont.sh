#!/bin/bash
# (gpurun; host only, no GPU use) Per-op CPU of the engine-style file loads and JPEG rewrites on
# tmpfs with T threads of one process vs T processes (shared fd table / mm vs none).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3io; mkdir -p $O
for T in 8 16; do
  for P in 0 1 2; do
    R=/dev/shm/r3io_$T_$P; rm -rf $R; mkdir -p $R
    timeout -k 10 120 build/bin/io_contention $R $T 4000 3 $P >> $O/io.txt 2>&1 || exit 10
    rm -rf $R
  done
done
nproc >> $O/io.txt; cat /sys/fs/cgroup/cpu.max >> $O/io.txt 2>/dev/null; true
