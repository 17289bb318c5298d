#!/bin/bash
# (gpurun; host only) Where the loader's 4x gap comes from (engine 23.7 us per load vs 3.2 us for a
# hot 131 KB pread): io_contention mode 4 at 1 / 4 / 16 workers, with 200 files (26 MB, L3-resident)
# and 8000 files (1 GB, DRAM and cold page-cache metadata). gpurun_out/r3lg/.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3lg; mkdir -p $O
R=/dev/shm/nm03_lg
for round in 1 2; do
  for nf in 200 8000; do
    for T in 1 4 16; do
      rm -rf $R; mkdir -p $R
      echo "== files $nf workers $T" >> $O/io.txt
      timeout -k 5 120 build/bin/io_contention $R $T $nf 4 4 >> $O/io.txt 2>&1 || { rm -rf $R; exit 10; }
    done
  done
done
rm -rf $R
