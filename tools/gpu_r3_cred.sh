#!/bin/bash
# (gpurun; host only) Does a per-thread struct cred close the threads-vs-processes gap of small-file
# I/O? tools/io_contention.cpp at 16 workers: threads with private fd tables (mode 2), + private cred
# (mode 4), processes (mode 1); 3 interleaved rounds. gpurun_out/r3cred/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3cred; mkdir -p $O
R=/dev/shm/nm03_ioc; rm -rf $R; mkdir -p $R
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max >> $O/nproc.txt 2>/dev/null
for round in 1 2 3; do
  for m in 2 4 1; do
    timeout -k 5 120 build/bin/io_contention $R 16 16000 3 $m >> $O/io.txt 2>&1 || { rm -rf $R; exit 10; }
  done
done
rm -rf $R
# Engine A/B: NM03_PRIVATE_CRED=0/1, host-only bench and the full bench, 3 interleaved rounds.
for round in 1 2 3; do
  for c in 0 1; do
    NM03_PRIVATE_CRED=$c timeout -k 10 300 python3 bench.py --host-only --wipe-passes 0 --single-passes 0 > $O/host_c${c}_$round.log 2>&1 || exit 20
    NM03_PRIVATE_CRED=$c timeout -k 10 300 python3 bench.py --wipe-passes 0 --single-passes 10 > $O/gpu_c${c}_$round.log 2>&1 || exit 21
  done
done
