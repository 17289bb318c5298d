#!/bin/bash
# Host-thread sweep (gpurun): bench.py at 4/8/12/16 pool threads, with per-slice loader/writer CPU
# time from the engine (thread CPU clocks) and the cgroup's CPU usage. JSON in gpurun_out/thread_sweep.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/thread_sweep.txt
: > $O
for t in 4 8 12 16; do
  echo "threads $t" >> $O
  timeout -k 10 200 python bench.py --threads $t --keep-data 2>/dev/null | grep metric >> $O || exit 31
done
echo "threads 16 numa0" >> $O
NM03_NUMA=0 timeout -k 10 200 python bench.py --threads 16 2>/dev/null | grep metric >> $O || exit 32
