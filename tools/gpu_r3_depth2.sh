#!/bin/bash
# (gpurun; host-only engine, no GPU use) Deep pipelining diagnosis: per-run latency and stage times
# at depth 2 / 4 with private worker fd tables (default), shared tables, and private tables without
# worker directory fds. gpurun_out/r3dq/. (Historical: NM03_WORKER_DIRFDS selected the per-worker
# directory-fd cache this probe measured; the cache was removed, workers with private tables use full paths.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3dq; mkdir -p $O
export DP_ROOT=/dev/shm/r3dq_data/ DP_THREADS=16
for v in "1 1" "0 1" "1 0"; do
  set -- $v
  for d in 2 4; do
    rm -rf /dev/shm/r3dq_out; export DP_OUT=/dev/shm/r3dq_out
    echo "private=$1 worker_dirfds=$2" >> $O/probe.txt
    NM03_PRIVATE_FDS=$1 NM03_WORKER_DIRFDS=$2 timeout -k 10 120 python3 tools/depth_probe.py $d 24 >> $O/probe.txt 2>&1 || exit 10
  done
done
rm -rf /dev/shm/r3dq_out /dev/shm/r3dq_data
