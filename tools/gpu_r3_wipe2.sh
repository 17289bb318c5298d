#!/bin/bash
# (gpurun) Wipe figure with per-pass rediscovery (3 bench runs), syscall cost on the box. gpurun_out/r3w2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3w2; mkdir -p $O
timeout -k 5 60 build/bin/syscall_probe > $O/syscall_probe.txt 2>&1 || exit 10
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --single-passes 20 > $O/bench_$i.log 2>&1 || exit 40
done
