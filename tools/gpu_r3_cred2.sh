#!/bin/bash
# (gpurun) NM03_PRIVATE_CRED=0/1: 5 interleaved pairs of the full bench + 2 host-only pairs. gpurun_out/r3cred2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3cred2; mkdir -p $O
for round in 1 2 3 4 5; do
  for c in 1 0; do
    NM03_PRIVATE_CRED=$c timeout -k 10 300 python3 bench.py --steps 40 --wipe-passes 0 --single-passes 0 > $O/gpu_c${c}_$round.log 2>&1 || exit 21
  done
done
for round in 1 2; do
  for c in 1 0; do
    NM03_PRIVATE_CRED=$c timeout -k 10 300 python3 bench.py --host-only --steps 40 --wipe-passes 0 --single-passes 0 > $O/host_c${c}_$round.log 2>&1 || exit 20
  done
done
