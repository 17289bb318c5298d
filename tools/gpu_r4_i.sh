#!/bin/bash
# (gpurun) Round 4: what the cold CLI's hipInit is made of. gpurun_out/r4i/hip_init.txt:
# hip_init_probe plain vs linked against librccl (the CLIs link it: its fat binary is registered at
# load), and with HIP_ENABLE_DEFERRED_LOADING=0; 5 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4i; mkdir -p $O
B=build/bin
for r in 1 2 3 4 5; do
  echo "plain:" >> $O/hip_init.txt; timeout -k 5 60 $B/hip_init_probe >> $O/hip_init.txt 2>&1 || exit 10
  echo "rccl:" >> $O/hip_init.txt; timeout -k 5 60 $B/hip_init_probe_rccl >> $O/hip_init.txt 2>&1 || exit 11
  echo "deferred=0 rccl:" >> $O/hip_init.txt
  HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 5 60 $B/hip_init_probe_rccl >> $O/hip_init.txt 2>&1 || exit 12
done
