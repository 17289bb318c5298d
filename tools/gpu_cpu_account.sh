#!/bin/bash
# Host CPU accounting (gpurun): two bench.py runs; per-step CPU of loaders, writers, slot threads,
# the whole process and the cgroup. JSON in gpurun_out/cpu_account.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/cpu_account.txt
: > $O
for r in 1 2; do
  echo "default" >> $O
  timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
done
