#!/bin/bash
# (gpurun) headline bench: streams × progressive chunk sweep, 2 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/c3_streams.txt
: > $O
for r in 1 2; do
  for v in "6 2048" "3 2048" "3 8192" "5 2048" "5 8192" "7 2048" "3 0"; do
    set -- $v
    echo "streams$1 chunk$2" >> $O
    NM03_UPLOAD_CHUNK_KB=$2 timeout -k 10 200 python bench.py --keep-data --streams $1 2>/dev/null | grep metric >> $O || exit 31
  done
done
