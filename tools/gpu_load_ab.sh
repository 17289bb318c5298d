#!/bin/bash
# A/B (gpurun): loader read path — direct pread with a 16 KiB / 4 KiB header prefix vs staged
# whole-file read + streaming stores (NM03_LOAD_MODE / NM03_LOAD_PREFIX), interleaved 3x.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/load_ab.txt
: > $O
for r in 1 2 3; do
  for v in "direct 16384" "direct 4096" "staged 0"; do
    set -- $v
    echo "$1 $2" >> $O
    NM03_LOAD_MODE=$1 NM03_LOAD_PREFIX=$2 timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
