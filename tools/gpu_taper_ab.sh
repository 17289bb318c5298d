#!/bin/bash
# A/B (gpurun): uniform vs tapered batch schedule (NM03_BATCH_TAPER), 5 interleaved pairs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/taper_ab.txt
: > $O
for r in 1 2 3 4 5; do
  for t in 0 1; do
    echo "taper$t" >> $O
    NM03_BATCH_TAPER=$t timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
