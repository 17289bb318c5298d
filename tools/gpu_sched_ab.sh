#!/bin/bash
# A/B (gpurun): batch schedule — uniform 64 (default) vs tapered 64 vs uniform 48 / 32, interleaved 2x,
# then a timeline of the default. Results in gpurun_out/sched_ab.txt, gpurun_out/timeline.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/sched_ab.txt
: > $O
for r in 1 2; do
  for v in "0 64 6" "1 64 6" "0 48 8" "0 32 10"; do
    set -- $v
    echo "taper$1 b$2 s$3" >> $O
    NM03_BATCH_TAPER=$1 timeout -k 10 200 python bench.py --keep-data --batch-size $2 --streams $3 2>/dev/null | grep metric >> $O || exit 31
  done
done
bash tools/gpu_timeline.sh || exit 32
