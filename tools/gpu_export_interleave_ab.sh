#!/bin/bash
# Export order A/B (gpurun): writers round-robin over the batch's output directories
# (NM03_EXPORT_INTERLEAVE=1, default) vs slice order (0). GPU tests first; then the headline and the
# wipe-each-pass figure (every pass creates its 930 JPEGs in freshly emptied directories), 4 rounds.
# gpurun_out/exp_il/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/exp_il; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 31
for i in 1 2 3 4; do
  for il in 1 0; do
    NM03_EXPORT_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 50 > $O/il${il}_$i.log 2>&1 || exit 33
    echo "interleave=$il round $i $(grep -o '"value": [0-9.]*' $O/il${il}_$i.log | head -1) wipe $(grep -o '"wipe_each_pass": {"value": [0-9.]*' $O/il${il}_$i.log)" >> $O/summary.txt
  done
done
