#!/bin/bash
# (gpurun) GPU tests, then 12-bit transfer packing A/B (NM03_PACK12=0/1) on the headline bench,
# interleaved 4x, plus isolated kernel stats (K0 unpack cost).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 30
bash tools/gpu_kprof.sh || exit 20
O=gpurun_out/pack12_ab.txt
: > $O
for r in 1 2 3 4; do
  for v in 0 1; do
    echo "pack$v" >> $O
    NM03_PACK12=$v timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
