#!/bin/bash
# (gpurun) LDS-staged gray render in the JPEG encoder: GPU tests, isolated kernel A/B (NM03_JPEG_DBG=12
# = global patch loads), bench A/B interleaved 3x.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 30
rm -f gpurun_out/split.txt
VARIANTS="0 12" bash tools/gpu_jpeg_split.sh || exit 20
O=gpurun_out/lds_ab.txt
: > $O
for r in 1 2 3; do
  for v in 12 0; do
    echo "dbg$v" >> $O
    NM03_JPEG_DBG=$v timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
