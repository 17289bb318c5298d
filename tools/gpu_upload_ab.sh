#!/bin/bash
# (gpurun) GPU tests, then A/B of progressive uploads: NM03_UPLOAD_CHUNK_KB=0 (one upload per batch)
# vs 1024 / 2048 (default) / 4096, interleaved 3x; timeline of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 30
O=gpurun_out/upload_ab.txt
: > $O
for r in 1 2 3; do
  for c in 0 1024 2048 4096; do
    echo "chunk$c" >> $O
    NM03_UPLOAD_CHUNK_KB=$c timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
  done
done
bash tools/gpu_timeline.sh || exit 32
