#!/bin/bash
# JPEG iteration: JPEG/engine GPU tests, then the isolated kernel profile (1 stream, batch 64).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/jf
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "jpeg or engine or volume_cli" > gpurun_out/jf/pytest_jpeg.log 2>&1 || exit 31
bash tools/gpu_kprof_quick.sh || exit 32
