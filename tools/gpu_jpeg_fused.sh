#!/bin/bash
# Fused JPEG stuffing check: JPEG + engine GPU tests first (byte-identity vs libjpeg/golden), then
# the whole GPU suite, a bench and rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/jf
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "jpeg or engine_single or engine_cohort" > gpurun_out/jf/pytest_jpeg.log 2>&1 || exit 31
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/jf/pytest_gpu.log 2>&1 || exit 32
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/jf/bench.log 2>&1 || exit 33
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/jf/prof -o b -- python3 bench.py --steps 20 --warmup 2 --no-secondary > gpurun_out/jf/prof.log 2>&1 || exit 34
