#!/bin/bash
# (gpurun) the GPU test suite only; log in gpurun_out/pytest_gpu.log.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/pytest_gpu.log 2>&1
