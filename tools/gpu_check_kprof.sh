#!/bin/bash
# GPU tests (JPEG/engine subset by default) then isolated kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
bash tools/gpu_kprof.sh || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 53
