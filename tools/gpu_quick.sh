#!/bin/bash
# Quick perf probe (gpurun): GPU tests, bench x2 (+ spin-wait A/B), timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 53
NM03_EVENT_SPIN=1 timeout -k 10 300 python bench.py > gpurun_out/bench_spin.log 2>&1 || exit 54
timeout -k 10 300 python bench.py > gpurun_out/bench2.log 2>&1 || exit 56
bash tools/gpu_timeline.sh || exit 55
