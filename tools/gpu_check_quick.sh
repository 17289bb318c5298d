#!/bin/bash
# (gpurun) GPU tests + isolated kernel stats at batch 64 and 16 (tools/gpu_kprof.sh) + 3 bench runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 30
bash tools/gpu_kprof.sh && cp gpurun_out/kprof.txt gpurun_out/kprof_b64.txt || exit 20
bash tools/gpu_kprof.sh --batch-size 16 && cp gpurun_out/kprof.txt gpurun_out/kprof_b16.txt || exit 21
O=gpurun_out/quick_bench.txt
: > $O
for r in 1 2 3; do
  echo "run$r" >> $O
  timeout -k 10 200 python bench.py --keep-data 2>/dev/null | grep metric >> $O || exit 31
done
