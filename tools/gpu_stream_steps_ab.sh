#!/bin/bash
# A/B (gpurun): bench.py with one engine call per cohort pass (default) vs --stream-steps, interleaved. gpurun_out/ss/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ss
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --keep-data > gpurun_out/ss/bench_step_$i.log 2>&1 || exit 32
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --keep-data --stream-steps > gpurun_out/ss/bench_stream_$i.log 2>&1 || exit 33
done
rm -rf /dev/shm/nm03_bench_data*
