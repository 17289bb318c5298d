#!/bin/bash
# A/B (gpurun): loader read path NM03_LOAD_MODE=staged (default) vs mapped, interleaved bench.py
# runs; engine GPU tests once under mapped. gpurun_out/map/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/map
NM03_LOAD_MODE=mapped timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q -k "engine or cli" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/map/pytest_mapped.log 2>&1 || exit 31
for i in 1 2 3 4; do
  for v in staged mapped; do
    NM03_LOAD_MODE=$v timeout -k 10 300 python bench.py --steps 100 --warmup 5 --keep-data > gpurun_out/map/bench_${v}_$i.log 2>&1 || exit 32
  done
done
rm -rf /dev/shm/nm03_bench_data*
