#!/bin/bash
# hipGraph replay of the batch chain vs eager launches on the pipelined bench (gpurun), interleaved 3×.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/gab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "cohort_configs" > $O/pytest.log 2>&1 || exit 31
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/eager_$i.log 2>&1 || exit 41
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --graphs > $O/graphs_$i.log 2>&1 || exit 42
done
