#!/bin/bash
# Quick check (gpurun): GPU tests, isolated kernel stats (batch 64, one stream), 3 bench runs. gpurun_out/ck/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ck
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ck/pytest_gpu.log 2>&1 || exit 31
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ck/k -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
  > gpurun_out/ck/k.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/ck/k/run_kernel_stats.csv > gpurun_out/ck/kstats.txt || exit 5
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/ck/bench_$i.log 2>&1 || exit 6
done
