#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/kp
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kp/k -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
  > gpurun_out/kp/k.log 2>&1 || exit 4
python3 tools/kstats.py gpurun_out/kp/k/run_kernel_stats.csv > gpurun_out/kp/kstats.txt || exit 5
