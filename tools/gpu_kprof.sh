#!/bin/bash
# Isolated kernel durations (gpurun): the native cohort driver with ONE stream (no kernel
# overlap, so per-kernel times are not inflated by concurrency) under rocprofv3 --kernel-trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 "$@" \
  > gpurun_out/kprof.log 2>&1 || exit 2
python3 tools/kstats.py gpurun_out/kprof/run_kernel_stats.csv > gpurun_out/kprof.txt || exit 3
