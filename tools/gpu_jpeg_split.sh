#!/bin/bash
# Isolated JPEG encoder time split by truncated variants (NM03_JPEG_DBG; outputs invalid):
# 1 = render only, 2 = + FDCT/quant/AC coding, 4 = everything but the output write, 0 = full.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/split
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for v in 1 2 4 0; do
  NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split/d$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
    > gpurun_out/split/d$v.log 2>&1 || exit 4
  python3 tools/kstats.py gpurun_out/split/d$v/run_kernel_stats.csv | grep jpeg > gpurun_out/split/d$v.txt
done
