#!/bin/bash
# Wave-quantisation probe (gpurun): isolated K1/K2/K4 kernel times vs batch size (WGs per launch =
# 16 × batch for the 64×64-tile kernels) on the native cohort bench, one stream. gpurun_out/bq/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/bq; mkdir -p $O
D=/tmp/bq_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for b in ${BATCHES:-32 48 56 60 62 64 66 72 96 128}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$b -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size $b \
    > $O/b$b.log 2>&1 || exit 33
  echo "batch $b" >> $O/summary.txt
  python3 tools/kstats.py $O/b$b/run_kernel_stats.csv | grep -E "median|sharpen|srg|jpeg" >> $O/summary.txt || exit 34
done
