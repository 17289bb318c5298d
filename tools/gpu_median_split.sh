#!/bin/bash
# Median kernel split (gpurun): isolated profile with NM03_MEDIAN_DBG variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for v in ${VARIANTS:-0 1}; do
  NM03_MEDIAN_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/msplit$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
    > gpurun_out/msplit$v.log 2>&1 || exit $((10 + v))
  echo "variant $v" >> gpurun_out/msplit.txt
  python3 tools/kstats.py gpurun_out/msplit$v/run_kernel_stats.csv | grep -E "median|sharpen" >> gpurun_out/msplit.txt
done
