#!/bin/bash
# Time split of the fused JPEG kernel (gpurun): isolated kernel profile of each truncated variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for v in ${VARIANTS:-0 1 2 3 4}; do
  NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/split$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
    > gpurun_out/split$v.log 2>&1 || exit $((10 + v))
  echo "variant $v" >> gpurun_out/split.txt
  python3 tools/kstats.py gpurun_out/split$v/run_kernel_stats.csv | grep jpeg_fused >> gpurun_out/split.txt
done
