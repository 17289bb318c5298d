#!/bin/bash
# JPEG encoder occupancy A/B (gpurun): NM03_JPEG_OCC=5 (5 workgroups/CU, ≤ 96 VGPRs, smaller LDS
# union) vs the default 4 — JPEG GPU tests under OCC=5, then isolated kernel times at batch 64 and
# 128, alternated twice. gpurun_out/jocc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/jocc; mkdir -p $O
NM03_JPEG_OCC=5 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "jpeg or cohort_configs or sequential_equals" > $O/pytest_occ5.log 2>&1 || exit 31
D=/tmp/jocc_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for i in 1 2; do
  for occ in 4 5; do
    for b in 64 128; do
      NM03_JPEG_OCC=$occ timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o$occ-$i-b$b -o run \
        -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size $b \
        > $O/o$occ-$i-b$b.log 2>&1 || exit 33
      echo "occ $occ run $i batch $b" >> $O/summary.txt
      python3 tools/kstats.py $O/o$occ-$i-b$b/run_kernel_stats.csv | grep -E "jpeg" >> $O/summary.txt || exit 34
    done
  done
done
for i in 1 2; do
  for occ in 4 5; do
    NM03_JPEG_OCC=$occ timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-secondary > $O/bench_o${occ}_$i.log 2>&1 || exit 35
  done
done
