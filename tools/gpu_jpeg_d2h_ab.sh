#!/bin/bash
# JPEG export A/B (gpurun): HBM + gather + SDMA copy (NM03_JPEG_D2H=1) vs encoder stores into
# host-mapped memory (0) vs HBM + gather kernel storing into host-mapped memory (2). GPU tests first, then isolated kernel times (batch 64, one stream) and the
# headline bench, interleaved. gpurun_out/d2h/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/d2h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 31
D=/tmp/d2h_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for i in 1 2; do
  for t in 1 0 2; do
    NM03_JPEG_D2H=$t timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/k$t-$i -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
      > $O/k$t-$i.log 2>&1 || exit 33
    echo "d2h=$t run $i" >> $O/summary.txt
    python3 tools/kstats.py $O/k$t-$i/run_kernel_stats.csv >> $O/summary.txt || exit 34
  done
done
for i in 1 2 3; do
  for t in 1 0 2; do
    NM03_JPEG_D2H=$t timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 \
      > $O/bench_$t-$i.log 2>&1 || exit 35
    echo "bench d2h=$t $i $(grep -o '"value": [0-9.]*' $O/bench_$t-$i.log | head -1)" >> $O/summary.txt
  done
done
