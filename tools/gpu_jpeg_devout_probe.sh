#!/bin/bash
# JPEG store-phase probe (gpurun): isolated kernel times (batch 64, one stream) and the headline
# bench with the encoder writing over PCIe into mapped host memory (default) vs into HBM
# (NM03_JPEG_DEVOUT_PROBE=1, timing only: the JPEG files it writes are garbage). gpurun_out/devout/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/devout; mkdir -p $O
D=/tmp/devout_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for i in 1 2; do
  for t in host hbm; do
    P=0; [ $t = hbm ] && P=1
    NM03_JPEG_DEVOUT_PROBE=$P timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t$i -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
      > $O/$t$i.log 2>&1 || exit 33
    echo "$t$i" >> $O/summary.txt
    python3 tools/kstats.py $O/$t$i/run_kernel_stats.csv >> $O/summary.txt || exit 34
  done
done
for i in 1 2 3; do
  for t in host hbm; do
    P=0; [ $t = hbm ] && P=1
    NM03_JPEG_DEVOUT_PROBE=$P timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 \
      > $O/bench_$t$i.log 2>&1 || exit 35
    echo "bench $t$i $(grep -o '"value": [0-9.]*' $O/bench_$t$i.log | head -1)" >> $O/summary.txt
  done
done
