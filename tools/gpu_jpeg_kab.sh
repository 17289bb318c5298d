#!/bin/bash
# JPEG encoder A/B (gpurun): GPU tests touching the encoder, then isolated kernel times at batch 64
# and 128 for the current tree and abprev/ (take abprev/ out of .gpurunignore), alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/jkab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "jpeg or engine or cli or volume" > $O/pytest.log 2>&1 || exit 31
D=/tmp/jkab_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for i in 1 2; do
  for t in cur prev; do
    R=.; [ $t = prev ] && R=abprev
    for b in 64 128; do
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t$i-b$b -o run \
        -- $R/build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size $b \
        > $O/$t$i-b$b.log 2>&1 || exit 33
      echo "$t$i batch $b" >> $O/summary.txt
      python3 tools/kstats.py $O/$t$i-b$b/run_kernel_stats.csv | grep -E "jpeg" >> $O/summary.txt || exit 34
    done
  done
done
