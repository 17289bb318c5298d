#!/bin/bash
# Batch-schedule A/B (gpurun): NM03_BATCH_SPREAD=1 (equal-size batches; short lists spread over the
# slots) vs 0 (full batches + remainder). GPU tests with spread on, then interleaved: the headline
# bench (1 rank), config 2 (one patient, batch 25, 3 streams, nm03_bench) and config.strong with
# 8 ranks sharing the GPU (58-slice shards). gpurun_out/spread/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/spread; mkdir -p $O
NM03_BATCH_SPREAD=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_spread.log 2>&1 || exit 31
T=/tmp/spread_data; build/bin/nm03_synth --data-root $T/patient/ --patients 1 --threads 16 > /dev/null || exit 32
for i in 1 2 3; do
  for sp in 0 1; do
    NM03_BATCH_SPREAD=$sp timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 > $O/bench_${sp}_$i.log 2>&1 || exit 33
    NM03_BATCH_SPREAD=$sp timeout -k 10 120 build/bin/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/sp_o2 --steps 50 --warmup 5 --batch-size 25 --streams 3 > $O/c2_${sp}_$i.json 2>&1 || exit 34
    echo "spread=$sp $i bench $(grep -o '"value": [0-9.]*' $O/bench_${sp}_$i.log | head -1) c2 $(grep -o '"slices_per_s": [0-9.]*' $O/c2_${sp}_$i.json)" >> $O/summary.txt
  done
done
for i in 1 2; do
  for sp in 0 1; do
    NM03_BATCH_SPREAD=$sp NM03_DEVICE_OVERRIDE=0 timeout -k 10 400 python bench.py --gpus 8 --steps 20 --warmup 3 --wipe-passes 0 > $O/r8_${sp}_$i.log 2>&1 || exit 35
    echo "spread=$sp $i 8 ranks weak $(grep -o '"value": [0-9.]*' $O/r8_${sp}_$i.log | head -1) strong $(grep -o '"strong": {"value": [0-9.]*' $O/r8_${sp}_$i.log)" >> $O/summary.txt
  done
done
