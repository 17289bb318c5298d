#!/bin/bash
# K1 (median + sharpen) A/B on one box (gpurun): GPU kernel tests, then isolated kernel stats
# (native cohort bench, batch 64, one stream) for the current tree and abprev/ (take abprev/ out of
# .gpurunignore for the call), alternated twice, then one PMC pass of instruction counts on the
# current tree. Summaries in gpurun_out/k1ab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/k1ab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "median or sharpen or engine or pipeline" > $O/pytest.log 2>&1 || exit 31
D=/tmp/k1_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 32
for i in 1 2; do
  for t in cur prev; do
    R=.; [ $t = prev ] && R=abprev
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$t$i -o run \
      -- $R/build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
      > $O/$t$i.log 2>&1 || exit 33
    python3 tools/kstats.py $O/$t$i/run_kernel_stats.csv > $O/kstats_$t$i.txt || exit 34
  done
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
  --output-format csv -d $O/pmc -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 64 --streams 1 > $O/pmc.log 2>&1 || exit 35
