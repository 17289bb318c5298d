#!/bin/bash
# (gpurun) JPEG time split on the spread order (NM03_JPEG_DBG truncated variants, outputs invalid):
# 7 = tables + ticket, 1 = + render and stop, 2 = + FDCT/quant/AC coding, 4 = + scan/look-back/assembly,
# 15 = + output staging, 0 = full; plus the 5-per-CU encoder (NM03_JPEG_OCC=5). Isolated, batch 96.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3split2; mkdir -p $O
D=/tmp/r3s2_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for v in 7 1 2 4 15 0; do
  NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
    > $O/d$v.log 2>&1 || exit 42
  python3 tools/kstats.py $O/d$v/run_kernel_stats.csv | grep jpeg | sed "s/^/dbg$v /" >> $O/summary.txt
done
for rep in 1 2; do
  for occ in 5 4; do
    NM03_JPEG_OCC=$occ timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o${occ}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
      > $O/o${occ}_$rep.log 2>&1 || exit 43
    python3 tools/kstats.py $O/o${occ}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/occ$occ rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
