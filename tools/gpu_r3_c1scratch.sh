#!/bin/bash
# (gpurun) Config 1 (one slice, 5 canvases + JPEGs) with the scratch-free default encoder vs the
# 5-per-CU variant that spills to scratch (NM03_JPEG_OCC=5): does a scratch-using kernel cost
# per-dispatch latency? Plus a kernel trace of each. gpurun_out/r3c1/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3c1; mkdir -p $O
T=/tmp/nm03_c1; build/bin/nm03_synth --data-root $T/ --patients 2 --threads 16 > /dev/null || exit 10
for rep in 1 2 3; do
  for occ in 4 5; do
    NM03_JPEG_OCC=$occ timeout -k 10 120 build/bin/nm03_bench --config single --data-root $T/ --steps 50 --warmup 5 > $O/c1_o${occ}_$rep.json || exit 11
    echo "occ$occ rep$rep $(cat $O/c1_o${occ}_$rep.json)" >> $O/summary.txt
  done
done
for occ in 4 5; do
  NM03_JPEG_OCC=$occ timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_o$occ -o run -- build/bin/nm03_bench --config single --data-root $T/ --steps 20 --warmup 5 > $O/kt_o$occ.log 2>&1 || exit 12
  python3 tools/kstats.py $O/kt_o$occ/run_kernel_stats.csv > $O/kt_o$occ.txt || exit 13
done
rm -rf $T
