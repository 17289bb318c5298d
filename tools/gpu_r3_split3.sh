#!/bin/bash
# (gpurun) JPEG: FDCT + quantisation alone (NM03_JPEG_DBG=16) vs + AC coding (2), isolated batch 96,
# 2 reps. gpurun_out/r3split3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3split3; mkdir -p $O
D=/tmp/r3s3_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for v in 16 2 0; do
    NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d${v}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
      > $O/d${v}_$rep.log 2>&1 || exit 42
    python3 tools/kstats.py $O/d${v}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/dbg$v rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
