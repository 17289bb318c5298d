#!/bin/bash
# (gpurun) JPEG-focused check: JPEG/engine GPU tests, then isolated kernel stats at batch 96 (one
# stream; full kernel and the NM03_JPEG_DBG=7 prologue variant), 2 reps each. gpurun_out/r3ji/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3ji; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "jpeg_kernel" > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3ji_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for v in 0 17; do
    NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d${v}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 ${EXTRA} \
      > $O/d${v}_$rep.log 2>&1 || exit 42
    python3 tools/kstats.py $O/d${v}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/dbg$v rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
