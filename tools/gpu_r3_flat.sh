#!/bin/bash
# (gpurun) JPEG flat-wave path A/B: GPU tests, isolated encoder stats at batch 96 (one
# stream) with the path (dbg 0) and without (NM03_JPEG_DBG=18), interleaved; then bench pairs and
# the in-bench kernel table of each. gpurun_out/r3flat/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3flat; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3flat_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for v in 0 18; do
    NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d${v}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
      > $O/d${v}_$rep.log 2>&1 || exit 42
    python3 tools/kstats.py $O/d${v}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/dbg$v rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
for rep in 1 2 3; do
  for v in 0 18; do
    NM03_JPEG_DBG=$v timeout -k 10 300 python3 bench.py --single-passes 20 > $O/bench_d${v}_$rep.log 2>&1 || exit 50
  done
done
for v in 0 18; do
  NM03_JPEG_DBG=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_d$v -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 3 > $O/prof_d$v.log 2>&1 || exit 51
  python3 tools/kstats.py $O/prof_d$v/bench_kernel_stats.csv > $O/bench_kernels_d$v.txt || exit 52
done
