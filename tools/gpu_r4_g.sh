#!/bin/bash
# (gpurun) Round 4: JPEG encoder workgroups of 512 vs 256 blocks. gpurun_out/r4g/:
#  * GPU tests (jpeg_wg 512 byte identity);
#  * isolated kernel time (1 stream, batch 96, rocprofv3 stats), interleaved 3 rounds;
#  * bench-run kernel stats (4 streams) and headline, interleaved 2 rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4g; mkdir -p $O
B=build/bin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
D=/tmp/r4g_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for r in 1 2 3; do
  for wg in 256 512; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso_${wg}_$r -o k \
      -- $B/nm03_bench --config cohort --data-root $D/ --steps 5 --warmup 1 --streams 1 --batch-size 96 --jpeg-wg $wg \
      > $O/iso_${wg}_$r.log 2>&1 || exit 12
  done
done
rm -rf $D
P="--steps 30 --warmup 3 --single-passes 0 --cli-runs 0 --wipe-passes 0 --keep-data"
for r in 1 2; do
  for wg in 256 512; do
    timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench_${wg}_$r -o k \
      -- python3 bench.py $P --jpeg-wg $wg > $O/bench_${wg}_$r.json 2> $O/bench_${wg}_$r.err || exit 20
  done
done
rm -rf /dev/shm/nm03_bench_data*
