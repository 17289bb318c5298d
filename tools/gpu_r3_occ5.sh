#!/bin/bash
# (gpurun) JPEG encoder at 5 vs 4 workgroups per CU (NM03_JPEG_OCC) on the dot-product FDCT:
# isolated batch 96 one stream (2 interleaved reps), then the in-bench kernel table of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3occ5; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "jpeg" > $O/pytest.log 2>&1 || exit 31
NM03_JPEG_OCC=5 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "jpeg" > $O/pytest_occ5.log 2>&1 || exit 32
D=/tmp/r3occ_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for occ in 4 5; do
    NM03_JPEG_OCC=$occ timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/o${occ}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
      > $O/o${occ}_$rep.log 2>&1 || exit 42
    python3 tools/kstats.py $O/o${occ}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/occ$occ rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
for occ in 4 5; do
  NM03_JPEG_OCC=$occ timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_o$occ -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 3 > $O/prof_o$occ.log 2>&1 || exit 51
  python3 tools/kstats.py $O/prof_o$occ/bench_kernel_stats.csv | grep jpeg | sed "s/^/bench occ$occ /" >> $O/summary.txt
done
