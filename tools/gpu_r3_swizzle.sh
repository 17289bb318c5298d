#!/bin/bash
# (gpurun) JPEG gray staging rows swizzled for conflict-free patch reads (default) vs plain rows
# (NM03_JPEG_SWIZZLE=0): GPU tests, isolated batch 96 (2 interleaved reps), in-bench kernel table of
# each, 3 bench pairs. gpurun_out/r3swz/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3swz; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3sw_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for sp in 1 0; do
    NM03_JPEG_SWIZZLE=$sp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/i${sp}_$rep -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
      > $O/i${sp}_$rep.log 2>&1 || exit 42
    python3 tools/kstats.py $O/i${sp}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/iso swizzle$sp rep$rep /" >> $O/summary.txt
  done
done
rm -rf $D
for sp in 1 0; do
  NM03_JPEG_SWIZZLE=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$sp -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 3 > $O/b$sp.log 2>&1 || exit 51
  python3 tools/kstats.py $O/b$sp/bench_kernel_stats.csv | grep jpeg | sed "s/^/bench swizzle$sp /" >> $O/summary.txt
done
for rep in 1 2 3; do
  for sp in 1 0; do
    NM03_JPEG_SWIZZLE=$sp timeout -k 10 300 python3 bench.py --steps 50 --wipe-passes 0 --single-passes 20 > $O/h${sp}_$rep.log 2>&1 || exit 60
    python3 - $O/h${sp}_$rep.log "swizzle$sp rep$rep" >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        j = json.loads(l); c = j['config']
        print(f"{sys.argv[2]:14s} value={j['value']:9.0f} cpu/step={c['rank0_process_cpu_ms_per_step']:6.2f} shard8={c['strong'].get('single_pass_shard8_ms')}")
PY
  done
done
