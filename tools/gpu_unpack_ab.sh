#!/bin/bash
# A/B (gpurun): upload expansion fused into the median's tile load (default) vs the standalone K0
# pass (NM03_SEPARATE_UNPACK=1). GPU tests, isolated kernel stats of both, an LDS-conflict PMC pass
# of the default, then interleaved 1-GPU bench pairs. Results: gpurun_out/abu/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/abu
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abu/pytest_gpu.log 2>&1 || exit 31
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for v in 0 1; do
  NM03_SEPARATE_UNPACK=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abu/k$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 64 \
    > gpurun_out/abu/k$v.log 2>&1 || exit 4$v
  python3 tools/kstats.py gpurun_out/abu/k$v/run_kernel_stats.csv > gpurun_out/abu/kstats_$v.txt || exit 5$v
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU \
  --output-format csv -d gpurun_out/abu/pmc -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 64 --streams 1 \
  > gpurun_out/abu/pmc.log 2>&1 || exit 70
python3 tools/pmc_summary.py gpurun_out/abu/pmc gpurun_out/abu/k0/run_kernel_stats.csv > gpurun_out/abu/pmc_summary.txt 2>&1 || exit 71
for i in 1 2 3; do
  for v in 0 1; do
    NM03_SEPARATE_UNPACK=$v timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/abu/bench_${v}_$i.log 2>&1 || exit 6$v
  done
done
