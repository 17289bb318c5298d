#!/bin/bash
# (gpurun) Sharpen/SRG bit-exact tests, then the isolated JPEG encoder time split by truncated
# variants at batch 96 (NM03_JPEG_DBG; outputs invalid): 8 = empty workgroup, 7 = tables + ticket,
# 6 = no render (stop before FDCT), 1 = render only, 2 = + FDCT/quant/AC coding,
# 4 = everything but the output write, 0 = full. Plus one LDS-conflict PMC pass. gpurun_out/r3j/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3j; mkdir -p $O/pmc
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "sharpen or region_grow or engine_single or volume_vs_golden or cohort_configs" > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3j_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for v in 8 7 6 1 2 4 0; do
  NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d$v -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
    > $O/d$v.log 2>&1 || exit 42
  python3 tools/kstats.py $O/d$v/run_kernel_stats.csv > $O/d$v.txt || exit 43
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $O/pmc/p1 -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 96 --streams 1 > $O/pmc/p1.log 2>&1 || exit 71
python3 tools/pmc_summary.py $O/pmc $O/d0/run_kernel_stats.csv > $O/pmc_summary.txt 2>&1 || exit 69
rm -rf $D
