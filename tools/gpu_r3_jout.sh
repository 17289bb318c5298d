#!/bin/bash
# (gpurun) JPEG output-store A/B, isolated at batch 96 (one stream): 16-byte stores (default),
# r2 dword stores (NM03_JPEG_DBG=13), staged but not stored (15), and the host-mapped output
# allocated coherent / non-coherent (NM03_JPEG_OUT_MEM). gpurun_out/r3o/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "jpeg or engine or cli_sequential_equals or sharpen" > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3o_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
    > $O/$n.log 2>&1 || return 1
  python3 tools/kstats.py $O/$n/run_kernel_stats.csv | grep jpeg | sed "s/^/$n /" >> $O/summary.txt
}
for rep in 1 2; do
  run s16_$rep NM03_JPEG_DBG=0 || exit 42
  run dw_$rep NM03_JPEG_DBG=13 || exit 43
  run nostore_$rep NM03_JPEG_DBG=15 || exit 44
  run coh_$rep NM03_JPEG_OUT_MEM=coherent || exit 45
  run noncoh_$rep NM03_JPEG_OUT_MEM=noncoherent || exit 46
done
mkdir -p $O/pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES --output-format csv -d $O/pmc/p1 -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 96 --streams 1 > $O/pmc/p1.log 2>&1 || exit 71
python3 tools/pmc_summary.py $O/pmc $O/s16_1/run_kernel_stats.csv > $O/pmc_summary.txt 2>&1 || exit 69
rm -rf $D
