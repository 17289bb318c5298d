#!/bin/bash
# (gpurun) Why the flat-wave path did not move the encoder: JPEG/engine GPU tests on the dot-product
# FDCT, isolated encoder time at batch 96 (one stream) for NM03_JPEG_FLAT=1/0 x full / dbg 2 (stop
# after the AC coding), 2 interleaved reps, and per-kernel PMC (VALU/SALU instructions, busy and
# wave cycles) for FLAT=1/0. gpurun_out/r3flat2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3flat2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "jpeg or engine or smoke" > $O/pytest.log 2>&1 || exit 31
D=/tmp/r3flat_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for rep in 1 2; do
  for v in 0 2; do
    for f in 1 0; do
      NM03_JPEG_FLAT=$f NM03_JPEG_DBG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/d${v}f${f}_$rep -o run \
        -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size 96 \
        > $O/d${v}f${f}_$rep.log 2>&1 || exit 42
      python3 tools/kstats.py $O/d${v}f${f}_$rep/run_kernel_stats.csv | grep jpeg | sed "s/^/dbg$v flat$f rep$rep /" >> $O/summary.txt
    done
  done
done
for f in 1 0; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    NM03_JPEG_FLAT=$f timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_f$f/p$i -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 1 --warmup 1 --batch-size 96 --streams 1 \
      > $O/pmc_f$f.p$i.log 2>&1 || exit $((70+i))
  done
  echo "== flat $f" >> $O/pmc_summary.txt
  python3 tools/pmc_summary.py $O/pmc_f$f | grep -A12 jpeg_fused >> $O/pmc_summary.txt
done
rm -rf $D
