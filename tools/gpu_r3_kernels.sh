#!/bin/bash
# (gpurun) Round-3 kernel evidence: GPU tests, isolated kernel times (one stream) at batch 64 and 96,
# hardware counters per kernel at batch 96 (one --pmc pass per counter group), and the bench's
# kernel stats under its 4-stream concurrency. Logs in gpurun_out/r3k/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O/pmc
P=$O/progress.txt
echo "start $(date)" > $P
[ -n "$SKIP_TESTS" ] || bash tools/gpu_tests.sh || exit 31
echo "pytest ok $(date)" >> $P
D=/tmp/nm03_r3k_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
for b in 64 96; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso$b -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 4 --warmup 1 --streams 1 --batch-size $b \
    > $O/iso$b.log 2>&1 || exit 42
  python3 tools/kstats.py $O/iso$b/run_kernel_stats.csv > $O/iso$b.txt || exit 43
done
echo "iso ok $(date)" >> $P
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/pmc/p$i -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 96 --streams 1 \
    > $O/pmc/p$i.log 2>&1 || exit $((70+i))
done
python3 tools/pmc_summary.py $O/pmc $O/iso96/run_kernel_stats.csv > $O/pmc_summary_b96.txt 2>&1 || exit 69
echo "pmc ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 5 > $O/bench_prof.log 2>&1 || exit 51
python3 tools/kstats.py $O/bench/bench_kernel_stats.csv > $O/bench_kernels.txt || exit 52
timeout -k 10 300 python bench.py > $O/bench_a.log 2>&1 || exit 53
timeout -k 10 300 python bench.py > $O/bench_b.log 2>&1 || exit 54
rm -rf $D
echo "done $(date)" >> $P
