#!/bin/bash
# Final round-3 tree: hardware counters per kernel (gpurun), one rocprofv3 --pmc pass per counter group, on the native
# cohort bench with ONE stream (no kernel overlap) and batch 64: instruction mix, VALU/LDS
# activity, LDS bank conflicts, HBM/L2 bytes (FETCH_SIZE / WRITE_SIZE, own passes: 3 + 2 TCC
# counters). No tracing domain is combined with --pmc. Summary: gpurun_out/pmcr3/summary.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcr3
D=/tmp/nm03_pmc_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 61
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcr3/p$i -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 96 --streams 1 \
    > gpurun_out/pmcr3/p$i.log 2>&1 || exit $((70+i))
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcr3/kt -o run \
  -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --batch-size 96 --streams 1 \
  > gpurun_out/pmcr3/kt.log 2>&1 || exit 79
python3 tools/pmc_summary.py gpurun_out/pmcr3 gpurun_out/pmcr3/kt/run_kernel_stats.csv > gpurun_out/pmcr3/summary.txt 2>&1 || exit 69
