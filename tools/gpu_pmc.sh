#!/bin/bash
# Hardware counters per kernel (gpurun): one rocprofv3 --pmc pass per counter group, on the
# native cohort bench (1 step). No tracing domains are combined with --pmc.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
D=/tmp/nm03_pmc_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 61
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
           "${@}"; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o run \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 1 --warmup 1 --batch-size 64 --streams 6 \
    > gpurun_out/pmc/p$i.log 2>&1 || exit $((70+i))
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1 || exit 69
