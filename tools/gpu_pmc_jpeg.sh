#!/bin/bash
# PMC counters of the JPEG encoder profiling variants (gpurun): VARIANTS="1 6" by default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcj
D=/tmp/nm03_pmc_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 61
for v in ${VARIANTS:-1 6}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    NM03_JPEG_DBG=$v timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcj/v$v/p$i -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 1 --warmup 1 --batch-size 64 --streams 1 \
      > gpurun_out/pmcj/v$v.p$i.log 2>&1 || exit $((70+i))
  done
  echo "== variant $v" >> gpurun_out/pmcj/summary.txt
  python3 tools/pmc_summary.py gpurun_out/pmcj/v$v | grep -A16 jpeg_fused >> gpurun_out/pmcj/summary.txt
done
