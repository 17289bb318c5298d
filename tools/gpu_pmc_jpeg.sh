#!/bin/bash
# (gpurun) JPEG encoder SQ counters per truncation variant (see tools/gpu_r4_k.sh), isolated engine
# runs (1 stream, batch 96). Usage: bash tools/gpu_pmc_jpeg.sh <out-name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-pmc}; mkdir -p $O
B=build/bin
D=/tmp/pmc_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for v in 7 1 16 2 4 0 40 41; do
  NM03_PROFILE_VARIANT=jpeg=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/v$v -o k \
    -- $B/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --streams 1 --batch-size 96 \
    > $O/v$v.log 2>&1 || exit 12
done
rm -rf $D
