#!/bin/bash
# (gpurun) Round 4 (second half of tools/gpu_r4_k.sh, whose bench run had dropped its data): JPEG encoder instruction mix per phase. For each truncation variant
# (NM03_PROFILE_VARIANT=jpeg=N: 7 tables+ticket, 1 +render, 16 +FDCT+quant, 2 +AC coding,
# 4 +scan/bit range/look-back, 0 full; 40/41 gray/label only) one rocprofv3 --pmc pass of SQ
# counters over the isolated encoder (1 stream, batch 96). Before that: config 5 (256-slice volume)
# under rocprofv3 --kernel-trace (exit status and CSV written), and the headline bench's kernel stats.
# gpurun_out/r4k/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4k2; mkdir -p $O
B=build/bin
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --single-passes 0 --cli-runs 0 --wipe-passes 0 --keep-data > $O/bench.json 2> $O/bench.err || exit 7
DD=/dev/shm/nm03_bench_data-node0; [ -d $DD ] || DD=$(ls -d /dev/shm/nm03_bench_data* | head -1)
for i in 1 2 3; do  # cold CLI start-up detail (engine set-up split in the info log)
  NM03_LOG=info timeout -k 10 60 $B/img_processing_parallel --gpus 1 --data-root $DD/ --out /dev/shm/r4k_cli --quiet \
    --json $O/cli_$i.json > $O/cli_$i.log 2>&1 || exit 8
done
rm -rf /dev/shm/nm03_bench_data* /dev/shm/r4k_cli
D=/tmp/r4k_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
for v in 7 1 16 2 4 0 40 41; do
  NM03_PROFILE_VARIANT=jpeg=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/v$v -o k \
    -- $B/nm03_bench --config cohort --data-root $D/ --steps 2 --warmup 1 --streams 1 --batch-size 96 \
    > $O/v$v.log 2>&1 || exit 12
done
rm -rf $D
