#!/bin/bash
# (gpurun) Round 4, fourth call. gpurun_out/r4d/:
#  * GPU tests (device-resident z-slab exchange; staged through pinned memory by the host comm);
#  * JPEG encoder split, isolated (1 stream, batch 96, rocprofv3 kernel stats): full (0), gray only
#    (40), label only (41), tables + ticket (7), render only (1), + FDCT/quant/coding (2), all but
#    the output stores (4), staged but not stored (15);
#  * config 5: img_processing_parallel --mode 3d over 1 / 2 / 4 ranks on one GPU, outputs compared;
#  * cold-run sweep: reaper threads 2/4/6 × create_writers 4/8, 2 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4d; mkdir -p $O
B=build/bin
true
mkdir -p $O/split
D=/tmp/r4d_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for v in 0 40 41 7 1 2 4 15; do
  NM03_PROFILE_VARIANT=jpeg=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split/v$v -o k \
    -- $B/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 96 \
    > $O/split/v$v.log 2>&1 || exit 12
done
rm -rf $D
T=/tmp/r4vol
$B/nm03_synth --data-root $T/vol/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 20
for n in 1 2 4; do
  extra=""; [ $n -gt 1 ] && extra="--split-volume"
  NM03_DEVICE_OVERRIDE=0 timeout -k 10 180 $B/img_processing_parallel --mode 3d --gpus $n $extra --data-root $T/vol/ \
    --out $T/out$n --json $O/c5_cli_$n.json > $O/c5_cli_$n.log 2>&1 || exit $((20+n))
done
diff -r $T/out1 $T/out2 > $O/diff_1_2.txt && diff -r $T/out1 $T/out4 > $O/diff_1_4.txt || exit 30
echo "split-volume outputs identical" > $O/diff_ok.txt
rm -rf $T
A="--steps 40 --warmup 5 --wipe-passes 40 --single-passes 0 --cli-runs 0 --keep-data"
for r in 1 2; do
  for arm in "2 4" "4 4" "6 4" "4 8" "6 8"; do
    set -- $arm
    echo "round $r reaper=$1 cw=$2" >> $O/cold_ab.jsonl
    timeout -k 10 200 python3 bench.py $A --reaper-threads $1 --create-writers $2 >> $O/cold_ab.jsonl 2>> $O/cold_ab.err || exit 40
  done
done
