#!/bin/bash
# Latency-bound configs (1: single slice, 2: one patient) and the native cohort driver, current tree
# vs abprev/ (the round's session-start commit, built in place; take abprev/ out of .gpurunignore),
# plus the current tree with the AVX-512 packer and the export interleave switched off. 3 rounds,
# interleaved. gpurun_out/smallab/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/smallab; mkdir -p $O
T=/tmp/nm03_sab
build/bin/nm03_synth --data-root $T/cohort/ --threads 16 > /dev/null || exit 101
build/bin/nm03_synth --data-root $T/patient/ --patients 1 --threads 16 > /dev/null || exit 102
for i in 1 2 3; do
  for v in cur prev cur_noopt; do
    B=build/bin; E=""
    [ $v = prev ] && B=abprev/build/bin
    [ $v = cur_noopt ] && E="NM03_PACK_AVX512=0 NM03_EXPORT_INTERLEAVE=0"
    env $E timeout -k 10 120 $B/nm03_bench --config single --data-root $T/cohort/ --steps 50 --warmup 5 > $O/c1_${v}_$i.json || exit 111
    env $E timeout -k 10 120 $B/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/sab_o2 --steps 50 --warmup 5 --batch-size 25 --streams 3 > $O/c2_${v}_$i.json || exit 121
    env $E timeout -k 10 120 $B/nm03_bench --config cohort --data-root $T/cohort/ --out /tmp/sab_o3 --steps 20 --warmup 3 --batch-size 64 --streams 6 > $O/c3_${v}_$i.json || exit 131
    echo "$v $i c1 $(grep -o '"ms_per_slice": [0-9.]*' $O/c1_${v}_$i.json) c2 $(grep -o '"slices_per_s": [0-9.]*' $O/c2_${v}_$i.json) c3 $(grep -o '"slices_per_s": [0-9.]*' $O/c3_${v}_$i.json)" >> $O/summary.txt
  done
done
