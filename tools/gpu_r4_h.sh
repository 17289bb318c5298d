#!/bin/bash
# (gpurun) Round 4: median k=7 network 16 outputs wide (abmed/: worktree build, 128-thread
# workgroups) vs 8 wide (current tree), isolated kernel stats (1 stream, batch 96), 3 interleaved
# rounds; output trees of both builds compared byte for byte. gpurun_out/r4h/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4h; mkdir -p $O
D=/tmp/r4h_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for r in 1 2 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cur_$r -o k \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/r4h_cur --steps 5 --warmup 1 --streams 1 --batch-size 96 \
    > $O/cur_$r.log 2>&1 || exit 12
  LD_LIBRARY_PATH=$PWD/abmed/lib:/opt/rocm/lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w16_$r -o k \
    -- abmed/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/r4h_w16 --steps 5 --warmup 1 --streams 1 --batch-size 96 \
    > $O/w16_$r.log 2>&1 || exit 13
done
diff -r /tmp/r4h_cur /tmp/r4h_w16 > $O/diff.txt && echo "trees identical" > $O/diff_ok.txt
rm -rf $D /tmp/r4h_cur /tmp/r4h_w16
