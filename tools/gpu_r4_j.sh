#!/bin/bash
# (gpurun) Round 4: after the fast-exit handler moved to libnm03's load and the 512-block JPEG fix.
# gpurun_out/r4j/: exit-handler order under rocprofv3 (tools/exit_order); GPU tests; JPEG encoder split under rocprofv3 (exit status + CSV written);
# then tools/gpu_r4_g.sh (JPEG wg 256 vs 512), _f.sh (large-BAR A/B, CLI start-up log), _h.sh
# (median 16-wide network A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4j; mkdir -p $O/split
B=build/bin
{ timeout -k 5 30 build/bin/exit_order_probe; echo "plain exit $?"; } > $O/exit_order.txt 2>&1
timeout -k 5 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/exit_order -o e -- build/bin/exit_order_probe \
  >> $O/exit_order.txt 2>&1
echo "rocprofv3 exit $? csv $(ls $O/exit_order/*kernel_stats.csv 2>/dev/null | wc -l)" >> $O/exit_order.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
D=/tmp/r4j_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for v in 0 40 41 7 1 2 4 15; do
  NM03_PROFILE_VARIANT=jpeg=$v timeout -k 10 60 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split/v$v -o k \
    -- $B/nm03_bench --config cohort --data-root $D/ --steps 3 --warmup 1 --streams 1 --batch-size 96 \
    > $O/split/v$v.log 2>&1
  rc=$?
  echo "v$v exit $rc csv $(ls $O/split/v$v/*kernel_stats.csv 2>/dev/null | wc -l)" >> $O/split/status.txt
  [ $rc -eq 0 ] || exit 12  # (CSV presence recorded, not required)
done
rm -rf $D
sed -i 's/^timeout -k 10 400 python -u -m pytest.*/true/' tools/gpu_r4_f.sh tools/gpu_r4_g.sh  # tests ran above
bash tools/gpu_r4_g.sh || exit $((100 + $?))
bash tools/gpu_r4_f.sh || exit $((150 + $?))
bash tools/gpu_r4_h.sh || exit $((200 + $?))
