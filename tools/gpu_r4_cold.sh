#!/bin/bash
# (gpurun) Round 4, second call. gpurun_out/r4b/:
#  * the GPU test suite after the knob prune (k0/gather/graphs/d2h paths removed);
#  * hip_init_probe: HIP start-up split, default vs HIP_VISIBLE_DEVICES=0;
#  * config 5 under rocprofv3 again (nm03_bench now ends in cli_exit: exit status 0 expected);
#  * cold-run A/B (wipe passes): create_writers 0/4/8 × wipe by background reaper vs inline unlinks,
#    3 interleaved rounds, then one default bench (cli_wall).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4b; mkdir -p $O
B=build/bin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
for i in 1 2 3; do
  timeout -k 5 60 $B/hip_init_probe >> $O/hip_init.txt 2>&1 || exit 20
  HIP_VISIBLE_DEVICES=0 timeout -k 5 60 $B/hip_init_probe >> $O/hip_init.txt 2>&1 || exit 22
done
T=/tmp/r4vol
$B/nm03_synth --data-root $T/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 30
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 \
  -- $B/nm03_bench --config volume --data-root $T/ --steps 10 --warmup 2 > $O/c5_prof.json 2> $O/c5_prof.err
echo "profiled run exit $?" > $O/c5_prof_status.txt
rm -rf $T
grep -q "exit 0" $O/c5_prof_status.txt || exit 31
A="--steps 40 --warmup 5 --wipe-passes 40 --single-passes 0 --cli-runs 0 --keep-data"
for r in 1 2 3; do
  for arm in "0 inline" "4 reaper" "8 reaper" "4 inline" "0 reaper"; do
    set -- $arm
    echo "round $r cw=$1 wipe=$2" >> $O/cold_ab.jsonl
    timeout -k 10 200 python3 bench.py $A --create-writers $1 --wipe-mode $2 >> $O/cold_ab.jsonl 2>> $O/cold_ab.err || exit 40
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 50
