#!/bin/bash
# Round 6, first box call: the driver's default bench record, a CPU sampling profile of the
# headline's steady state (bench.py --cpu-profile, cpu_sampler.h) and the wipe-each-pass figure at
# 20 vs 150 passes, interleaved (builder-box vs driver-box gap).
# Usage: gpurun -- 'bash tools/gpu_r6_profile.sh'   → gpurun_out/r6_profile/
set -o pipefail
O=gpurun_out/r6_profile
mkdir -p $O
export PYTHONUNBUFFERED=1
B="python -u bench.py --keep-data"
timeout -k 10 240 $B --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 240 $B --steps 4000 --warmup 5 --no-secondary --wipe-passes 0 --single-passes 0 --cli-runs 0 \
  --cpu-profile $O/cpu > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
for r in 1 2 3; do
  for w in 20 150; do
    timeout -k 10 240 $B --steps 20 --warmup 5 --no-secondary --single-passes 0 --cli-runs 0 --wipe-passes $w \
      > $O/wipe_${w}_$r.json 2>> $O/wipe.err || exit 1
  done
done
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
