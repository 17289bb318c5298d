#!/bin/bash
# (gpurun) Round 4, third call. gpurun_out/r4c/:
#  * GPU test suite (flat label workgroups in the JPEG encoder);
#  * JPEG kernel time with vs without the flat-workgroup path (NM03_PROFILE_VARIANT=jpeg=32 turns
#    only that path off), rocprofv3 kernel stats of 20-step bench runs, 2 interleaved rounds;
#  * cold-run A/B: create_writers 4 / 0, wipe pipeline depth 3 / 2, 3 interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
P="--steps 20 --warmup 3 --single-passes 0 --cli-runs 0 --wipe-passes 0 --keep-data"
for r in 1 2; do
  for v in 0 32; do
    NM03_PROFILE_VARIANT=jpeg=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$r -o k \
      -- python3 bench.py $P > $O/prof_${v}_$r.json 2> $O/prof_${v}_$r.err || exit 20
  done
done
A="--steps 40 --warmup 5 --wipe-passes 40 --single-passes 0 --cli-runs 0 --keep-data"
for r in 1 2 3; do
  for arm in "4 3" "0 3" "4 2"; do
    set -- $arm
    echo "round $r cw=$1 depth=$2" >> $O/cold_ab.jsonl
    timeout -k 10 200 python3 bench.py $A --create-writers $1 --wipe-depth $2 >> $O/cold_ab.jsonl 2>> $O/cold_ab.err || exit 40
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 50
