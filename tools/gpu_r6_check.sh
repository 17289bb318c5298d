#!/bin/bash
# Round 6 box call: the GPU suite, a symbolised CPU profile of the headline's steady state (the
# binary that ran is the one symbolised, on the box), and an interleaved A/B of HIP/ROCr runtime
# knobs against the runtime thread that burns a CPU in ioctl (profiles/r6/cpu_profile/).
# Usage: gpurun -- 'bash tools/gpu_r6_check.sh [tests|prof|knobs]...'  → gpurun_out/r6_check/
#        KNOBS="base A=1 B=0" selects the knob variants.
set -o pipefail
O=gpurun_out/r6_check
mkdir -p $O
export PYTHONUNBUFFERED=1
steps="${*:-tests prof knobs}"
B="python -u bench.py --keep-data"
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
      tail -3 $O/pytest_gpu.log
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
      ;;
    prof)
      timeout -k 10 240 $B --steps 4000 --warmup 5 --no-secondary --wipe-passes 0 --single-passes 0 --cli-runs 0 \
        --cpu-profile $O/cpu > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
      timeout -k 10 600 python tools/cpu_profile.py $O/cpu.rank0 --top 40 --json $O/cpu_profile.json \
        > $O/cpu_profile.txt 2>&1 || exit 1
      head -60 $O/cpu_profile.txt
      ;;
    knobs)
      for r in 1 2; do
        for v in ${KNOBS:-base HSA_ENABLE_INTERRUPT=0 ROC_ACTIVE_WAIT_TIMEOUT=0 ROC_SIGNAL_POOL_SIZE=64}; do
          e=""; [ "$v" != base ] && e="$v"
          timeout -k 10 240 env $e $B --steps 2000 --warmup 5 --no-secondary --wipe-passes 0 --single-passes 0 \
            --cli-runs 0 > $O/knob_${v}_$r.json 2>> $O/knobs.err || exit 1
        done
      done
      ;;
  esac
done
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
