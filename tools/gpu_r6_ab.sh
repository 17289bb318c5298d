#!/bin/bash
# Round 6: interleaved A/B of the round-start build (abprev/: its bench.py, package and CLI) against
# this tree — headline bench (host CPU per step) and cold CLI walls — plus a symbolised CPU profile of
# this tree. Usage: gpurun -- 'bash tools/gpu_r6_ab.sh [bench|cold|prof|tests|preload|timeline]...' → gpurun_out/r6_ab/
set -o pipefail
O=gpurun_out/r6_ab
mkdir -p $O
export PYTHONUNBUFFERED=1
steps="${*:-bench cold prof}"
D=/dev/shm/nm03_bench_data
for s in $steps; do
  case $s in
    bench)
      for r in $(seq ${ROUNDS_B:-4}); do
        for v in ${VARIANTS:-old new}; do
          # "old" = abprev/, "new" = this tree, "new:VAR=VAL" = this tree with an environment variant
          # "new@--flag=value" = this tree with an extra bench.py argument
          S=bench.py; e=""; a=""
          [ $v = old ] && S=abprev/bench.py
          case $v in new:*) e="${v#new:}";; new@*) a="${v#new@}";; esac
          timeout -k 10 240 env $e python -u $S $a --keep-data --data-root $D --steps ${STEPS:-2000} --warmup 5 --no-secondary \
            --wipe-passes 0 --single-passes 0 --cli-runs 0 > "$O/bench_${v}_$r.json" 2>> $O/bench.err || exit 1
        done
      done
      ;;
    cold)
      C=/dev/shm/nm03_cold_cohort
      [ -d $C ] || build/bin/nm03_synth --data-root $C/ --threads 16 > /dev/null || exit 1
      timeout -k 10 600 python -u tools/cold_ab.py $C/ ${ROUNDS:-12} ${COLD_VARIANTS:-old=abprev/bin:abprev/nm03_capstone_project_amd/lib new=build/bin} \
        > $O/cold_ab.jsonl 2> $O/cold_ab.err || exit 1
      rm -rf $C /dev/shm/cold_ab_*
      cat $O/cold_ab.jsonl | cut -c1-400
      ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
        > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
      tail -2 $O/pytest_gpu.log
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || exit 1
      ;;
    preload)
      C=/dev/shm/nm03_cold_cohort
      [ -d $C ] || build/bin/nm03_synth --data-root $C/ --threads 16 > /dev/null || exit 1
      for k in 1 2 3; do
        for t in 1 2; do
          echo "== NM03_PRELOAD_TRACE=$t run $k" >> $O/preload.txt
          NM03_PRELOAD_TRACE=$t timeout -k 10 60 build/bin/img_processing_parallel --data-root $C/ --out /dev/shm/pl_out --quiet \
            --json $O/preload_${t}_$k.json > /dev/null 2>> $O/preload.txt || exit 1
        done
      done
      cat $O/preload.txt
      rm -rf $C /dev/shm/pl_out
      ;;
    timeline)
      # kernel + copy trace of the pipelined steady state (no counters): union-busy of kernels and H2D
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o bench -- \
        python3 -u bench.py --keep-data --data-root $D --steps ${TL_STEPS:-1000} --warmup 5 --no-secondary --wipe-passes 0 \
        --single-passes 0 --cli-runs 0 $TL_ARGS > $O/bench_tl.json 2> $O/bench_tl.err || exit 1
      python3 tools/timeline.py --window $O/tl > $O/timeline.txt 2>&1 || exit 1
      cat $O/timeline.txt
      find $O/tl -name '*.csv' -size +20M -delete
      ;;
    prof)
      timeout -k 10 240 python -u bench.py --keep-data --data-root $D --steps 4000 --warmup 5 --no-secondary --wipe-passes 0 \
        --single-passes 0 --cli-runs 0 --cpu-profile $O/cpu > $O/bench_prof.json 2> $O/bench_prof.err || exit 1
      timeout -k 10 600 python tools/cpu_profile.py $O/cpu.rank0 --top 40 --chains __lll_lock --json $O/cpu_profile.json \
        > $O/cpu_profile.txt 2>&1 || exit 1
      head -45 $O/cpu_profile.txt | cut -c1-200
      ;;
  esac
done
python3 - <<'PY'
import glob, json, statistics, collections
d = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6_ab/bench_*_[0-9].json")):
    v = f.split("bench_")[1].rsplit("_", 1)[0]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    c = j["config"]
    d[v].append((j["value"], c["rank0_process_cpu_ms_per_step"], c["rank0_thread_cpu_ms_per_step"]))
for v, rows in d.items():
    print(v, "value median", round(statistics.median(r[0] for r in rows)), "cpu/step median",
          round(statistics.median(r[1] for r in rows), 3), [r[2] for r in rows])
PY
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
