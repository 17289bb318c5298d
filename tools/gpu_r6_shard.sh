#!/bin/bash
# Round 6: per-GPU rate of config 3's strong-scaling shard at the driver's step count. One GPU runs
# rank 0's share of an N-rank job (bench.py --emulate-shard-of N: 465/N slices per pass) with the
# driver's --steps/--warmup, interleaved over N (and over VARIANTS, ';'-separated extra bench.py
# arguments, "-" = none), so the round-end SCALE run's per-rank step latency (pipeline fill/drain
# inside a short timed region) is known before it happens.
# Usage: gpurun -- 'bash tools/gpu_r6_shard.sh' → gpurun_out/r6_shard/ (OUT=dir to change)
set -o pipefail
O=${OUT:-gpurun_out/r6_shard}
mkdir -p $O
export PYTHONUNBUFFERED=1
D=/dev/shm/nm03_bench_data
IFS=';' read -r -a VARS <<< "${VARIANTS:--}"
for r in $(seq ${ROUNDS:-3}); do
  for i in "${!VARS[@]}"; do
    v=${VARS[$i]}
    a=(); e=()
    if [ "$v" != "-" ]; then  # leading NAME=VAL words go to the environment (e.g. LD_LIBRARY_PATH=<older lib dir>)
      for w in $v; do if [[ ${#a[@]} -eq 0 && "$w" == *=* && "$w" != --* ]]; then e+=("$w"); else a+=("$w"); fi; done
    fi
    for n in ${SHARDS:-1 2 4 8}; do
      for st in ${STEPS:-20 200}; do
        timeout -k 10 240 env "${e[@]}" python -u bench.py --keep-data --data-root $D --steps $st --warmup 5 --no-secondary \
          --wipe-passes 0 --single-passes 0 --cli-runs 0 --emulate-shard-of $n "${a[@]}" \
          > "$O/shard${n}_steps${st}_v${i}_$r.json" 2>> $O/bench.err || exit 1
      done
    done
  done
done
for i in "${!VARS[@]}"; do echo "v$i = ${VARS[$i]}"; done
OUT=$O python3 - <<'PY'
import collections, glob, json, os, statistics
d = collections.defaultdict(list)
for f in sorted(glob.glob(os.environ["OUT"] + "/shard*_steps*_[0-9].json")):
    k = f.split("/")[-1].rsplit("_", 1)[0]
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    d[k].append((j["value"], j["ms_per_step"]))
for k in sorted(d, key=lambda s: (int(s[5:].split("_")[0]), s)):
    v = [x[0] for x in d[k]]
    print(f"{k:24s} slices/s median {statistics.median(v):10.0f}  range {min(v):.0f}-{max(v):.0f}  "
          f"ms/step {statistics.median(x[1] for x in d[k]):.3f}")
PY
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
