#!/bin/bash
# Round 6: host thread placement A/B for the headline. The box gives a 16-CPU quota over a whole NUMA node
# (128 logical CPUs); the pool floats over all of them by default. Variants restrict the process's CPU set
# (the engine's partition follows sched_getaffinity) before Python starts: PLACES="name=cpulist ..."
# ("all" = no restriction). → gpurun_out/r6_place/
set -o pipefail
O=gpurun_out/r6_place
mkdir -p $O
export PYTHONUNBUFFERED=1
D=/dev/shm/nm03_bench_data
for r in $(seq ${ROUNDS:-3}); do
  for v in ${PLACES:-all}; do
    name=${v%%=*}; cpus=${v#*=}
    pre=""; [ "$cpus" != "all" ] && pre="taskset -c $cpus"
    timeout -k 10 240 $pre python -u bench.py --keep-data --data-root $D --steps ${STEPS:-3000} --warmup 5 --no-secondary \
      --wipe-passes 0 --single-passes 0 --cli-runs 0 > "$O/bench_${name}_$r.json" 2>> $O/bench.err || exit 1
  done
done
python3 - <<'PY'
import collections, glob, json, statistics
d = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6_place/bench_*_[0-9].json")):
    v = f.split("bench_")[1].rsplit("_", 1)[0]
    j = json.loads(open(f).read().strip().splitlines()[-1])
    d[v].append((j["value"], j["config"]["rank0_process_cpu_ms_per_step"], j["config"]["per_rank"]["threads"]))
for v, rows in d.items():
    print(f"{v:10s} slices/s median {statistics.median(r[0] for r in rows):9.0f} range {min(r[0] for r in rows):.0f}-"
          f"{max(r[0] for r in rows):.0f} cpu/step {statistics.median(r[1] for r in rows):.2f} threads {rows[0][2]}")
PY
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
