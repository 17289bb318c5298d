#!/bin/bash
# Round 6: wipe-each-pass figure (config.wipe_each_pass, 200 passes) under bench.py argument variants
# (VARIANTS ';'-separated, "-" = defaults), interleaved rounds. → gpurun_out/r6_wipe/
set -o pipefail
O=gpurun_out/r6_wipe
mkdir -p $O
export PYTHONUNBUFFERED=1
D=/dev/shm/nm03_bench_data
IFS=';' read -r -a VARS <<< "${VARIANTS:--}"
for r in $(seq ${ROUNDS:-4}); do
  for i in "${!VARS[@]}"; do
    a=""; [ "${VARS[$i]}" != "-" ] && a="${VARS[$i]}"
    timeout -k 10 240 python -u bench.py --keep-data --data-root $D --steps 20 --warmup 5 --no-secondary --single-passes 0 \
      --cli-runs 0 --wipe-passes ${PASSES:-200} $a > "$O/wipe_v${i}_$r.json" 2>> $O/bench.err || exit 1
  done
done
for i in "${!VARS[@]}"; do echo "v$i = ${VARS[$i]}"; done
python3 - <<'PY'
import collections, glob, json, statistics
d = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6_wipe/wipe_v*_[0-9].json")):
    v = f.split("wipe_")[1].rsplit("_", 1)[0]
    w = json.loads(open(f).read().strip().splitlines()[-1])["config"]["wipe_each_pass"]
    d[v].append((w["value"], w["rank0_process_cpu_ms_per_step"]))
for v, rows in sorted(d.items()):
    print(f"{v}: wipe median {statistics.median(r[0] for r in rows):9.0f} range {min(r[0] for r in rows):.0f}-"
          f"{max(r[0] for r in rows):.0f} cpu/pass {statistics.median(r[1] for r in rows):.1f} ms")
PY
rm -rf /dev/shm/nm03_bench_data /dev/shm/nm03_bench_out
echo done
