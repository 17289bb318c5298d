#!/bin/bash
# (gpurun) Does per-rank start-up serialise in the driver? k = 1/2/4/8 independent cold
# img_processing_parallel processes started at once on device 0 (each its own output tree), then the
# launcher form: one --gpus k run whose k ranks share device 0 (NM03_DEVICE_OVERRIDE=0, host comm).
# Per process: hipInit, streams, engine set-up and processing from its --json; per batch: the wall
# of the slowest process.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-startup}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
D=/dev/shm/su_data
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for rep in 1 2; do
  for k in 1 2 4 8; do
    s=$(date +%s.%N)
    pids=()
    for i in $(seq 1 $k); do
      (cd /tmp && timeout -k 10 120 $R/build/bin/img_processing_parallel --gpus 1 --data-root $D/ --out /dev/shm/su_out_$i \
        --quiet --threads 2 --json $R/$O/indep_k${k}_r${rep}_$i.json > /dev/null 2>&1) &
      pids+=($!)
    done
    rc=0
    for p in "${pids[@]}"; do wait $p || rc=$?; done
    e=$(date +%s.%N)
    echo "indep k=$k rep=$rep wall_s $(python3 -c "print(round($e-$s,4))") rc=$rc" >> $O/walls.txt
    [ $rc = 0 ] || exit 2
  done
  for k in 1 2 4 8; do
    s=$(date +%s.%N)
    (cd /tmp && NM03_DEVICE_OVERRIDE=0 timeout -k 10 120 $R/build/bin/img_processing_parallel --gpus $k --data-root $D/ \
      --out /dev/shm/su_out_l --quiet --json $R/$O/launch_k${k}_r${rep}.json > /dev/null 2>&1) || exit 3
    e=$(date +%s.%N)
    echo "launch k=$k rep=$rep wall_s $(python3 -c "print(round($e-$s,4))")" >> $O/walls.txt
  done
done
rm -rf $D /dev/shm/su_out_*
python3 - "$O" <<'PY' > $O/summary.txt
import glob, json, os, sys, collections
o = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(o, "indep_k*_r*_*.json"))):
    k = int(os.path.basename(f).split("_")[1][1:])
    d = json.load(open(f))
    rows[k].append({x: round(d[x] * 1e3, 1) for x in ("hip_init_s", "streams_s", "engine_setup_s", "processing_wall_s")})
for k in sorted(rows):
    med = {x: sorted(r[x] for r in rows[k])[len(rows[k]) // 2] for x in rows[k][0]}
    mx = {x: max(r[x] for r in rows[k]) for x in rows[k][0]}
    print(f"independent k={k}: median {med}  max {mx}")
for f in sorted(glob.glob(os.path.join(o, "launch_k*_r*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), {x: d.get(x) for x in ("hip_init_s", "streams_s", "engine_setup_s", "processing_wall_s", "wall_s")})
print(open(os.path.join(o, "walls.txt")).read())
PY
echo done
