#!/bin/bash
# Interleaved A/B of bench.py under environment variants (gpurun): ROUNDS × each variant, JSON
# lines to gpurun_out/ab.jsonl, medians to gpurun_out/ab.txt. Variants are "NAME=VAL,NAME2=VAL" or "-".
#   bash tools/ab_bench.sh 4 "-" "NM03_JPEG_LDS_PAD=10000"
# AB_ROOT=<dir> in a variant runs <dir>/bench.py (e.g. a build of an older commit);
# AB_ARGS="--batch-size 48 --streams 8" passes bench.py flags.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq $rounds); do
  for v in "$@"; do
    envs=()
    [ "$v" != "-" ] && IFS=',' read -ra envs <<< "$v"
    script=bench.py
    for e in "${envs[@]}"; do [ "${e%%=*}" = "AB_ROOT" ] && script="${e#*=}/bench.py"; done
    args=()
    for e in "${envs[@]}"; do [ "${e%%=*}" = "AB_ARGS" ] && read -ra args <<< "${e#*=}"; done
    line=$(env "${envs[@]}" timeout -k 10 200 python $script --steps ${STEPS:-100} --warmup 5 "${args[@]}" 2>/dev/null | grep metric) || exit 7
    echo "{\"variant\": \"$v\", \"round\": $r, \"bench\": $line}" >> gpurun_out/ab.jsonl
  done
done
python3 - <<'PY' > gpurun_out/ab.txt
import json, statistics, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab.jsonl"):
    j = json.loads(l); d[j["variant"]].append(j["bench"]["value"])
for k, v in d.items():
    print(f"{k:40s} median {statistics.median(v):10.0f}  runs {[round(x) for x in v]}")
PY
