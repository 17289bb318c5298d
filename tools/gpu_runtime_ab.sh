#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/rab_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2; do
timeout -k 10 120 python tools/runtime_ab.py $D/ >> gpurun_out/rab.jsonl 2>>gpurun_out/rab.err || exit 2
timeout -k 10 120 python tools/runtime_ab.py $D/ torch >> gpurun_out/rab.jsonl 2>>gpurun_out/rab.err || exit 3
timeout -k 10 120 build/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/rab_o --steps 20 --warmup 3 >> gpurun_out/rab.jsonl || exit 4
done
