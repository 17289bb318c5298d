#!/bin/bash
# Engine configuration sweep (gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep_engine.py --steps ${STEPS:-10} --repeat ${REPEAT:-1} --grid "${1:-24,32,48,64,96:4,6,8,12:16}" > gpurun_out/sweep.jsonl 2>gpurun_out/sweep.err || exit 81
