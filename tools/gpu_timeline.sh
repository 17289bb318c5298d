#!/bin/bash
# Timeline run (gpurun): kernel + memory-copy + marker traces of bench.py (no counters), then
# tools/timeline.py summary into gpurun_out/timeline.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export NM03_ROCTX=1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d gpurun_out/tl -o bench \
  -- python3 bench.py --steps 3 --warmup 1 "$@" > gpurun_out/tl.log 2>&1 || exit 41
python3 tools/timeline.py gpurun_out/tl -v > gpurun_out/timeline.txt 2>&1 || exit 42
