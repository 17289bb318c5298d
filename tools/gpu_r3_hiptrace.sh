#!/bin/bash
# (gpurun) HIP API + kernel + copy + marker trace of bench.py single passes (no counters), for the
# single-pass latency breakdown (tools/tl_single.py). gpurun_out/r3h/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3h; mkdir -p $O
export NM03_ROCTX=1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d $O/tl -o bench \
  -- python3 bench.py --steps 2 --warmup 1 --single-passes 5 --wipe-passes 0 > $O/tl.log 2>&1 || exit 41
