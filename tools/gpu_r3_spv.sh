#!/bin/bash
# (gpurun) Small-batch inline upload on the final tree: full GPU test suite, then a HIP trace of
# single passes (tools/tl_single.py). gpurun_out/r3spv/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3spv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 31
export NM03_ROCTX=1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d $O/tl -o bench \
  -- python3 bench.py --steps 2 --warmup 1 --single-passes 5 --wipe-passes 0 > $O/tl.log 2>&1 || exit 41
