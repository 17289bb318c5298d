#!/bin/bash
# (gpurun) Round check of the tree: the GPU test suite, the driver's smoke(), the default bench.py
# record, and interleaved cold CLIs with the default copy path (shader copies for this short job) and
# with the DMA engines. Every step under its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-roundcheck}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
RUNS=${RUNS:-7} VARIANTS="-;ARGS=--copy-engine sdma" bash tools/gpu_cold_cli.sh ${1:-roundcheck}/cold || exit 4
echo done
