#!/bin/bash
# (gpurun) run_single read-back change: GPU tests using run_single / test_pipeline, then config 1
# (nm03_bench --config single) 3 times. gpurun_out/r3c1/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3c1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "single or signed or test_pipeline or engine_large" > $O/pytest.log 2>&1 || exit 31
T=/tmp/r3c1; build/bin/nm03_synth --data-root $T/ --threads 16 > /dev/null || exit 41
for i in 1 2 3; do
  timeout -k 10 120 build/bin/nm03_bench --config single --data-root $T/ --steps 50 --warmup 5 >> $O/c1.txt 2>&1 || exit 42
done
rm -rf $T
