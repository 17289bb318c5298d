#!/bin/bash
# Round check (gpurun): pytest -m gpu, 1-GPU bench, rocprofv3 kernel stats of bench.py, smoke(). Logs in gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress_round.txt
echo "start $(date)" > $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 31
echo "pytest ok $(date)" >> $P
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 32
echo "smoke ok $(date)" >> $P
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 33
timeout -k 10 300 python bench.py > gpurun_out/bench_b.log 2>&1 || exit 34
echo "bench ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 20 --warmup 2 > gpurun_out/prof_bench.log 2>&1 || exit 35
echo "done $(date)" >> $P
