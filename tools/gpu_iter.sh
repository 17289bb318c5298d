#!/bin/bash
# Iteration run (gpurun): pytest -m gpu → bench → rocprofv3 kernel stats of the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress_iter.txt
echo "start $(date)" > $P
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> $P
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || exit 31
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --graphs > gpurun_out/bench_graphs.log 2>&1 || exit 35
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench2.log 2>&1 || exit 36
echo "bench ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_iter -o bench -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_iter.log 2>&1 || exit 32
echo "done $(date)" >> $P
build/bin/nm03_synth --data-root /tmp/vol/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 33
timeout -k 10 300 build/bin/nm03_bench --config volume --data-root /tmp/vol/ --steps 3 --warmup 1 > gpurun_out/volume.log 2>&1 || exit 34
echo "volume ok $(date)" >> $P
