#!/bin/bash
# (gpurun) FDCT MFMA microbenchmark, GPU tests, kernel stats of the bench, then the L3-pinning A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/combo
P=gpurun_out/combo/progress.txt
echo "start $(date)" > $P
timeout -k 10 120 build/bin/fdct_mfma_bench 1048576 16 > gpurun_out/combo/fdct_mfma.txt 2>&1; echo "fdct rc=$?" >> $P
timeout -k 10 120 build/bin/fdct_mfma_bench 262144 64 >> gpurun_out/combo/fdct_mfma.txt 2>&1; echo "fdct2 rc=$?" >> $P
bash tools/gpu_tests.sh || exit 31
echo "pytest ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/combo/prof -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 3 > gpurun_out/combo/prof_bench.log 2>&1 || exit 32
echo "prof ok $(date)" >> $P
bash tools/gpu_pin_l3.sh
