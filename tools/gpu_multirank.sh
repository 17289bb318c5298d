#!/bin/bash
# Multi-rank checks on a one-GPU box (gpurun): the GPU test-suite (incl. the N-rank CLI and bench
# tests), then bench.py at 1 rank, 2 and 4 self-launched ranks sharing device 0 (host comm), and
# the torchrun launch form the driver uses for N > 1. Logs in gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress_multirank.txt
echo "start $(date)" > $P
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || exit 31
echo "pytest ok $(date)" >> $P
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 || exit 32
echo "bench1 ok $(date)" >> $P
export NM03_DEVICE_OVERRIDE=0
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench2.log 2>&1 || exit 33
echo "bench2 ok $(date)" >> $P
timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 2 > gpurun_out/bench4.log 2>&1 || exit 34
echo "bench4 ok $(date)" >> $P
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench2_torchrun.log 2>&1 || exit 35
echo "done $(date)" >> $P
ls /dev/shm > gpurun_out/shm_after.txt
