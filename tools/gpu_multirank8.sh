#!/bin/bash
# 8-rank rehearsal on a one-GPU box (gpurun): bench.py with 8 self-launched ranks and under
# torch.distributed.run --nproc-per-node 8 (the driver's N=8 launch form), every rank on device 0
# (NM03_DEVICE_OVERRIDE=0, host comm: RCCL refuses two ranks on one device). Logs in gpurun_out/mr8/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mr8; mkdir -p $O
echo "start $(date)" > $O/progress.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench1.log 2>&1 || exit 31
echo "bench1 ok $(date)" >> $O/progress.txt
export NM03_DEVICE_OVERRIDE=0
timeout -k 10 400 python bench.py --gpus 8 --steps 10 --warmup 2 > $O/bench8.log 2>&1 || exit 32
echo "bench8 ok $(date)" >> $O/progress.txt
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29613 bench.py --gpus 8 --steps 10 --warmup 2 > $O/bench8_torchrun.log 2>&1 || exit 33
echo "done $(date)" >> $O/progress.txt
ls /dev/shm > $O/shm_after.txt
