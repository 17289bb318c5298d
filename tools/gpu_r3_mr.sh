#!/bin/bash
# (gpurun) Multi-rank rehearsal on one GPU (NM03_DEVICE_OVERRIDE=0, host comm): bench.py --gpus 2 and
# --gpus 8 (self-launched) and --gpus 8 under torch.distributed.run. gpurun_out/r3mr/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3mr; mkdir -p $O
export NM03_DEVICE_OVERRIDE=0
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 3 --single-passes 3 > $O/bench2.log 2>&1 || exit 31
timeout -k 10 400 python bench.py --gpus 8 --steps 10 --warmup 2 --single-passes 3 > $O/bench8.log 2>&1 || exit 32
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29615 bench.py --gpus 8 --steps 10 --warmup 2 --single-passes 3 > $O/bench8_torchrun.log 2>&1 || exit 33
ls /dev/shm > $O/shm_after.txt
