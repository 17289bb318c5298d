#!/bin/bash
# Batch-wait A/B (gpurun): current tree (chunked adaptive sleep) vs abprev/ (one long sleep), interleaved:
# 1-rank bench ×4 and 2 ranks sharing the GPU under torchrun ×2. Take abprev/ out of .gpurunignore.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/wab; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > $O/cur_$i.log 2>&1 || exit 41
  (cd abprev && timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary > ../$O/prev_$i.log 2>&1) || exit 42
done
export NM03_DEVICE_OVERRIDE=0
for i in 1 2; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29700 + i)) bench.py --gpus 2 --steps 20 --warmup 3 --no-secondary > $O/cur_tr_$i.log 2>&1 || exit 43
  (cd abprev && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29710 + i)) bench.py --gpus 2 --steps 20 --warmup 3 --no-secondary > ../$O/prev_tr_$i.log 2>&1) || exit 44
done
