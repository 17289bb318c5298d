#!/bin/bash
# Multi-rank rehearsal on a one-GPU box (gpurun): bench.py under torchrun with 2 and 4 ranks that
# all share device 0, collectives over gloo (RCCL refuses two ranks per device). Exercises the
# plan broadcast, sharding, barriers, max/sum reductions and the rank-0 JSON line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export NM03_DIST_BACKEND=gloo NM03_DEVICE_OVERRIDE=0
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 1 --threads $((16 / n)) --keep-output \
    > gpurun_out/multirank_$n.log 2>&1 || exit $((90 + n))
  find /dev/shm/nm03_bench_out -name "*.jpg" | wc -l > gpurun_out/multirank_${n}_files.txt
  ls /dev/shm/nm03_bench_out >> gpurun_out/multirank_${n}_files.txt; rm -rf /dev/shm/nm03_bench_out
done
ls /dev/shm > gpurun_out/shm_after.txt
