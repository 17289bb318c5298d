#!/bin/bash
# (gpurun) Round 4, sixth call. gpurun_out/r4f/:
#  * GPU tests incl. bar_upload byte identity;
#  * A/B (interleaved, 3 rounds): pixels uploaded by SDMA from pinned host memory (default) vs
#    written by the loaders into VRAM through the large BAR (--bar-upload): headline, host CPU per
#    step, loader CPU per slice, H2D time;
#  * cold CLI start-up detail: img_processing_parallel with NM03_LOG=info (engine set-up split).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4f; mkdir -p $O
B=build/bin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
A="--steps 60 --warmup 5 --wipe-passes 0 --single-passes 0 --cli-runs 0 --keep-data"
for r in 1 2 3; do
  for arm in "" "--bar-upload"; do
    echo "round $r arm=${arm:-sdma}" >> $O/bar_ab.jsonl
    timeout -k 10 200 python3 bench.py $A $arm >> $O/bar_ab.jsonl 2>> $O/bar_ab.err || exit 20
  done
done
D=/dev/shm/nm03_bench_data-node1; [ -d $D ] || D=/dev/shm/nm03_bench_data
for i in 1 2 3; do
  NM03_LOG=info timeout -k 10 60 $B/img_processing_parallel --gpus 1 --data-root $D/ --out /tmp/r4f_cli --quiet \
    --json $O/cli_$i.json > $O/cli_$i.log 2>&1 || exit 30
done
rm -rf /tmp/r4f_cli /dev/shm/nm03_bench_data*
