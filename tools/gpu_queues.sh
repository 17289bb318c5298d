#!/bin/bash
# (gpurun) HIP stream / HW-queue creation cost at start-up (tools/queue_probe.cpp), and the cold CLI
# with fewer HW queues.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5queues}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
for rep in 1 2; do
  for q in 1 2 4; do
    for cfg in "5 1" "5 5" "2 1"; do
      GPU_MAX_HW_QUEUES=$q timeout -k 5 60 build/bin/queue_probe $cfg >> $O/probe.txt 2>&1 || exit 2
    done
  done
done
D=/dev/shm/r5q_data
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 3
for rep in 1 2 3; do
  for q in 1 2 4; do
    (cd /tmp && GPU_MAX_HW_QUEUES=$q NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $R/build/bin/img_processing_parallel \
      --data-root $D/ --out /dev/shm/r5q_out --quiet --json $R/$O/cli_q${q}_$rep.json > $R/$O/cli_q${q}_$rep.log 2>&1) || exit 4
  done
done
rm -rf $D /dev/shm/r5q_out
echo done
