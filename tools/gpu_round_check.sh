#!/bin/bash
# (gpurun) Round-5 check: the GPU test suite, then the cold-CLI anatomy of the new start-up
# (default HW queues vs GPU_MAX_HW_QUEUES=2) and a warm --repeat throughput for both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5check}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || exit 1
D=/dev/shm/r5c_data
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 3
for rep in 1 2 3; do
  for q in 4 2; do
    (cd /tmp && GPU_MAX_HW_QUEUES=$q NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $R/build/bin/img_processing_parallel \
      --data-root $D/ --out /dev/shm/r5c_out --quiet --json $R/$O/cli_q${q}_$rep.json > $R/$O/cli_q${q}_$rep.log 2>&1) || exit 4
  done
done
for q in 4 2; do
  (cd /tmp && GPU_MAX_HW_QUEUES=$q timeout -k 10 60 $R/build/bin/img_processing_parallel \
    --data-root $D/ --out /dev/shm/r5c_out --quiet --repeat 30 --json $R/$O/rep30_q$q.json > $R/$O/rep30_q$q.log 2>&1) || exit 5
done
rm -rf $D /dev/shm/r5c_out
echo done
