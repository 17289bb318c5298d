#!/bin/bash
# (gpurun) Round 4: GPU tests, then the cold CLI's start-up split (NM03_LOG=info: engine set-up by
# phase) and 10 exact CLI walls on the bench cohort. gpurun_out/r4cli/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4cli; mkdir -p $O
B=build/bin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
D=/dev/shm/r4cli_data
$B/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for i in 1 2 3; do
  NM03_LOG=info timeout -k 10 60 $B/img_processing_parallel --gpus 1 --data-root $D/ --out /dev/shm/r4cli_out --quiet \
    --json $O/cli_$i.json > $O/cli_$i.log 2>&1 || exit 12
done
timeout -k 10 300 python3 tools/cli_wall.py "$B" "$D/" 10 img_processing_parallel > $O/cli_wall.jsonl || exit 13
rm -rf $D /dev/shm/r4cli_out
