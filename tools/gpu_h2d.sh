#!/bin/bash
# H2D probe + current timeline (gpurun). Results in gpurun_out/h2d.txt and gpurun_out/timeline.txt.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 build/h2d_probe > gpurun_out/h2d.txt 2>&1 || exit 21
HSA_ENABLE_SDMA=0 timeout -k 10 120 build/h2d_probe > gpurun_out/h2d_nosdma.txt 2>&1 || exit 22
bash tools/gpu_timeline.sh || exit 23
