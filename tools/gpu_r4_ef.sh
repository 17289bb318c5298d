#!/bin/bash
# (gpurun) Round 4: tools/gpu_r4_e.sh + tools/gpu_r4_f.sh in one box session (pod congested).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r4_e.sh || exit $?
sed -i 's/^timeout -k 10 400 python -u -m pytest.*/true/' tools/gpu_r4_f.sh  # tests already ran in _e
bash tools/gpu_r4_f.sh || exit $((100 + $?))
