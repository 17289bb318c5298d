#!/bin/bash
# (gpurun) Round 4: tools/gpu_r4_e.sh + _f.sh + _g.sh in one box session (pod congested, boxes flaky).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r4_i.sh || exit 99
bash tools/gpu_r4_e.sh || exit $?
sed -i 's/^timeout -k 10 400 python -u -m pytest.*/true/' tools/gpu_r4_f.sh tools/gpu_r4_g.sh  # tests ran in _e
bash tools/gpu_r4_g.sh || exit $((100 + $?))
bash tools/gpu_r4_f.sh || exit $((150 + $?))
bash tools/gpu_r4_h.sh || exit $((200 + $?))
