#!/bin/bash
# (gpurun) First-use costs in a cold CLI process: engine run times of repetition 1 vs 2 (NM03_LOG=info),
# with lazy (default) and eager code-object loading, and eager slots.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out/first_run.txt; : > $O
D=/dev/shm/nm03_fr_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2 3; do
  for v in "" "HIP_ENABLE_DEFERRED_LOADING=0" "NM03_EAGER_SLOTS=1"; do
    echo "== [$v] run $r" >> $O
    (cd /tmp && env $v NM03_LOG=info timeout -k 10 60 $GRAFT_REPO_ROOT/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/nm03_fr_out --json /tmp/fr.json --quiet --repeat 2 2>&1 | grep -E "run:|set-up" >> $GRAFT_REPO_ROOT/$O) || exit 3
    python3 -c "import json; d=json.load(open('/tmp/fr.json')); print({k: d[k] for k in ('hip_init_s','engine_ctor_s','engine_setup_s','processing_wall_s')})" >> $O
  done
done
