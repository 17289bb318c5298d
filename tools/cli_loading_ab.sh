#!/bin/bash
# (gpurun) Cold CLI wall: deferred (default) vs eager code-object loading, interleaved 6×.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out; O=gpurun_out/cli_loading.txt; : > $O
D=/dev/shm/nm03_cl_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2 3 4 5 6; do
  for v in 1 0; do
    s=$(date +%s.%N)
    (cd /tmp && HIP_ENABLE_DEFERRED_LOADING=$v timeout -k 10 60 $GRAFT_REPO_ROOT/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/nm03_cl_out --json /tmp/cl.json --quiet > /dev/null 2>&1) || exit 3
    e=$(date +%s.%N)
    python3 -c "
import json
d = json.load(open('/tmp/cl.json'))
print(f'[deferred={$v}] wall {($e - $s) * 1e3:.1f} ms; hip_init {1e3*d[\"hip_init_s\"]:.1f}, ctor {1e3*d[\"engine_ctor_s\"]:.1f}, processing {1e3*d[\"processing_wall_s\"]:.1f} ms')" >> $O || exit 4
  done
done
