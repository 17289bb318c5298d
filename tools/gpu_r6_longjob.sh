#!/bin/bash
# Round 6: start-up phases of a long CLI job (> 4096 slices per rank: DMA copies, every slot its own stream) vs
# the short cold job, interleaved. → gpurun_out/r6_long/
set -o pipefail
O=gpurun_out/r6_long
mkdir -p $O
C=/dev/shm/nm03_long_cohort
build/bin/nm03_synth --data-root $C/ --threads 16 > /dev/null || exit 1
for r in $(seq ${ROUNDS:-3}); do
  for v in short long; do
    a=""; [ $v = long ] && a="--repeat 10"
    timeout -k 10 120 build/bin/img_processing_parallel --data-root $C/ --out /dev/shm/long_out --quiet $a \
      --json $O/${v}_$r.json > /dev/null 2> $O/${v}_$r.err || exit 2
    python3 -c "
import json; j = json.load(open('$O/${v}_$r.json'))
print('$v $r', {k: (round(j[k] * 1e3, 2) if isinstance(j[k], float) else j[k]) for k in ('copy_engine', 'shared_stream', 'hip_init_s', 'kernel_load_s', 'streams_s', 'engine_ctor_s', 'engine_setup_s', 'engine_wait_s', 'processing_wall_s', 'wall_s')})"
  done
done
rm -rf $C /dev/shm/long_out
echo done
