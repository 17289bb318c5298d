#!/bin/bash
# Loader A/B with the batched unmap (one MAP_FIXED PROT_NONE remap of the slot's range per batch,
# instead of one munmap per file as in profiles/iter6/mapped_load_ab.txt): staged (default) vs
# mapped, 4 interleaved bench.py pairs. gpurun_out/mapped2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/mapped2; mkdir -p $O
for i in 1 2 3 4; do
  for mode in staged mapped; do
    NM03_LOAD_MODE=$mode timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 \
      > $O/${mode}_$i.log 2>&1 || exit 40
    echo "$mode $i $(grep -o '"value": [0-9.]*' $O/${mode}_$i.log | head -1) $(grep -o '"load_cpu_s": [0-9.]*' $O/${mode}_$i.log | head -1)" >> $O/summary.txt
  done
done
