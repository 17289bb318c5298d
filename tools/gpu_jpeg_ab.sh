#!/bin/bash
# A/B of the JPEG encoder against the tree in abprev/ (git worktree, built with build.py):
# isolated kernel profile (1 stream, batch 64) of both, interleaved, plus concurrent (6 streams).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/ab
D=/tmp/kprof_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for i in 1 2; do
  for t in new old; do
    B=build/bin/nm03_bench; [ $t = old ] && B=abprev/build/bin/nm03_bench
    for st in 1 6; do
      timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/${t}_s${st}_$i -o run \
        -- $B --config cohort --data-root $D/ --steps 5 --warmup 1 --streams $st --batch-size 64 \
        > gpurun_out/ab/${t}_s${st}_$i.log 2>&1 || exit 4
      python3 tools/kstats.py gpurun_out/ab/${t}_s${st}_$i/run_kernel_stats.csv > gpurun_out/ab/${t}_s${st}_$i.txt
    done
  done
done
