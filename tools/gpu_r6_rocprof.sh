#!/bin/bash
# Round 6: rocprofv3 --kernel-trace --stats of the headline bench on the final tree (per-kernel table).
# → gpurun_out/r6_rocprof/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6_rocprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof -o bench -- \
  python3 -u bench.py --steps ${STEPS:-500} --warmup 5 --no-secondary --wipe-passes 0 --single-passes 0 --cli-runs 0 \
  > $O/bench.json 2> $O/bench.err || exit 1
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) > $O/kstats.txt 2>&1 || true
python3 tools/timeline.py --window $O/prof > $O/timeline.txt 2>&1 || exit 2
cat $O/kstats.txt $O/timeline.txt
find $O/prof -name '*trace.csv' -size +20M -delete
echo done
