#!/bin/bash
# (gpurun) Kernel A/B: the working tree's build (build/bin) against a baseline build staged in
# abbase/{bin,lib} (git-ignored; built from the previous commit). GPU tests on the candidate, then
# isolated engine runs (nm03_bench cohort, 1 stream, batch 96, rocprofv3 kernel stats) interleaved
# for 3 rounds, output trees compared, and one 20-step bench of the candidate with kernel stats.
# Usage: bash tools/gpu_ab_kernels.sh <out-name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${1:-ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
D=/tmp/ab_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 11
for r in 1 2 3; do
  LD_LIBRARY_PATH=$PWD/abbase/lib:/opt/rocm/lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base_$r -o k \
    -- abbase/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/ab_base --steps 5 --warmup 1 --streams 1 --batch-size 96 \
    > $O/base_$r.log 2>&1 || exit 12
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cand_$r -o k \
    -- build/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/ab_cand --steps 5 --warmup 1 --streams 1 --batch-size 96 \
    > $O/cand_$r.log 2>&1 || exit 13
done
diff -r /tmp/ab_base /tmp/ab_cand > $O/diff.txt && echo "trees identical" > $O/diff_ok.txt
rm -rf $D /tmp/ab_base /tmp/ab_cand
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bench -o k \
  -- python3 bench.py --steps 20 --warmup 3 --single-passes 0 --cli-runs 0 --wipe-passes 0 > $O/bench.json 2> $O/bench.err || exit 20
