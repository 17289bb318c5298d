#!/bin/bash
# (gpurun) Final-tree check of the late round-3 session: smoke, GPU tests, 3 bench runs, kernel stats
# of one, and a 2-rank rehearsal on the one GPU (host comm). gpurun_out/r3f2/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3f2; mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit 30
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 31
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py > $O/bench_$i.log 2>&1 || exit 40
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 2 --wipe-passes 0 --single-passes 3 > $O/prof.log 2>&1 || exit 51
python3 tools/kstats.py $O/prof/bench_kernel_stats.csv > $O/bench_kernels.txt || exit 52
NM03_DEVICE_OVERRIDE=0 timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 4 --single-passes 10 > $O/bench2.log 2>&1 || exit 60
