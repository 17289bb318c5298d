#!/bin/bash
# (gpurun) End-of-session tree check: smoke, GPU tests, 3 default bench runs, a 2000-step sustained run.
# gpurun_out/r3f4/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3f6; mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || exit 30
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 31
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py > $O/bench_$i.log 2>&1 || exit 40
done
timeout -k 10 300 python3 bench.py --steps 2000 --warmup 10 --wipe-passes 0 --single-passes 0 > $O/long.log 2>&1 || exit 41
