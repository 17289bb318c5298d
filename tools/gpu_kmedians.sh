#!/bin/bash
# (gpurun) Per-kernel medians of full-batch dispatches for nm03_bench --config cohort under variant flag
# sets, ROUNDS (default 2) interleaved rounds (tools/kernel_medians.py). Usage: gpu_kmedians.sh <name> ["args1;args2;..."]
# ("-" = default flags; leading NAME=VAL words go to the environment, e.g. "LD_LIBRARY_PATH=ab_old" runs
# an older libnm03.so built there; BENCH=<path> runs another nm03_bench binary, e.g. one built from an
# older commit together with its library). The JPEG GPU tests run first (every encoder instance vs the golden model).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
B=build/bin
O=gpurun_out/${1:-kmed}
mkdir -p "$O"
IFS=';' read -r -a VARS <<< "${2:--;--render-filter nearest}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "jpeg or render" > $O/pytest_jpeg.log 2>&1 || exit 2
$B/nm03_synth --data-root /tmp/nm03_bench_data/ --threads 16 > /dev/null || exit 3
for r in $(seq ${ROUNDS:-2}); do
  i=0
  for v in "${VARS[@]}"; do
    a=(); envs=()
    if [ "$v" != "-" ]; then
      for w in $v; do if [[ ${#a[@]} -eq 0 && "$w" == *=* ]]; then envs+=("$w"); else a+=("$w"); fi; done
    fi
    bin=$B/nm03_bench; e2=()
    for e in "${envs[@]}"; do if [[ "$e" == BENCH=* ]]; then bin=${e#BENCH=}; else e2+=("$e"); fi; done
    env "${e2[@]}" timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/v${i}r$r -o k -- $bin --config cohort \
      --data-root /tmp/nm03_bench_data/ --out /tmp/kmed_out --steps 3 --warmup 1 --batch-size 96 --streams 4 "${a[@]}" \
      > $O/v${i}r$r.log 2>&1 || exit 4
    echo "== variant $i ($v) round $r: $(grep -o "slices_per_s.: [0-9]*" $O/v${i}r$r.log | head -1)" >> $O/summary.txt
    python tools/kernel_medians.py $(find $O/v${i}r$r -name "*kernel_trace.csv") >> $O/summary.txt
    i=$((i + 1))
  done
done

python tools/kernel_medians.py --summary $O/summary.txt
