set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
O=gpurun_out/c4_r2.txt; : > $O
B=build/bin; T=/tmp/nm03_c4
$B/nm03_synth --data-root $T/stress/ --stress 10000 --stress-dim 512 --threads 16 > /dev/null || exit 101
for r in 1 2; do
  echo "streams3 $(timeout -k 10 200 $B/nm03_bench --config cohort --data-root $T/stress/ --out /tmp/c4o --steps 3 --warmup 1 --batch-size 64 --streams 3 --median-window 5 --max-dim 512)" >> $O || exit 102
done
