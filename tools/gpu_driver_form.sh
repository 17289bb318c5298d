set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/drv
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/run_$i.log 2>&1 || exit 41
done
