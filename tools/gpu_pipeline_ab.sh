set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || exit 31
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_pipe_$i.log 2>&1 || exit 32
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-pipeline > gpurun_out/bench_nopipe_$i.log 2>&1 || exit 33
done
timeout -k 10 300 python bench.py --steps 100 --warmup 5 > gpurun_out/bench_pipe_100.log 2>&1 || exit 34
