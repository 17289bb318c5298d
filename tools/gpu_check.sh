#!/bin/bash
# GPU validation run used with gpurun: torch sanity → pytest -m gpu → 1-GPU bench. Logs in gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "start $(date)" > gpurun_out/progress.txt
timeout -k 10 300 python -c "import torch; print(torch.__version__, torch.cuda.is_available(), torch.cuda.get_device_name(0))" > gpurun_out/torch.log 2>&1 || exit 11
echo "torch ok $(date)" >> gpurun_out/progress.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc $(date)" >> gpurun_out/progress.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
echo "bench rc=$? $(date)" >> gpurun_out/progress.txt
