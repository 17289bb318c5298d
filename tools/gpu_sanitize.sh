#!/bin/bash
# Host-side sanitizers around the GPU engine (gpurun): the ASan and TSan builds of nm03_bench
# (host code instrumented, device code untouched) drive full cohort runs on the MI355X —
# slot workers, prioritised pool, pinned buffers, file writers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D=/tmp/nm03_san_gpu
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 300 build-address/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/san_o1 \
  --steps 3 --warmup 1 > gpurun_out/san_address.log 2>&1; echo "address rc=$? reports=$(grep -c 'ERROR: AddressSanitizer' gpurun_out/san_address.log)" >> gpurun_out/san.txt
TSAN_OPTIONS="halt_on_error=0 suppressions=$PWD/tools/tsan.supp" timeout -k 10 600 build-thread/bin/nm03_bench --config cohort --data-root $D/ --out /tmp/san_o2 \
  --steps 2 --warmup 1 > gpurun_out/san_thread.log 2>&1; echo "thread rc=$? reports=$(grep -c 'WARNING: ThreadSanitizer' gpurun_out/san_thread.log)" >> gpurun_out/san.txt
