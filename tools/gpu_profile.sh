#!/bin/bash
# GPU profiling/baseline run (gpurun): rocprofv3 kernel stats of bench.py, the BASELINE.md
# CPU reference-equivalent run, the 3D volume config and a 512² stress config. Logs: gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress_prof.txt
echo "start $(date)" > $P
B=build/bin
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --keep-output > gpurun_out/bench2.log 2>&1 || exit 21
echo "bench ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || exit 22
echo "rocprof ok $(date)" >> $P
# the bench removes its own cohort at exit: the CPU reference and the CLIs get one of their own
$B/nm03_synth --data-root /tmp/nm03_bench_data/ --threads 16 > /dev/null || exit 20
timeout -k 10 400 $B/nm03_bench --config cpu-reference --data-root /tmp/nm03_bench_data/ --out /tmp/cpuref_out --steps 2 --warmup 1 --threads 16 --batch-size 25 > gpurun_out/cpu_reference.log 2>&1 || exit 23
echo "cpuref ok $(date)" >> $P
( time $B/img_processing_parallel --data-root /tmp/nm03_bench_data/ --out /tmp/o_par --quiet --json gpurun_out/cli_parallel.json ) > gpurun_out/cli_parallel.log 2>&1 || exit 24
( time $B/img_processing_sequential --data-root /tmp/nm03_bench_data/ --out /tmp/o_seq --quiet --json gpurun_out/cli_sequential.json ) > gpurun_out/cli_sequential.log 2>&1 || exit 25
echo "cli ok $(date)" >> $P
$B/nm03_synth --data-root /tmp/vol/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 26
timeout -k 10 300 $B/nm03_bench --config volume --data-root /tmp/vol/ --steps 3 --warmup 1 > gpurun_out/volume.log 2>&1 || exit 27
echo "volume ok $(date)" >> $P
$B/nm03_synth --data-root /tmp/stress/ --stress 2000 --stress-dim 512 --threads 16 > /dev/null || exit 28
timeout -k 10 300 $B/nm03_bench --config cohort --data-root /tmp/stress/ --median-window 5 --max-dim 512 --batch-size 32 --steps 3 --warmup 1 --out /tmp/stress_out > gpurun_out/stress.log 2>&1 || exit 29
echo "stress ok $(date)" >> $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_stress -o stress -- $B/nm03_bench --config cohort --data-root /tmp/stress/ --median-window 5 --max-dim 512 --batch-size 32 --steps 1 --warmup 0 --out /tmp/stress_out > gpurun_out/prof_stress.log 2>&1 || exit 30
echo "done $(date)" >> $P
