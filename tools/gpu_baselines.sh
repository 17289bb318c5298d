#!/bin/bash
# BASELINE.md measurements (gpurun): every BASELINE.json config on the MI355X engine and on the
# reference-equivalent CPU model (golden ops, 16 threads, batch 25, serial export), plus wall
# clock of repeated unmodified CLI invocations. JSON lines → gpurun_out/baselines/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/baselines
mkdir -p $O
B=build/bin
T=/tmp/nm03_bl
echo "synth $(date)" > $O/progress.txt
$B/nm03_synth --data-root $T/cohort/ --threads 16 > /dev/null || exit 101
$B/nm03_synth --data-root $T/patient/ --patients 1 --threads 16 > /dev/null || exit 102
$B/nm03_synth --data-root $T/vol/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 103
$B/nm03_synth --data-root $T/stress/ --stress 10000 --stress-dim 512 --threads 16 > /dev/null || exit 104
$B/nm03_synth --data-root $T/stress_cpu/ --stress 400 --stress-dim 512 --threads 16 > /dev/null || exit 105
echo "gpu $(date)" >> $O/progress.txt
# config 1: test_pipeline single slice
timeout -k 10 120 $B/nm03_bench --config single --data-root $T/cohort/ --steps 50 --warmup 5 > $O/c1_gpu.json || exit 111
timeout -k 10 120 $B/nm03_bench --config single-cpu --data-root $T/cohort/ --steps 10 --warmup 2 > $O/c1_cpu.json || exit 112
# config 2: one patient
timeout -k 10 120 $B/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/bl_o2 --steps 50 --warmup 5 --batch-size 25 --streams 3 > $O/c2_gpu.json || exit 121
# config 2 as written ("per-slice streams"): one slice per launch chain, 4 slots = 4 HIP streams (the
# box's GPU_MAX_HW_QUEUES), so up to 4 slices are in flight, each on its own stream
timeout -k 10 120 $B/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/bl_o2s --steps 50 --warmup 5 --batch-size 1 --streams 4 > $O/c2_gpu_per_slice_streams.json || exit 123
timeout -k 10 120 $B/nm03_bench --config cpu-reference --data-root $T/patient/ --out /tmp/bl_o2c --steps 3 --warmup 1 --batch-size 25 --threads 16 > $O/c2_cpu.json || exit 122
# config 3: full cohort (bench.py is the headline; native driver for the same work)
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --data-root $T/cohort > $O/c3_gpu_bench.json || exit 131
timeout -k 10 120 $B/nm03_bench --config cohort --data-root $T/cohort/ --out /tmp/bl_o3 --steps 20 --warmup 3 --batch-size 96 --streams 4 > $O/c3_gpu_native.json || exit 132
timeout -k 10 300 $B/nm03_bench --config cpu-reference --data-root $T/cohort/ --out /tmp/bl_o3c --steps 2 --warmup 1 --batch-size 25 --threads 16 > $O/c3_cpu.json || exit 133
echo "c3 done $(date)" >> $O/progress.txt
# config 4: 512² × 10k, 5×5 median (CPU reference on a 400-slice subset of the same shape)
timeout -k 10 300 $B/nm03_bench --config cohort --data-root $T/stress/ --out /tmp/bl_o4 --steps 3 --warmup 1 --batch-size 64 --streams 3 --median-window 5 --max-dim 512 > $O/c4_gpu.json || exit 141
timeout -k 10 300 $B/nm03_bench --config cpu-reference --data-root $T/stress_cpu/ --out /tmp/bl_o4c --steps 1 --warmup 0 --batch-size 25 --threads 16 --median-window 5 > $O/c4_cpu.json || exit 142
echo "c4 done $(date)" >> $O/progress.txt
# config 5: 256³ volume
timeout -k 10 120 $B/nm03_bench --config volume --data-root $T/vol/ --steps 10 --warmup 2 > $O/c5_gpu.json || exit 151
timeout -k 10 300 $B/nm03_bench --config volume-cpu --data-root $T/vol/ --steps 2 --warmup 1 --threads 16 > $O/c5_cpu.json || exit 152
echo "c5 done $(date)" >> $O/progress.txt
# CLI wall clock: 10 timed invocations of each unmodified CLI on the full cohort, exact (wait4)
timeout -k 10 600 python3 tools/cli_wall.py "$B" "$T/cohort/" 10 > $O/cli_wall.jsonl || exit 161
echo "done $(date)" >> $O/progress.txt
