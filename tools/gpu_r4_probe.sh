#!/bin/bash
# (gpurun) Round 4, first call — probes and the starting point. gpurun_out/r4a/:
#  * create_probe: tmpfs create / O_TMPFILE / rewrite / unlink / rename-to-trash cost per slice
#    (two 12 KB files) at 1/4/8/16 private workers, shared vs directory-affine vs per-worker dirs;
#  * bar_probe: can the CPU write VRAM (large BAR), at what rate;
#  * bench.py (20 steps) incl. the new config.cli_wall (10 exact CLI invocations);
#  * config 5 under rocprofv3 with the crash handler installed (last: it has exited 139 before).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r4a; mkdir -p $O
B=build/bin
timeout -k 5 300 $B/create_probe /dev/shm/nm03_cp 1,4,8,16 930 3 > $O/create_probe.txt 2>&1 || { rm -rf /dev/shm/nm03_cp; exit 10; }
timeout -k 5 60 $B/bar_probe > $O/bar_probe.txt 2>&1 || exit 20
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 30
T=/tmp/r4vol
$B/nm03_synth --data-root $T/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 40
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 \
  -- $B/nm03_bench --config volume --data-root $T/ --steps 10 --warmup 2 > $O/c5_prof.json 2> $O/c5_prof.err
echo "profiled run exit $?" > $O/c5_prof_status.txt
rm -rf $T
