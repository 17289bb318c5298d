#!/bin/bash
# (gpurun) Config 5 evidence + 8-rank rehearsal. gpurun_out/r3c5/:
#  * 256³ volume (one 256-slice patient): nm03_bench --config volume JSON and its rocprofv3 kernel
#    table (no host sync inside srg_volume: the sweeps are one cooperative launch);
#  * the same volume through img_processing_parallel --mode 3d, single rank and --split-volume over
#    2 / 4 ranks sharing the GPU (host comm), --json each, output trees compared byte for byte;
#  * bench.py --gpus 8 on one GPU (NM03_DEVICE_OVERRIDE=0): 8 per-rank device records, comm nranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3c5; mkdir -p $O
B=build/bin; T=/tmp/r3c5
$B/nm03_synth --data-root $T/vol/ --patients 1 --min-slices 256 --max-slices 256 --threads 16 > /dev/null || exit 101
timeout -k 10 120 $B/nm03_bench --config volume --data-root $T/vol/ --steps 10 --warmup 2 > $O/c5_gpu.json || exit 111
for n in 1 2 4; do
  extra=""; [ $n -gt 1 ] && extra="--split-volume"
  NM03_DEVICE_OVERRIDE=0 timeout -k 10 180 $B/img_processing_parallel --mode 3d --gpus $n $extra --data-root $T/vol/ \
    --out $T/out$n --json $O/c5_cli_$n.json > $O/c5_cli_$n.log 2>&1 || exit $((120+n))
done
diff -r $T/out1 $T/out2 > $O/diff_1_2.txt && diff -r $T/out1 $T/out4 > $O/diff_1_4.txt || exit 130
echo "split-volume outputs identical" > $O/diff_ok.txt
NM03_DEVICE_OVERRIDE=0 timeout -k 10 400 python bench.py --gpus 8 --steps 10 --warmup 2 --single-passes 3 > $O/bench8.log 2>&1 || exit 140
# Last (nothing on the GPU after it): under rocprofv3 this process has segfaulted in a library
# destructor at exit (__cxa_finalize) after writing its results; the stats files are complete then.
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c5 \
  -- $B/nm03_bench --config volume --data-root $T/vol/ --steps 10 --warmup 2 > $O/c5_prof.json 2>&1
echo "profiled run exit $?" > $O/c5_prof_status.txt
python3 tools/kstats.py $O/prof/c5_kernel_stats.csv > $O/c5_kernels.txt || exit 113
rm -rf $T
