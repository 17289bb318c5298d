#!/bin/bash
# 12-bit packer A/B on the box's Zen 5 host (gpurun): AVX-512 VBMI (default where available) vs AVX2
# (NM03_PACK_AVX512=0). Single-threaded host path costs (tools/host_path_bench.sh) both ways, the
# engine GPU tests that cover packing, then 4 interleaved headline pairs. gpurun_out/pack512/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/pack512; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pack12 or engine" > $O/pytest.log 2>&1 || exit 31
timeout -k 10 120 bash tools/host_path_bench.sh 7 > $O/hpb_avx512.txt 2>&1 || exit 32
NM03_PACK_AVX512=0 timeout -k 10 120 bash tools/host_path_bench.sh 7 > $O/hpb_avx2.txt 2>&1 || exit 33
for i in 1 2 3 4; do
  for v in 1 0; do
    NM03_PACK_AVX512=$v timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-secondary --wipe-passes 0 > $O/b${v}_$i.log 2>&1 || exit 34
    echo "avx512=$v round $i $(grep -o '"value": [0-9.]*' $O/b${v}_$i.log | head -1) $(grep -o '"load_cpu_s": [0-9.]*' $O/b${v}_$i.log | head -1) $(grep -o '"usage": [0-9.]*' $O/b${v}_$i.log | head -1)" >> $O/summary.txt
  done
done
