#!/bin/bash
# (gpurun) Shader upload of small batches (NM03_SHADER_UPLOAD_KB=4096) vs SDMA (0): engine GPU tests
# with it on, then single-pass latency (bench.py) and config 2 (one patient, batch 25, 3 streams,
# native nm03_bench) interleaved. gpurun_out/r3u/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3u; mkdir -p $O
NM03_SHADER_UPLOAD_KB=4096 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "engine or cli_sequential_equals or cli_parallel_multirank" > $O/pytest.log 2>&1 || exit 31
T=/tmp/r3u; build/bin/nm03_synth --data-root $T/patient/ --patients 1 --threads 16 > /dev/null || exit 41
for rep in 1 2 3; do
  for kb in 0 4096; do
    NM03_SHADER_UPLOAD_KB=$kb timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --wipe-passes 0 --single-passes 20 > $O/sp_${kb}_$rep.log 2>&1 || exit 42
    python3 - $O/sp_${kb}_$rep.log kb$kb >> $O/summary.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        st = json.loads(l)['config']['strong']
        print(f"{sys.argv[2]:7s} sp={st['single_pass_ms']}/{st['single_pass_min_ms']} sp8={st['single_pass_shard8_ms']}/{st['single_pass_shard8_min_ms']} uncapped8={st['single_pass_shard8_uncapped_ms']}")
PY
    NM03_SHADER_UPLOAD_KB=$kb timeout -k 10 120 build/bin/nm03_bench --config cohort --data-root $T/patient/ --out /tmp/r3u_o2 --steps 50 --warmup 5 --batch-size 25 --streams 3 > $O/c2_${kb}_$rep.json 2>&1 || exit 43
    echo "kb$kb c2 $(cat $O/c2_${kb}_$rep.json | tail -1)" >> $O/summary.txt
  done
done
rm -rf $T /tmp/r3u_o2
