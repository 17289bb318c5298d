#!/bin/bash
# (gpurun) Is the JPEG encoder instruction-fetch bound? List the PMC counters, then per-kernel
# instruction-cache and wait counters (each group in its own pass, only names the box lists), batch
# 96, one stream, both FLAT settings. gpurun_out/r3ic/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r3ic; mkdir -p $O
timeout -k 10 -s KILL 90 rocprofv3 -L > $O/avail.txt 2>&1 || timeout -k 10 -s KILL 90 rocprofv3 --list-avail > $O/avail.txt 2>&1 || exit 20
D=/tmp/r3ic_data
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 41
i=0
for grp in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  ok=""
  for c in $grp; do grep -qw "$c" $O/avail.txt && ok="$ok $c"; done
  echo "pass $i: $ok" >> $O/passes.txt
  [ -z "$ok" ] && continue
  for f in 1 0; do
    NM03_JPEG_FLAT=$f timeout -k 10 -s KILL 120 rocprofv3 --pmc $ok --output-format csv -d $O/f$f/p$i -o run \
      -- build/bin/nm03_bench --config cohort --data-root $D/ --steps 1 --warmup 1 --batch-size 96 --streams 1 \
      > $O/f$f.p$i.log 2>&1 || exit $((70+i))
  done
done
for f in 1 0; do
  echo "== flat $f" >> $O/summary.txt
  python3 tools/pmc_summary.py $O/f$f | grep -A24 jpeg_fused >> $O/summary.txt
done
rm -rf $D
