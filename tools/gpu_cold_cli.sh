#!/bin/bash
# (gpurun) Cold CLI anatomy: per-batch timelines of fresh img_processing_parallel runs
# (NM03_BATCH_TRACE=1), an in-process --repeat 2 (cold pass vs warm pass), and one rocprofv3
# trace of a cold run (kernels, copies, HIP API, roctx ranges).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5cold}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
D=/dev/shm/r5_data
CLI="$R/build/bin/img_processing_parallel --data-root $D/ --out /dev/shm/r5_out --quiet"
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for r in 1 2 3 4; do
  (cd /tmp && NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $CLI --json $R/$O/cli_$r.json > $R/$O/cli_$r.log 2>&1) || exit 2
done
(cd /tmp && NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $CLI --repeat 2 --json $R/$O/rep2.json > $R/$O/rep2.log 2>&1) || exit 3
(cd /tmp && NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $CLI --batch-size 96 --streams 4 --json $R/$O/b96.json > $R/$O/b96.log 2>&1) || exit 4
cd /tmp || exit 5
NM03_ROCTX=1 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --hip-runtime-trace \
  --output-format csv -d $R/$O/trace -o cli -- $R/build/bin/img_processing_parallel --data-root $D/ \
  --out /dev/shm/r5_out --quiet --json $R/$O/traced.json > $R/$O/traced.log 2>&1 || exit 6
rm -rf $D /dev/shm/r5_out
echo done
