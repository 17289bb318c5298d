#!/bin/bash
# L3-domain (CCD) affine loads/exports (NM03_PIN=l3) vs the floating pool (set): host-only engine
# and the full bench, interleaved. Logs in gpurun_out/pin_l3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/pin_l3
mkdir -p $O
P=$O/progress.txt
echo "start $(date)" > $P
D=/dev/shm/nm03_pin_l3_data
for rep in 1 2 3; do
  for pin in set l3; do
    NM03_PIN=$pin timeout -k 10 200 python bench.py --host-only --steps 100 --warmup 5 --keep-data --data-root $D \
      --wipe-passes 0 --single-passes 0 >> $O/host_$pin.log 2>&1 || exit 21
  done
  echo "host rep $rep ok $(date)" >> $P
done
for rep in 1 2 3 4; do
  for pin in set l3; do
    NM03_PIN=$pin timeout -k 10 200 python bench.py --keep-data --data-root $D --wipe-passes 0 --single-passes 0 \
      >> $O/gpu_$pin.log 2>&1 || exit 22
  done
  echo "gpu rep $rep ok $(date)" >> $P
done
rm -rf $D ${D}-node*
echo "done $(date)" >> $P
