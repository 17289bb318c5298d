#!/bin/bash
# Host path vs CPU placement (gpurun): the rank's CPU set restricted with taskset to 2 / 4 / 8 CCDs
# (CPU 0-15 = CCDs 0-1, one thread per core), 8 cores + SMT siblings, or the default (node 0).
# host-only engine and the full bench, interleaved. Logs in gpurun_out/host_ccd/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/host_ccd
mkdir -p $O
P=$O/progress.txt
echo "start $(date)" > $P
D=/dev/shm/nm03_host_ccd_data
run() {  # <tag> <cpus|all> <extra bench args...>
  local tag=$1 cpus=$2
  shift 2
  if [ "$cpus" = all ]; then
    timeout -k 10 200 python bench.py --keep-data --data-root $D --wipe-passes 0 --single-passes 0 "$@" >> $O/$tag.log 2>&1
  else
    timeout -k 10 200 taskset -c $cpus python bench.py --keep-data --data-root $D --wipe-passes 0 --single-passes 0 "$@" >> $O/$tag.log 2>&1
  fi
}
for rep in 1 2; do
  for v in "all:all" "c2:0-15" "c4:0-31" "c8:0-63" "c1smt:0-7,128-135"; do
    tag=${v%%:*}; cpus=${v#*:}
    run host_$tag $cpus --host-only --steps 100 --warmup 5 || exit 21
  done
  echo "host rep $rep ok $(date)" >> $P
done
for rep in 1 2 3; do
  for v in "all:all" "c2:0-15" "c4:0-31"; do
    tag=${v%%:*}; cpus=${v#*:}
    run gpu_$tag $cpus || exit 22
  done
  echo "gpu rep $rep ok $(date)" >> $P
done
rm -rf $D ${D}-node*
echo "done $(date)" >> $P
