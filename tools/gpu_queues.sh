#!/bin/bash
# (gpurun) HIP stream / HW-queue creation cost at start-up (tools/queue_probe.cpp), the cold CLI
# with fewer HW queues, hipInit by NUMA node, and the comgr pre-load (PART=numa|queues|comgr|all).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5queues}
mkdir -p "$O"
R=$GRAFT_REPO_ROOT
if [ "${PART:-all}" = comgr ]; then
  # When does the HIP runtime map libamd_comgr, and does loading it on a second thread while
  # hipInit runs shorten the start-up? Interleaved, 3 streams per run.
  for r in $(seq 1 ${RUNS:-10}); do
    echo "plain $(GPU_MAX_HW_QUEUES=2 timeout -k 5 60 build/bin/queue_probe 3 1)" >> $O/comgr_probe.txt || exit 8
    echo "pre   $(GPU_MAX_HW_QUEUES=2 PROBE_PREDLOPEN=1 timeout -k 5 60 build/bin/queue_probe 3 1)" >> $O/comgr_probe.txt || exit 9
  done
  echo done; exit 0
fi
if [ "${PART:-all}" = numa ] || [ "${PART:-all}" = all ]; then
  # Is the cold hipInit bimodal by the NUMA node the initialising thread runs on? queue_probe
  # (hipInit + first allocation + 1 stream) pinned to each node's CPUs (taskset, before any HIP call)
  # and unpinned, interleaved; plus the GPU's own node from sysfs.
  for c in /sys/class/drm/card*/device/numa_node; do echo "$c $(cat $c)"; done > $O/gpu_nodes.txt 2>&1
  N0=$(cat /sys/devices/system/node/node0/cpulist)
  N1=$(cat /sys/devices/system/node/node1/cpulist 2>/dev/null || echo "$N0")
  echo "GPU_MAX_HW_QUEUES in the environment: '${GPU_MAX_HW_QUEUES:-unset}'" > $O/numa_probe.txt
  for r in $(seq 1 ${RUNS:-8}); do
    echo "node0 $(timeout -k 5 60 taskset -c $N0 build/bin/queue_probe 1 1)" >> $O/numa_probe.txt || exit 5
    echo "node1 $(timeout -k 5 60 taskset -c $N1 build/bin/queue_probe 1 1)" >> $O/numa_probe.txt || exit 6
    echo "free  $(timeout -k 5 60 build/bin/queue_probe 1 1)" >> $O/numa_probe.txt || exit 7
  done
  [ "${PART:-all}" = numa ] && { echo done; exit 0; }
fi
for rep in 1 2; do
  for q in 1 2 4; do
    for cfg in "5 1" "5 5" "2 1"; do
      GPU_MAX_HW_QUEUES=$q timeout -k 5 60 build/bin/queue_probe $cfg >> $O/probe.txt 2>&1 || exit 2
    done
  done
done
D=/dev/shm/r5q_data
timeout -k 5 60 build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 3
for rep in 1 2 3; do
  for q in 1 2 4; do
    (cd /tmp && GPU_MAX_HW_QUEUES=$q NM03_BATCH_TRACE=1 NM03_LOG=info timeout -k 10 60 $R/build/bin/img_processing_parallel \
      --data-root $D/ --out /dev/shm/r5q_out --quiet --json $R/$O/cli_q${q}_$rep.json > $R/$O/cli_q${q}_$rep.log 2>&1) || exit 4
  done
done
rm -rf $D /dev/shm/r5q_out
echo done
