#!/bin/bash
# A/B (gpurun): bench input cohort as one copy per NUMA node (--numa-data auto) vs one shared copy
# (off), interleaved; host NUMA layout; a 2-rank gloo rehearsal of the auto path. gpurun_out/numa/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/numa
{ ls /sys/devices/system/node; for d in /sys/devices/system/node/node*; do echo "$d $(cat $d/cpulist)"; done;
  python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; } > gpurun_out/numa/layout.txt 2>&1
{ cat /sys/fs/cgroup/cpuset.cpus.effective /sys/fs/cgroup/cpuset.mems.effective; grep -i cpus_allowed_list /proc/self/status;
  python3 -c "
import os
a = sorted(os.sched_getaffinity(0)); print('aff', a[:4], '...', a[-4:])
for s in ([0], [1], list(range(64)), list(range(64, 128)), list(range(0, 64)) + list(range(128, 192))):
    try:
        os.sched_setaffinity(0, s); print('ok', s[:3], len(s))
    except OSError as e:
        print('fail', s[:3], len(s), e)
"; } >> gpurun_out/numa/layout.txt 2>&1
timeout -k 10 120 python -c "
import torch, nm03_capstone_project_amd as m
n = m.native(); print('gpu0 node', n.numa_device_node(0))
from nm03_capstone_project_amd.parallel.numa_data import numa_nodes
print('nodes with cpus', numa_nodes(n.numa_node_cpus))" >> gpurun_out/numa/layout.txt 2>&1 || exit 20
for i in 1 2 3; do
  for v in auto off; do
    timeout -k 10 300 python bench.py --steps 100 --warmup 5 --numa-data $v > gpurun_out/numa/bench_${v}_$i.log 2>&1 || exit 21
  done
done
NM03_DIST_BACKEND=gloo NM03_DEVICE_OVERRIDE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --threads 8 \
  > gpurun_out/numa/multirank_2.log 2>&1 || exit 22
ls /dev/shm > gpurun_out/numa/shm_after.txt
