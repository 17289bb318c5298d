#!/bin/bash
# Host topology probe (gpurun): NUMA nodes, CPU lists, GPU PCI NUMA node, cgroup CPU share.
mkdir -p gpurun_out
{
echo "== nodes"; for n in /sys/devices/system/node/node*; do echo "$n $(cat $n/cpulist) mem=$(grep MemTotal $n/meminfo | awk '{print $4}')"; done
echo "== cgroup"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null
echo "== affinity"; python3 -c "import os; print(len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:8])"
echo "== gpus"; for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d $(cat $d/numa_node) $(cat $d/vendor 2>/dev/null) $(basename $(readlink -f $d))"; done
echo "== kfd"; for d in /sys/class/kfd/kfd/topology/nodes/*; do echo "$d $(grep -E 'simd_count|location_id|domain' $d/properties | tr '\n' ' ')"; done
echo "== tmp"; df -h /tmp; mount | grep -E " /tmp | / " | head -3
} > gpurun_out/numa.txt 2>&1
