#!/bin/bash
# Round 3 host-path investigation on the GPU box (gpurun): host memory bandwidth probe, the
# host-only engine (bench.py --host-only) over pool sizes and pinning policies, and the full bench
# with NM03_PIN=set vs core, interleaved. Logs in gpurun_out/host_r3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/host_r3
mkdir -p $O
P=$O/progress.txt
echo "start $(date)" > $P
{ nproc; cat /sys/fs/cgroup/cpu.max; grep -E "Cpus_allowed_list" /proc/self/status; lscpu | grep -E "Model name|NUMA node|L3"; } > $O/host.txt 2>&1
timeout -k 10 200 build/bin/stream_probe 16 512 > $O/stream_probe.txt 2>&1 || exit 21
echo "probe ok $(date)" >> $P
D=/dev/shm/nm03_host_r3_data
hb() {  # host-only bench: <tag> <threads> <pin>
  NM03_PIN=$3 timeout -k 10 120 python bench.py --host-only --steps 100 --warmup 5 --threads $2 --wipe-passes 0 \
    --single-passes 0 --keep-data --data-root $D >> $O/host_$1.log 2>&1
}
for rep in 1 2; do
  for t in 4 8 12 16; do
    for pin in set core; do
      hb "t${t}_${pin}" $t $pin || exit 22
    done
  done
  echo "host rep $rep ok $(date)" >> $P
done
for rep in 1 2 3; do
  for pin in set core; do
    NM03_PIN=$pin timeout -k 10 200 python bench.py --keep-data --data-root $D --wipe-passes 0 >> $O/gpu_${pin}.log 2>&1 || exit 23
  done
  echo "gpu rep $rep ok $(date)" >> $P
done
rm -rf $D ${D}-node*
echo "done $(date)" >> $P
