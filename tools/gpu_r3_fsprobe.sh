#!/bin/bash
# (gpurun; host only) Filesystem facts of the box and the per-file read cost of a 131 KB file from
# tmpfs vs the root overlay's page cache (large folios?), 16 threads (io_contention mode 4).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3fs; mkdir -p $O
{ uname -a; df -T / /tmp /dev/shm "$GRAFT_REPO_ROOT"; mount | grep -E " / | /tmp | /dev/shm " ;
  cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled;
  ls /sys/kernel/mm/transparent_hugepage/; cat /sys/kernel/mm/transparent_hugepage/hugepages-*/shmem_enabled 2>/dev/null | head -3;
  ls -d /sys/kernel/mm/transparent_hugepage/hugepages-* ; findmnt -o TARGET,FSTYPE,OPTIONS / /tmp /dev/shm; } > $O/facts.txt 2>&1
for round in 1 2; do
  for root in /dev/shm/nm03_ioc /tmp/nm03_ioc; do
    rm -rf $root; mkdir -p $root
    echo "== $root" >> $O/io.txt
    timeout -k 5 120 build/bin/io_contention $root 16 8000 3 4 >> $O/io.txt 2>&1
    rm -rf $root
  done
done
exit 0
