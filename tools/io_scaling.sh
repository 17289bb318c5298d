#!/bin/bash
# File I/O scaling across processes (gpurun, CPU only): P concurrent io_probe processes × T threads
# writing separate trees, on the overlay /tmp and on tmpfs /dev/shm. Approximates N bench ranks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=/tmp/iop
build/bin/nm03_synth --data-root $D/ --threads 16 > /dev/null || exit 1
for fs in /tmp /dev/shm; do
  for P in 1 2 4; do
    T=$((16 / P)); [ $T -gt 4 ] && T=4
    pids=()
    for p in $(seq $P); do
      timeout -k 5 120 build/bin/nm03_ioprobe $D/ $fs/iosc_$p $T > gpurun_out/iosc_${fs//\//_}_${P}_$p.txt 2>&1 &
      pids+=($!)
    done
    for pid in "${pids[@]}"; do wait $pid; done
    rm -rf $fs/iosc_*
  done
done
