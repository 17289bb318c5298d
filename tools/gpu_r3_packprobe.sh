#!/bin/bash
# (gpurun; host only) tools/pack_probe.cpp on the box, 3 runs. gpurun_out/r3pp/.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3pp; mkdir -p $O
lscpu > $O/lscpu.txt 2>&1
for i in 1 2 3; do timeout -k 5 60 build/bin/pack_probe >> $O/probe.txt 2>&1 || exit 10; done
