#!/bin/bash
# (gpurun) tools/diag_norm.py on the current build and on an older build staged as a package copy
# in abpre/ (git-ignored). gpurun_out/diag_norm/.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/diag_norm; mkdir -p $O
timeout -k 10 120 python3 tools/diag_norm.py > $O/current.txt 2>&1 || exit 10
NM03_DIAG_ROOT=$PWD/abpre LD_LIBRARY_PATH=$PWD/abpre/nm03_capstone_project_amd/lib:/opt/rocm/lib \
  timeout -k 10 120 python3 tools/diag_norm.py > $O/abpre.txt 2>&1 || exit 12
