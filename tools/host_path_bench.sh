#!/bin/bash
# Build + run tools/host_path_bench.cpp (single-threaded per-step host costs) on a tmpfs cohort.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/bin
/opt/rocm/llvm/bin/clang++ -O2 -std=c++17 -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ tools/host_path_bench.cpp \
  -Lnm03_capstone_project_amd/lib -lnm03 -Wl,-rpath,$PWD/nm03_capstone_project_amd/lib -Wl,-rpath,/opt/rocm/lib \
  -o build/bin/host_path_bench
D=/dev/shm/hpb_data_$$; O=/dev/shm/hpb_out_$$
python -c "import nm03_capstone_project_amd as m; m.native().synth_cohort('$D/', threads=8)"
build/bin/host_path_bench $D/ $O ${1:-5}
rm -rf $D $O
