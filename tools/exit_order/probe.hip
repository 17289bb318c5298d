// See probe_dep.cpp. Build (tools/exit_order/build.sh): hipcc --offload-arch=gfx950.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void tiny(int* p) {
  if (threadIdx.x == 0) p[0] = 1;
}
static void h_main(int st, void*) { std::fprintf(stderr, "[exit-order] handler registered at the start of main (status %d)\n", st); }
static void h_hip(int st, void*) { std::fprintf(stderr, "[exit-order] handler registered after HIP init (status %d)\n", st); }

int main() {
  on_exit(h_main, nullptr);
  int* p = nullptr;
  if (hipMalloc(&p, 64) != hipSuccess) return 2;
  tiny<<<1, 64>>>(p);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  on_exit(h_hip, nullptr);
  std::fprintf(stderr, "[exit-order] main returns\n");
  return 0;
}
