// HIP error helpers and small host utilities for the kernel launchers.
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <string>

#include "nm03/jpeg.h"
#include "nm03/kernels.h"

namespace nm03::gpu {

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

bool sync_launches() {
  static const bool on = [] {
    const char* s = std::getenv("NM03_SYNC_LAUNCHES");
    return s && *s && *s != '0';
  }();
  return on;
}

int profile_variant(const char* kernel) {
  // NM03_PROFILE_VARIANT="jpeg=12,median=1": truncated kernel variants for time splits (output
  // invalid; profile them with rocprofv3 --kernel-trace --stats, e.g. through tools/ab_bench.sh). Parsed once.
  static const std::string spec = [] {
    const char* s = std::getenv("NM03_PROFILE_VARIANT");
    return std::string(s ? s : "");
  }();
  const std::string key = std::string(kernel) + "=";
  for (size_t p = 0; p < spec.size();) {
    size_t e = spec.find(',', p);
    if (e == std::string::npos) e = spec.size();
    if (spec.compare(p, key.size(), key) == 0) return std::atoi(spec.c_str() + p + key.size());
    p = e + 1;
  }
  return 0;
}

void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw DeviceError(std::string("launch of ") + what + " failed: " + hipGetErrorString(e));
  if (sync_launches()) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) throw DeviceError(std::string(what) + " failed: " + hipGetErrorString(e));
  }
}

void warm_copy_path(hipStream_t stream) {
  // Shader copies (HSA_ENABLE_SDMA=0, the CLI's --copy-engine for short jobs) run on the compute
  // queues with the blit kernels the runtime loaded with the first stream: nothing to bring up.
  if (const char* e = std::getenv("HSA_ENABLE_SDMA"); e && std::string(e) == "0") return;
  // Large enough for the copy engine (SDMA) path the engine's uploads take: a 4 KiB copy is done
  // another way and left the first batch's upload paying ≈ 7.5 ms (profiles/r5/cold/).
  constexpr size_t kBytes = size_t(4) << 20;
  void* h = nullptr;
  void* d = nullptr;
  check_hip(hipHostMalloc(&h, kBytes, hipHostMallocDefault), "hipHostMalloc (copy warm-up)");
  try {
    check_hip(hipMalloc(&d, kBytes), "hipMalloc (copy warm-up)");
    check_hip(hipMemcpyAsync(d, h, kBytes, hipMemcpyHostToDevice, stream), "H2D (copy warm-up)");
    check_hip(hipStreamSynchronize(stream), "copy warm-up");
  } catch (...) {
    if (d) (void)hipFree(d);
    (void)hipHostFree(h);
    throw;
  }
  (void)hipFree(d);
  (void)hipHostFree(h);
}

void jpeg_divisors(int quality, int32_t* out) {
  jpeg::Tables t = jpeg::make_tables(quality);
  for (int i = 0; i < 64; ++i) out[i] = t.div_luma[i];
}

}  // namespace nm03::gpu
