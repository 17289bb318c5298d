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

void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw DeviceError(std::string("launch of ") + what + " failed: " + hipGetErrorString(e));
  if (sync_launches()) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) throw DeviceError(std::string(what) + " failed: " + hipGetErrorString(e));
  }
}

void jpeg_divisors(int quality, int32_t* out) {
  jpeg::Tables t = jpeg::make_tables(quality);
  for (int i = 0; i < 64; ++i) out[i] = t.div_luma[i];
}

}  // namespace nm03::gpu
