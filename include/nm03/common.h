// nm03/common.h — shared macros, error types and small utilities for the NM03 MI355X engine.
//
// Everything in the engine (host codecs, golden model, HIP kernels, runtime) is compiled by
// hipcc/amdclang++ with -ffp-contract=off so that the f32 arithmetic of the CPU golden model and
// of the gfx950 kernels is bit-identical (see pixel_math.h).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__) || defined(__HIP__)
#define NM03_HD __host__ __device__ __forceinline__
#define NM03_DEVICE_COMPILE 1
#else
#define NM03_HD inline
#endif

namespace nm03 {

// Error thrown for any per-slice failure (bad DICOM, unsupported syntax, too-small image...).
// Mirrors the role of fast::Exception in the reference (main_sequential.cpp:182,190,267): it is
// caught at slice level, logged, and the slice is skipped.
class SliceError : public std::runtime_error {
 public:
  explicit SliceError(const std::string& m) : std::runtime_error(m) {}
};

// Error for device/runtime failures (HIP, RCCL). Fatal for the batch that raised it.
class DeviceError : public std::runtime_error {
 public:
  explicit DeviceError(const std::string& m) : std::runtime_error(m) {}
};

inline constexpr int kMaxSeeds = 256;

// Pixel storage types understood by the import stage (DICOM BitsAllocated/PixelRepresentation).
enum PixelType : uint8_t { kU16 = 0, kI16 = 1, kU8 = 2 };

inline size_t pixel_bytes(PixelType t) { return t == kU8 ? 1 : 2; }

inline uint32_t div_up(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

}  // namespace nm03
