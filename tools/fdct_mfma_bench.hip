// Exact islow FDCT on the matrix cores vs on the vector ALUs ("build and measure an
// integer-MFMA islow FDCT"). Both kernels compute libjpeg's islow forward DCT of 8×8 u8 blocks
// (jpeg_common.h, level shift folded: fdct(x − 128) = fdct(x) with DC − 8192), bit-exact to the host
// golden, one block per lane, 64 blocks per wave (the JPEG encoder's layout).
//
//  valu   : fdct_islow_pass1 + fdct_islow_pass2 in registers (the encoder today).
//  mfma   : pass 1 (rows) on v_mfma_i32_32x32x32_i8. The row transform before its rounding shift is
//           an exact integer matrix C1 (|entries| ≤ 11363); C1 = C0 + 256·C1hi splits it into two
//           signed int8 digits, x − 128 is int8, so two MFMAs per 16 blocks give the exact raw sums
//           (D0 + (D1 << 8)). K = 4 rows × 8 pixels against a block-diagonal B, N = 4 rows × 8
//           outputs, M = (block, row quad): 8 MFMAs per wave. Pixels go to LDS once (int8) and come
//           back in the A layout (one ds_read_b128 per group); the descaled row outputs go to LDS as
//           int16 and come back per lane for the VALU column pass (pass 2 inputs reach ±4096, two int8
//           digits each, which would make an MFMA pass 2 cost four products plus the recombination).
// Each wave repeats its 64 blocks `reps` times (input perturbed per repetition) so the timing is
// compute, not HBM. Output: μs per 64 blocks per wave-repetition for both, and the mismatch count.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude tools/fdct_mfma_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nm03/jpeg_common.h"

using namespace nm03::jpeg;

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

struct Coefs {
  int8_t c[2][8][8];  // [digit][u][c]: pass-1 raw row transform = Σ_c (c0 + 256 c1)[u][c] · x_c
};

// Host: the raw (pre-rounding) pass-1 outputs of a unit vector → the integer matrix.
static void pass1_raw(const int32_t* x, int64_t* out) {
  int64_t t0 = x[0] + x[7], t7 = x[0] - x[7], t1 = x[1] + x[6], t6 = x[1] - x[6];
  int64_t t2 = x[2] + x[5], t5 = x[2] - x[5], t3 = x[3] + x[4], t4 = x[3] - x[4];
  int64_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  out[0] = (t10 + t11) * 4;
  out[4] = (t10 - t11) * 4;
  int64_t z1 = (t12 + t13) * kF0_541;
  out[2] = z1 + t13 * kF0_765;
  out[6] = z1 - t12 * kF1_847;
  z1 = t4 + t7;
  int64_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7, z5 = (z3 + z4) * kF1_175;
  t4 *= kF0_298;
  t5 *= kF2_053;
  t6 *= kF3_072;
  t7 *= kF1_501;
  z1 *= -kF0_899;
  z2 *= -kF2_562;
  z3 = z3 * -kF1_961 + z5;
  z4 = z4 * -kF0_390 + z5;
  out[7] = t4 + z1 + z3;
  out[5] = t5 + z2 + z4;
  out[3] = t6 + z2 + z3;
  out[1] = t7 + z1 + z4;
}

__device__ __forceinline__ uint32_t perturb(uint32_t v, int rep) { return v ^ (uint32_t)(rep * 0x01010101u & 0x07070707u); }

__global__ __launch_bounds__(256) void fdct_valu(const uint8_t* __restrict__ in, int32_t* __restrict__ out, int reps,
                                                 uint32_t* sink) {
  const size_t blk = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(in + blk * 64);
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = src[i];
  uint32_t acc = 0;
  int32_t d[64];
  for (int rep = 0; rep < reps; ++rep) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t v = perturb(w[i], rep);
#pragma unroll
      for (int b = 0; b < 4; ++b) d[4 * i + b] = (int32_t)((v >> (8 * b)) & 0xFF);
    }
    fdct_islow(d);
    d[0] -= 8192;
#pragma unroll
    for (int i = 0; i < 64; ++i) acc += (uint32_t)d[i] * (uint32_t)(i + 1);
  }
  int32_t* o = out + blk * 64;
#pragma unroll
  for (int i = 0; i < 64; ++i) o[i] = d[i];
  if (acc == 0x7FFFFFFFu) sink[0] = acc;
}

__global__ __launch_bounds__(256) void fdct_mfma(const uint8_t* __restrict__ in, int32_t* __restrict__ out, int reps,
                                                 Coefs cf, uint32_t* sink) {
  __shared__ __attribute__((aligned(16))) int8_t spx[4][64 * 64];    // per wave: [block][row][col] (x − 128)
  __shared__ __attribute__((aligned(16))) int16_t sy[4][64 * 64];    // per wave: [block][row][u]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t blk = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(in + blk * 64);
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = src[i];
  // B fragments (constant per lane): lane l holds B[k = 16h + j][n = l & 31], j = 0..15.
  const int n = lane & 31, h = lane >> 5, u = n & 7, r4o = n >> 3;
  v4i bfr[2];
#pragma unroll
  for (int dg = 0; dg < 2; ++dg) {
    int32_t packed[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r4 = 2 * h + (j >> 3), c = j & 7;
      const int v = r4 == r4o ? (int)cf.c[dg][u][c] : 0;
      packed[j >> 2] |= (v & 0xFF) << (8 * (j & 3));
    }
    bfr[dg] = v4i{packed[0], packed[1], packed[2], packed[3]};
  }
  // descale of the row outputs: u ∈ {0, 4} are exact (× 4), the others (x + 2^10) >> 11
  const int add = (u == 0 || u == 4) ? 0 : 1024, shf = (u == 0 || u == 4) ? 0 : 11;
  int8_t* px = spx[wv];
  int16_t* y = sy[wv];
  uint32_t acc = 0;
  int32_t d[64];
  for (int rep = 0; rep < reps; ++rep) {
    // this lane's block → LDS as int8 (x − 128): 64 bytes
    uint32_t* dst = reinterpret_cast<uint32_t*>(px + lane * 64);
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[i] = perturb(w[i], rep) ^ 0x80808080u;  // x − 128 as int8
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // A: lane l holds A[m = l & 31][k = 16h + j]: block 16g + m/2, rows 4(m&1) + 2h, +1
      const int m = lane & 31;
      const v4i a = *reinterpret_cast<const v4i*>(px + (16 * g + (m >> 1)) * 64 + (4 * (m & 1) + 2 * h) * 8);
      v16i d0 = {0}, d1 = {0};
      d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bfr[0], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bfr[1], d1, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        // D: lane holds col n, row m = (i & 3) + 8 (i >> 2) + 4 h → block 16g + m/2, row 4(m&1) + r4o
        const int mm = (i & 3) + 8 * (i >> 2) + 4 * h;
        const int32_t raw = d0[i] + (d1[i] << 8);
        y[(16 * g + (mm >> 1)) * 64 + (4 * (mm & 1) + r4o) * 8 + u] = (int16_t)((raw + add) >> shf);
      }
    }
    __syncthreads();
    const int16_t* mine = y + lane * 64;
#pragma unroll
    for (int i = 0; i < 64; ++i) d[i] = mine[i];
    fdct_islow_pass2(d);
#pragma unroll
    for (int i = 0; i < 64; ++i) acc += (uint32_t)d[i] * (uint32_t)(i + 1);
    __syncthreads();
  }
  int32_t* o = out + blk * 64;
#pragma unroll
  for (int i = 0; i < 64; ++i) o[i] = d[i];
  if (acc == 0x7FFFFFFFu) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int nblocks = argc > 1 ? std::atoi(argv[1]) : (1 << 20);  // multiple of 256
  const int reps = argc > 2 ? std::atoi(argv[2]) : 16;
  Coefs cf;
  for (int c = 0; c < 8; ++c) {
    int32_t e[8] = {0};
    e[c] = 1;
    int64_t raw[8];
    pass1_raw(e, raw);
    for (int u = 0; u < 8; ++u) {
      const int64_t v = raw[u];
      const int64_t lo = ((v + 128) & 255) - 128, hi = (v - lo) / 256;
      if (hi < -128 || hi > 127) return 2;
      cf.c[0][u][c] = (int8_t)lo;
      cf.c[1][u][c] = (int8_t)hi;
    }
  }
  std::vector<uint8_t> h_in((size_t)nblocks * 64);
  uint32_t s = 12345;
  for (auto& v : h_in) {
    s = s * 1664525u + 1013904223u;
    v = (uint8_t)(s >> 24);
  }
  for (int b = 0; b < 64; ++b) std::memset(&h_in[(size_t)b * 64], b & 1 ? 255 : 0, 64);  // extreme blocks too
  uint8_t* d_in;
  int32_t *d_a, *d_b;
  uint32_t* sink;
  CK(hipMalloc(&d_in, h_in.size()));
  CK(hipMalloc(&d_a, (size_t)nblocks * 64 * 4));
  CK(hipMalloc(&d_b, (size_t)nblocks * 64 * 4));
  CK(hipMalloc(&sink, 4));
  CK(hipMemcpy(d_in, h_in.data(), h_in.size(), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int t = 0; t < 5; ++t) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    return best;
  };
  const float tv = time([&] { fdct_valu<<<nblocks / 256, 256>>>(d_in, d_a, reps, sink); });
  const float tm = time([&] { fdct_mfma<<<nblocks / 256, 256>>>(d_in, d_b, reps, cf, sink); });
  std::vector<int32_t> a((size_t)nblocks * 64), b((size_t)nblocks * 64);
  CK(hipMemcpy(a.data(), d_a, a.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), d_b, b.size() * 4, hipMemcpyDeviceToHost));
  // host golden of the last repetition for the first 4096 blocks
  size_t bad_v = 0, bad_m = 0;
  for (int blk = 0; blk < 4096 && blk < nblocks; ++blk) {
    int32_t d[64];
    for (int i = 0; i < 64; ++i) {
      uint32_t wv;
      std::memcpy(&wv, &h_in[(size_t)blk * 64 + (i & ~3)], 4);
      wv ^= (uint32_t)((reps - 1) * 0x01010101u & 0x07070707u);
      d[i] = (int32_t)((wv >> (8 * (i & 3))) & 0xFF);
    }
    fdct_islow(d);
    d[0] -= 8192;
    for (int i = 0; i < 64; ++i) {
      bad_v += a[(size_t)blk * 64 + i] != d[i];
      bad_m += b[(size_t)blk * 64 + i] != d[i];
    }
  }
  const double waves = nblocks / 64.0 * reps;
  std::printf("blocks %d reps %d\n", nblocks, reps);
  std::printf("valu: %.3f ms  %.4f us per 64 blocks per wave-rep (x %d SIMDs)  mismatches %zu\n", tv,
              tv * 1e3 / waves * 1024, nblocks, bad_v);
  std::printf("mfma: %.3f ms  %.4f us per 64 blocks per wave-rep (x %d SIMDs)  mismatches %zu\n", tm,
              tm * 1e3 / waves * 1024, nblocks, bad_m);
  std::printf("mfma / valu time = %.3f\n", tm / tv);
  return (bad_v || bad_m) ? 3 : 0;
}
